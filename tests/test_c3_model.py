"""The C3 latency model's insert count (bench.c3_model) against a direct simulation of the
timed steps: the bench repeats the same batches, and an Inc inserts a key exactly when the
(row, col) value before it is zero (SortedVectorMapStore::Inc, sorted_vector_map_store.hpp:
305-337; a zero value is removed by :329-334, so absent == 0)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _batches(seed, rows=40, K=12, B=5, per_batch=15):
    rng = np.random.RandomState(seed)
    out = []
    for b in range(B):
        recs = []
        for rid in rng.choice(rows, size=per_batch, replace=False):
            k = rng.randint(1, 5)
            cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
            vals = (rng.randint(1, 3, size=k) * (1 if b == 0 else rng.choice([-1, 1], size=k))).astype(np.int32)
            recs.append((int(rid), cols, vals))
        out.append(recs)
    return out, rows, K


def _simulate_inserts(batches, warmup, steps):
    value = {}
    inserts = 0
    for s in range(warmup + steps):
        for recs in batches:
            for rid, cols, vals in recs:
                for c, v in zip(cols, vals):
                    if v == 0:
                        continue
                    key = (rid, int(c))
                    before = value.get(key, 0)
                    if s >= warmup and before == 0:
                        inserts += 1
                    value[key] = before + int(v)
    return inserts / steps


def test_model_insert_count_matches_simulation():
    for seed in (1, 2, 3):
        batches, rows, K = _batches(seed)
        m = bench.c3_model(batches, rows, K, apply_ms=1.0, warmup=3, steps=7)
        if m is None:   # no latency JSON in this checkout
            return
        assert abs(m["inserts_per_step"] - round(_simulate_inserts(batches, 3, 7), 1)) < 1e-6
