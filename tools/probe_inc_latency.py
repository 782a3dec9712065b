"""Per-Inc latency of the sorted-map apply (SortedVectorMapStore::Inc,
sorted_vector_map_store.hpp:305-337) on MI355X, for the C3 cost model.

One row, one wave: the row's image is first filled to n entries, then one call of 16
messages x 1 record x 64 columns is applied to it — every column an existing key
("found": FindIndex + add in place; the steady state of C3, where the same columns recur
every step) or a new key ("insert": FindIndex + LinearSearchAndMove + the shift).  The
ordered_apply launch time (HIP events, timing mode 2) / Incs is the latency of one Inc in a
dependent chain at image size n, on the kernel the product picks for that size (<= 256
entries: the 256-entry register image, else the 1,024-entry one).  ("insert": 4 records
of 64 new keys, n -> n + 256.)

Usage: python tools/probe_inc_latency.py [--out profiles/r02/c3_inc_latency.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch
    import parameter_server_amd as psa
    from parameter_server_amd import wire
    K = 1024
    def one_call(n, nmsg, mode, rep):
        """ns of the ordered_apply launch of one call: nmsg records x 64 columns on row 0,
        whose image holds n entries (found/found_small: existing keys; insert: new keys)."""
        rng = np.random.RandomState(1000 * rep + n + 7 * nmsg)
        bgs = list(range(1, nmsg + 1))
        srv = psa.Server(0, 1, bgs + [99])
        srv.CreateTable(3, psa.TableInfo(row_kind=psa.ROW_SORTED_MAP, dtype=psa.I32, row_capacity=K,
                                         oplog_dense_serialized=False, max_rows=64, max_entries=K))
        perm = rng.permutation(K).astype(np.int32)
        have, fresh = np.sort(perm[:n]), perm[n:]
        if n:
            fill = wire.sparse_stream_np(3, 4, [(0, have, rng.randint(1, 100, size=n).astype(np.int32))])
            srv.ApplyOpLogUpdateVersion(fill.tobytes(), fill.size, 99, 0)
        msgs = []
        for b in range(nmsg):
            if mode != "insert":
                cols = np.sort(rng.choice(have, size=min(64, n), replace=False)).astype(np.int32)
            else:
                cols = np.sort(fresh[64 * b:64 * (b + 1)]).astype(np.int32)
            msgs.append(wire.sparse_stream_np(3, 4, [(0, cols, np.ones(cols.size, np.int32))]))
        dev = [torch.from_numpy(m).cuda() for m in msgs]
        torch.cuda.synchronize()
        srv.timing(2)
        srv.timing_reset()
        srv.apply_device([(d.data_ptr(), d.numel(), bg, 0) for d, bg in zip(dev, bgs)])
        srv.sync()
        ms, _ = srv.timing_read("ordered_apply")
        incs = sum(int(np.frombuffer(m[24:28].tobytes(), "<i4")[0]) for m in msgs)
        srv.close()
        return ms * 1e6, incs

    res = {"found": {}, "found_small": {}, "insert": {}, "fixed_ns_small": {}}
    for mode in ("found", "insert"):
        # found: 16 x 64 Incs (the call can add 1,024 entries: the 1,024-entry image);
        # insert: 4 x 64 new keys, n -> n + 256
        nmsg = {"found": 16, "insert": 4}[mode]
        for n in {"found": (32, 64, 128, 192, 256, 384, 512, 768, 960), "insert": (0, 128, 256, 512, 768)}[mode]:
            t = [one_call(n, nmsg, mode, rep) for rep in range(args.reps)]
            res[mode][n] = round(float(np.median([a / b for a, b in t])), 1)
            print(mode, n, res[mode][n], "ns/Inc", flush=True)
    # found_small: the 256-entry image (n + the call's Incs <= 256): one call of 64 Incs and
    # one of 128-192, the per-Inc latency from the difference (the launch's fixed cost cancels)
    for n in (32, 64, 96, 128):
        k2 = min(3, (256 - n) // 64)
        t1 = np.median([one_call(n, 1, "found", rep)[0] for rep in range(args.reps)])
        t2 = np.median([one_call(n, k2, "found", rep)[0] for rep in range(args.reps)])
        res["found_small"][n] = round(float((t2 - t1) / (64 * (k2 - 1))), 1)
        res["fixed_ns_small"][n] = round(float(t1 - 64 * res["found_small"][n]), 1)
        print("found_small", n, res["found_small"][n], "ns/Inc, fixed", res["fixed_ns_small"][n], "ns", flush=True)
    out = {"what": "ns per SortedVectorMapStore::Inc in one wave's dependent chain (one row, one wave; median of "
                   "reps; ordered_apply launch time / Incs). found: 16 records x 64 existing keys (add in place) on "
                   "an image of n entries, the 1,024-entry register image; found_small: the 256-entry image, from "
                   "calls of 64 and 128-192 existing-key Incs (fixed_ns_small: the launch's fixed part). insert: 4 records x 64 "
                   "new keys, the image growing n -> n + 256.",
           "found_ns": res["found"], "found_small_ns": res["found_small"], "insert_ns": res["insert"],
           "fixed_ns_small": res["fixed_ns_small"]}
    print(json.dumps(out))
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
