"""A/B the dense index/apply kernel variants on the C2 workload, interleaved in one
process (cdna_hip_programming.md §5.4 rule 24).  Prints per-variant kernel times."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch
import parameter_server_amd as psa
from parameter_server_amd import wire, _abi

p = argparse.ArgumentParser()
p.add_argument("--rows", type=int, default=1 << 20)
p.add_argument("--cols", type=int, default=256)
p.add_argument("--batches", type=int, default=8)
p.add_argument("--apply", default="0,1,2,3,4,5,6")
p.add_argument("--index", default="0,1,2")
p.add_argument("--layouts", default="0,1")
p.add_argument("--rounds", type=int, default=3)
p.add_argument("--steps", type=int, default=5)
args = p.parse_args()

rows, cap, B = args.rows, args.cols, args.batches
g = torch.Generator(device="cuda").manual_seed(1234)
table0 = torch.randn(rows, cap, device="cuda", generator=g) * 0.1
streams = []
for b in range(B):
    perm = torch.randperm(rows, device="cuda", generator=g).to(torch.int32)
    upd = torch.randn(rows, cap, device="cuda", generator=g) * 0.01
    streams.append(wire.dense_stream_torch(1, perm, upd))
    del upd
torch.cuda.synchronize()
bgs = [100 + b for b in range(B)]
srv = psa.Server(0, 1, bgs)
srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows))
srv.load_rows(1, 0, None, on_device_ptr=table0.data_ptr(), num_rows=rows)
L = _abi.load()
step_bytes = sum(s.numel() for s in streams) + 2 * rows * cap * 4
ver = [0]


def run(steps):
    for _ in range(steps):
        srv.apply_device([(s.data_ptr(), s.numel(), bgs[b], ver[0]) for b, s in enumerate(streams)])
        ver[0] += 1
    srv.sync()


run(2)
res = {}
apply_vs = [int(x) for x in args.apply.split(",")]
index_vs = [int(x) for x in args.index.split(",")]
layouts = [int(x) for x in args.layouts.split(",")]
for r in range(args.rounds):
    for lay in layouts:
        L.psx_debug_set_variant(2, lay)
        for av in apply_vs:
            L.psx_debug_set_variant(1, av)
            run(1)
            srv.timing(True)
            srv.timing_reset()
            run(args.steps)
            ms, n = srv.timing_read("dense_apply")
            srv.timing(False)
            res.setdefault(f"L{lay}_apply{av}", []).append(ms / n)
        L.psx_debug_set_variant(1, apply_vs[-1])
        for iv in index_vs:
            L.psx_debug_set_variant(0, iv)
            run(1)
            srv.timing(True)
            srv.timing_reset()
            run(args.steps)
            ms, n = srv.timing_read("dense_index")
            vms, vn = srv.timing_read("dense_verify")
            srv.timing(False)
            res.setdefault(f"L{lay}_index{iv}", []).append(ms / n)
            res.setdefault(f"L{lay}_verify", []).append(vms / vn)
out = {}
for k, v in res.items():
    v = sorted(v)
    out[k] = {"median_ms": v[len(v) // 2], "min_ms": v[0]}
    if "apply" in k:
        out[k]["GBps_algorithmic"] = round(step_bytes / (v[len(v) // 2] / 1e3) / 1e9, 1)
print(json.dumps(out, indent=1))
