"""A/B of the window-parallel walk's shape (threads x window, PSX_VARIANT_WALK_SHAPE), grid
(PSX_VARIANT_WALK_CUS) and composed-map levels (PSX_VARIANT_WALK_LEVELS) on the C3 batches
(bench.py c3_streams), interleaved in one process: per config a server of its own, rounds of
`steps` timed walked calls, the step rate in M updates/s (best and median of the rounds).
Usage: python tools/walk_sweep.py [--rounds 3] [--steps 20] [--configs 0:0:4,3:4:4,...]
(config = shape:cus:levels[:call_events], call_events PSX_VARIANT_CALL_EVENTS, default 0)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = "0:0:4,0:1:0,1:1:4,1:1:0,2:2:4,2:2:0,3:4:4,3:4:0,3:5:4,4:2:4,4:2:0"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--configs", default=DEFAULT)
    args = ap.parse_args()
    import torch
    import bench
    import parameter_server_amd as psa
    from parameter_server_amd import _abi
    L = _abi.load()
    streams, nupd = bench.c3_streams()
    B = len(streams)
    bgs = list(range(100, 100 + B))
    dev = [torch.from_numpy(s).cuda() for s in streams]
    # config: shape:cus:levels[:call_events][/variant=value...] (other psx_debug.h selectors)
    cfgs = []
    for tok in args.configs.split(","):
        head, *sets = tok.split("/")
        c = tuple(int(x) for x in (head + ":0").split(":")[:4]) if head.count(":") == 2 else \
            tuple(int(x) for x in head.split(":"))
        c = c + tuple((int(k), int(v)) for k, v in (x.split("=") for x in sets))
        cfgs.append(c)
    srvs, ver = [], []
    for _ in cfgs:
        srv = psa.Server(0, 1, bgs)
        srv.set_stream(torch.cuda.current_stream().cuda_stream)
        srv.CreateTable(3, psa.TableInfo(row_kind=psa.ROW_SORTED_MAP, dtype=psa.I32, row_capacity=1024,
                                         oplog_dense_serialized=False, max_rows=100_000, max_entries=1024))
        srvs.append(srv)
        ver.append(0)
    res = {c: [] for c in cfgs}
    for r in range(args.rounds):
        for i, c in enumerate(cfgs):
            L.psx_debug_set_variant(16, c[0])
            L.psx_debug_set_variant(12, c[1])
            L.psx_debug_set_variant(15, c[2])
            L.psx_debug_set_variant(17, c[3])
            for k, v in c[4:]:
                L.psx_debug_set_variant(k, v)
            srv = srvs[i]

            def step():
                srv.apply_device([(d.data_ptr(), d.numel(), bg, ver[i]) for d, bg in zip(dev, bgs)])
                ver[i] += 1

            for _ in range(3):
                step()
            srv.sync()
            torch.cuda.synchronize()
            w0 = L.psx_debug_get_variant(8)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            srv.sync()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            walked = L.psx_debug_get_variant(8) - w0
            res[c].append((nupd * args.steps / el / 1e6, walked))
        print(f"round {r} done", file=sys.stderr, flush=True)
    out = []
    for c in cfgs:
        v = sorted(x for x, _ in res[c])
        out.append({"shape": c[0], "cus": c[1], "levels": c[2], "call_events": c[3],
                    "variants": {str(k): x for k, x in c[4:]}, "best_Mups": round(v[-1], 1),
                    "median_Mups": round(v[len(v) // 2], 1), "walked_calls": res[c][-1][1],
                    "us_per_step": round(nupd / v[len(v) // 2], 2)})
    print(json.dumps(out, indent=1))
    for s in srvs:
        s.close()


if __name__ == "__main__":
    main()
