"""Interleaved A/B of C2 kernel selectors in one process (cdna_hip_programming.md §5.4
rule 24): the headline workload of bench.py, then R rounds; each round runs every
configuration for K steps and records the per-kernel HIP-event times.  Prints JSON with
the median ms of every kernel per configuration.
Usage: python tools/ab_c2.py --configs 0,0:1,2 [--rounds 5 --steps 5]
       (apply_variant[:rows[:store_nt[:layout]]], include/psx_debug.h; rows = 1 applies
       through psx_apply_indexed_rows with the batches' record-row lists; store_nt selects
       PSX_VARIANT_DENSE_STORE, default 1; layout 1 = the messages back to back in one
       allocation instead of one allocation each)"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="0,0:1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--cols", type=int, default=256)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--zeros", action="store_true", help="zero table and updates (data-dependence check)")
    ap.add_argument("--drift", action="store_true",
                    help="print every round's dense_apply ms with its time since the first round (one line each)")
    args = ap.parse_args()
    import torch
    import parameter_server_amd as psa
    from parameter_server_amd import wire, _abi
    L = _abi.load()
    rows, cap, B = args.rows, args.cols, args.batches
    g = torch.Generator(device="cuda").manual_seed(1234)
    table0 = torch.randn(rows, cap, device="cuda", generator=g) * 0.1
    if args.zeros:
        table0.zero_()
    streams, lists = [], []
    for b in range(B):
        perm = torch.randperm(rows, device="cuda", generator=g).to(torch.int32)
        upd = torch.randn(rows, cap, device="cuda", generator=g) * 0.01
        if args.zeros:
            upd.zero_()
        streams.append(wire.dense_stream_torch(1, perm, upd))
        lists.append(perm)
        del upd, perm
    # layout 1: the same messages back to back in one allocation (a receive buffer)
    contig = torch.empty(sum(x.numel() for x in streams), dtype=torch.uint8, device="cuda")
    cstreams, o = [], 0
    for x in streams:
        contig[o:o + x.numel()].copy_(x)
        cstreams.append(contig[o:o + x.numel()])
        o += x.numel()
    bgs = [100 + b for b in range(B)]
    srv = psa.Server(device=0, server_id=1, bg_ids=bgs)
    srv.set_stream(torch.cuda.current_stream().cuda_stream)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows))
    srv.load_rows(1, 0, None, on_device_ptr=table0.data_ptr(), num_rows=rows)
    del table0
    ver = [0]
    kernels = ("decode_streams", "dense_index", "dense_verify", "dense_apply", "finish_call")
    configs = []
    for c in args.configs.split(","):
        f = [int(x) for x in c.split(":")]
        configs.append(tuple((f + [0, 1, 0][len(f) - 1:])[:4]))
    res = {c: {k: [] for k in kernels + ("step",)} for c in configs}

    def run(c, steps):
        L.psx_debug_set_variant(1, c[0])
        L.psx_debug_set_variant(9, c[2])
        srv.timing(True)
        srv.timing_reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            msgs = [(s.data_ptr(), s.numel(), bgs[b], ver[0]) for b, s in enumerate(cstreams if c[3] else streams)]
            if c[1]:
                srv.apply_indexed_rows(msgs, [r.data_ptr() for r in lists])
            else:
                srv.apply_device(msgs)
            ver[0] += 1
        srv.sync()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out = {k: srv.timing_read(k) for k in kernels}
        srv.timing(False)
        return out, el / steps * 1e3

    for c in configs:   # warm-up of every configuration
        run(c, 2)
    t_start = time.perf_counter()
    for r in range(args.rounds):
        for c in configs:
            kt, step_ms = run(c, args.steps)
            if args.drift:
                ms, n = kt["dense_apply"]
                print(json.dumps({"round": r, "t_s": round(time.perf_counter() - t_start, 3), "config": c,
                                  "dense_apply": round(ms / max(n, 1), 4), "step": round(step_ms, 4)}), flush=True)
            for k in kernels:
                ms, n = kt[k]
                res[c][k].append(ms / max(n, 1))
            res[c]["step"].append(step_ms)
    out = {f"apply{c[0]}" + ("_rows" if c[1] else "") + f"_rowpolicy{c[2]}" + ("_contig" if c[3] else ""):
           {k: round(statistics.median(v), 4) for k, v in res[c].items()} for c in configs}
    print(json.dumps(out, indent=1))
    srv.close()


if __name__ == "__main__":
    main()
