"""C2's process-to-process spread: one process, one message layout, the
dense_apply launch time over R rounds (HIP events, psx timing mode 2).

  --layout 0  one torch allocation per message (what bench.py does)
  --layout 1  the 8 messages and the table's initial rows carved from ONE reservation made
              first in the process, every message starting on a 2 MiB boundary

Run it in several fresh processes, each under rocprofv3 --pmc with the translation
counters (tools/gpu_run.sh spread), to see whether the slow processes are the ones whose
vector-L1 translation misses wait longer (TCP_CLIENT_UTCL1_INFLIGHT per miss: the UTCL2 /
page-walk latency the L1 sees; this image exposes no UTCL2 counter)."""
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
    ap.add_argument("--layout", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import parameter_server_amd as psa
    from parameter_server_amd import wire
    rows, cap, B = 1 << 20, 256, 8
    msg_bytes = wire.dense_stream_bytes(rows, cap, 4)
    MiB2 = 2 << 20
    slot = (msg_bytes + MiB2 - 1) // MiB2 * MiB2
    resv = None
    if args.layout == 1:
        # the reservation first, before anything else touches the allocator
        resv = torch.empty(B * slot + MiB2, dtype=torch.uint8, device="cuda")
        base = (-resv.data_ptr()) % MiB2
    g = torch.Generator(device="cuda").manual_seed(1234)
    table0 = torch.randn(rows, cap, device="cuda", generator=g) * 0.1
    streams, lists = [], []
    for b in range(B):
        perm = torch.randperm(rows, device="cuda", generator=g).to(torch.int32)
        upd = torch.randn(rows, cap, device="cuda", generator=g) * 0.01
        s = wire.dense_stream_torch(1, perm, upd)
        if resv is not None:
            dst = resv[base + b * slot: base + b * slot + msg_bytes]
            dst.copy_(s)
            s = dst
        streams.append(s)
        lists.append(perm)
        del upd
    torch.cuda.synchronize()
    bgs = [100 + b for b in range(B)]
    srv = psa.Server(device=0, server_id=1, bg_ids=bgs)
    srv.set_stream(torch.cuda.current_stream().cuda_stream)
    srv.set_pipeline(1)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows))
    srv.load_rows(1, 0, None, on_device_ptr=table0.data_ptr(), num_rows=rows)
    del table0
    ver = [0]

    def step():
        msgs = [(s.data_ptr(), s.numel(), bgs[b], ver[0]) for b, s in enumerate(streams)]
        srv.apply_indexed_rows(msgs, [r.data_ptr() for r in lists])
        ver[0] += 1

    for _ in range(3):
        step()
    srv.sync()
    per = []
    for r in range(args.rounds):
        srv.timing(2)
        srv.timing_reset()
        for _ in range(args.steps):
            step()
        srv.sync()
        ms, n = srv.timing_read("dense_apply")
        per.append(ms / max(n, 1))
    srv.close()
    print(json.dumps({"layout": args.layout, "dense_apply_ms_median": round(statistics.median(per), 4),
                      "dense_apply_ms_rounds": [round(x, 4) for x in per],
                      "msg_ptr_mod_2MiB": [s.data_ptr() % MiB2 for s in streams],
                      "msg_ptrs_GiB": [round(s.data_ptr() / 2 ** 30, 3) for s in streams],
                      "pid": os.getpid(), "t": time.time()}), flush=True)


if __name__ == "__main__":
    main()
