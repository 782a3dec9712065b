"""Per-window timeline of the window-parallel walk on the C3 batches (bench.py c3_streams):
runs a few walked calls with PSX_DEBUG_WALK_TRACE on, reads the last call's timestamps
(include/psx_debug.h psx_debug_walk_trace) and prints, per message, when each window's
ticket was taken, its exit map was ready, its predecessor's state was seen and its own
state published — so the chain's per-hop cost and the speculative phase can be told apart.
Usage: python tools/walk_trace.py [--calls 5]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=5)
    args = ap.parse_args()
    import torch
    import bench
    import parameter_server_amd as psa
    from parameter_server_amd import _abi
    L = _abi.load()
    L.psx_debug_set_variant(11, 1)
    streams, nupd = bench.c3_streams()
    B = len(streams)
    bgs = list(range(100, 100 + B))
    srv = psa.Server(0, 1, bgs)
    srv.CreateTable(3, psa.TableInfo(row_kind=psa.ROW_SORTED_MAP, dtype=psa.I32, row_capacity=1024,
                                     oplog_dense_serialized=False, max_rows=100_000, max_entries=1024))
    dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
    torch.cuda.synchronize()
    for v in range(args.calls):
        srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(dev, bgs)])
    srv.sync()
    buf = np.zeros(10 * 4096, np.uint64)
    items = L.psx_debug_walk_trace(srv.handle, buf.ctypes.data_as(ctypes.c_void_p), 4096)
    assert items > 0, items
    raw = buf[: 10 * items].reshape(items, 10)
    xdbg = raw[:, 6].copy()
    tr = np.concatenate([raw[:, :6], raw[:, 7:10]], axis=1).astype(np.int64)
    t0 = tr[tr[:, 0] > 0, 0].min()
    us = (tr - t0) / 100.0   # 100 MHz ticks -> us
    out = {"items": int(items), "messages": B, "windows_per_message": int(items // B), "per_message": []}
    for b in range(B):
        rows = [us[j * B + b] for j in range(items // B) if tr[j * B + b, 0] > 0]
        if not rows:
            continue
        r = np.array(rows)
        hops = np.diff(r[:, 4])
        out["per_message"].append({
            "message": b, "windows": len(rows),
            "ticket_us": [round(x, 2) for x in r[:, 0]],
            "spec_done_us": [round(x, 2) for x in r[:, 2]],
            "seen_us": [round(x, 2) for x in r[:, 3]],
            "published_us": [round(x, 2) for x in r[:, 4]],
            "expanded_us": [round(x, 2) for x in r[:, 5]],
            "composed": [f"{int(xdbg[j * B + b]) & 0xFF:02x}:{int(xdbg[j * B + b]) >> 32:x}"
                         for j in range(items // B) if tr[j * B + b, 0] > 0],
            "load_us_mean": round(float((r[:, 1] - r[:, 0]).mean()), 2),
            "spec_us_mean": round(float((r[:, 2] - r[:, 1]).mean()), 2),
            "spec_n16_us_mean": round(float((r[:, 6] - r[:, 1]).mean()), 2),
            "spec_jump_us_mean": round(float((r[:, 7] - r[:, 6]).mean()), 2),
            "spec_exits_us_mean": round(float((r[:, 8] - r[:, 7]).mean()), 2),
            "spec_compose_us_mean": round(float((r[:, 2] - r[:, 8]).mean()), 2),
            "resolve_us_mean": round(float((r[:, 4] - r[:, 3]).mean()), 2),
            "hop_us_mean": round(float(hops.mean()), 2) if hops.size else None,
            "expand_us_mean": round(float((r[:, 5] - r[:, 4]).mean()), 2),
        })
    out["end_us"] = round(float(us[tr[:, 5] > 0, 5].max()), 2)
    print(json.dumps(out, indent=1))
    srv.close()


if __name__ == "__main__":
    main()
