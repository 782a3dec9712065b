"""Summarise the rocprofv3 --pmc pass of the C3 bench (tools/gpu_run.sh pmcc3) into the
DRAM-side bytes per C3 step that bench.py reports beside C3's algorithmic bytes.

Per kernel: the mean of TCC_EA0_RDREQ_128B x 128 + TCC_EA0_RDREQ_64B x 64 read bytes and
TCC_EA0_WRREQ_64B x 64 + (TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B) x 32 write bytes per dispatch
(the request sizes MI355X_MICROARCH.md's HBM section prescribes), times its dispatches; the
sum over psx kernels divided by the apply calls (walk_head dispatches, one per walked C3 step;
finish_call's when the calls were not walked — a folded finish has none).
These are L2 -> fabric requests: Infinity-Cache hits are counted (the guide), so the figure
is the memory-side traffic the step asks for, an upper bound on HBM bytes.

usage: python tools/pmc_c3.py ROOT OUT.json"""
import collections
import glob
import json
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import c3_kernel_signature  # noqa: E402


def main(root, out):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for f in glob.glob(os.path.join(root, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        for k, c, v, d in con.execute("select name, counter_name, counter_value, dispatch_id from pmc_events"):
            per[k][c][(f, d)] = per[k][c].get((f, d), 0.0) + float(v)
        con.close()
    kernels, calls, fin, total_r, total_w = {}, 0, 0, 0.0, 0.0
    for name, cs in per.items():
        if "psx" not in name[:120]:
            continue
        need = ("TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum")
        if any(c not in cs for c in need):
            continue
        disp = len(cs[need[0]])
        rd = sum(cs[need[0]].values()) * 128 + sum(cs[need[1]].values()) * 64
        wr = sum(cs[need[3]].values()) * 64 + (sum(cs[need[2]].values()) - sum(cs[need[3]].values())) * 32
        short = name.split("(")[0][:100]
        kernels[short] = {"dispatches": disp, "read_bytes": rd, "write_bytes": wr}
        total_r += rd
        total_w += wr
        if "walk_head" in name:
            calls += disp
        elif "finish_call" in name:
            fin += disp
    calls = calls or fin   # one walk_head per walked call; finish_call when the calls were not walked
    if not calls:
        raise SystemExit("no walk_head or finish_call dispatches: not a C3 bench profile")
    res = {"kernel_signature": c3_kernel_signature(), "calls": calls,
           "read_bytes_per_step": total_r / calls, "write_bytes_per_step": total_w / calls,
           "bytes_per_step": (total_r + total_w) / calls, "kernels": kernels,
           "what": "L2->fabric request bytes of every psx kernel, per C3 step (apply call)"}
    open(out, "w").write(json.dumps(res, indent=1))
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
