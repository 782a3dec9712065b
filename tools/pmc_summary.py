"""Summarise the rocprofv3 --pmc passes of tools/gpu_pmc.sh: per kernel, the mean of each
counter over its dispatches, plus the dense_apply HBM traffic per launch that bench.py
reports as roofline.traffic.

Traffic = TCC_EA0_RDREQ_128B x 128 + TCC_EA0_RDREQ_64B x 64 read bytes
+ TCC_EA0_WRREQ_64B x 64 + (TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B) x 32 write bytes: the
request counts times their sizes, as MI355X_MICROARCH.md "HBM" prescribes for gfx950
(FETCH_SIZE tallies a 128-B request at 64 B, so it is reported only as a cross-check,
doubled).

The output carries bench.kernel_signature() of the sources it was measured on; bench.py
refuses (traffic null) a JSON whose signature differs from the tree it runs from.

usage: python tools/pmc_summary.py gpurun_out/pmc [out.json] [kernel-substring]"""
import collections
import csv
import glob
import json
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_signature  # noqa: E402


def load(root):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                d = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                c = row["Counter_Name"]
                per[k][c][d] = per[k][c].get(d, 0.0) + float(row["Counter_Value"])
    # rocprofv3 on this image writes SQLite (pmc_results.db) instead of CSV
    for f in glob.glob(os.path.join(root, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        for k, c, v, d in con.execute("select name, counter_name, counter_value, dispatch_id from pmc_events"):
            per[k][c][(f, d)] = per[k][c].get((f, d), 0.0) + float(v)
        con.close()
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in per.items()}


KERNEL_KEYS = ("dense_apply_v3_kernel<float, 8, 16, true, 2", "dense_apply_v2_kernel<float, 8, 16, true, 2")


def dense_apply_traffic(kernels, keys=KERNEL_KEYS):
    for name, c in sorted(kernels.items(), key=lambda kv: [k in kv[0] for k in keys].index(True)
                          if any(k in kv[0] for k in keys) else len(keys)):
        if not any(k in name for k in keys):
            continue
        rd128 = c.get("TCC_EA0_RDREQ_128B_sum")
        rd64 = c.get("TCC_EA0_RDREQ_64B_sum")
        wr = c.get("TCC_EA0_WRREQ_sum")
        wr64 = c.get("TCC_EA0_WRREQ_64B_sum")
        if None in (rd128, rd64, wr, wr64):
            return None, name
        read = rd128 * 128 + rd64 * 64
        write = wr64 * 64 + (wr - wr64) * 32
        return {"kernel": name, "read_bytes": read, "write_bytes": write,
                "dense_apply_hbm_bytes_per_launch": read + write, "hbm_bytes_per_launch": read + write,
                "fetch_size_x2_bytes": 2 * 1024 * c["FETCH_SIZE"] if "FETCH_SIZE" in c else None,
                "write_size_bytes": 1024 * c["WRITE_SIZE"] if "WRITE_SIZE" in c else None}, name
    return None, None


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    kernels = load(root)
    keys = (sys.argv[3],) if len(sys.argv) > 3 else KERNEL_KEYS
    traffic, name = dense_apply_traffic(kernels, keys)
    out = {"kernels": kernels, "kernel_signature": kernel_signature()}
    if traffic:
        out.update(traffic)
    text = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(json.dumps(traffic, indent=1) if traffic else f"no complete dense_apply counters ({name})")
