"""Overlap of the ordered prep with the previous call's apply in a rocprofv3 kernel trace
(`rocprofv3 --kernel-trace --output-format csv`), for VERDICT r5 #2's evidence.

Usage: python tools/trace_overlap.py <kernel_trace.csv> [out.json]

For every ordered_place / ordered_fill / ordered_offsets launch it finds the
ordered_apply_reg launches running at the same time (any overlap of [start, end]) and
reports, per prep kernel name: launches, how many overlapped an apply, the overlapped
share of their time, and the average duration; plus the kernel sequence of one
pipelined call for reading by eye."""
import csv
import json
import sys
from collections import defaultdict


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName") or ""
        s = int(r.get("Start_Timestamp") or r.get("Start-Timestamp") or r.get("BeginNs") or 0)
        e = int(r.get("End_Timestamp") or r.get("End-Timestamp") or r.get("EndNs") or 0)
        rows.append((s, e, name))
    rows.sort()
    return rows


def short(name):
    for k in ("ordered_place", "ordered_fill", "ordered_offsets", "ordered_classify", "ordered_count",
              "walk_head", "walk_kernel", "dense_index", "dense_apply"):
        if k in name:
            return k
    if "ordered_apply_reg_kernel" in name:
        return "ordered_apply_reg<" + name.split("<", 1)[1].split(">", 1)[0] + ">"
    if "ordered_apply_lite" in name:
        return "ordered_apply_lite"
    return name.split("(")[0][-40:]


def main():
    rows = load(sys.argv[1])
    applies = [(s, e) for s, e, n in rows if "ordered_apply_reg_kernel" in n]
    stat = defaultdict(lambda: {"launches": 0, "overlapped_launches": 0, "ns": 0, "overlap_ns": 0})
    for s, e, n in rows:
        k = short(n)
        if k not in ("ordered_place", "ordered_fill", "ordered_offsets", "walk_kernel", "walk_head", "ordered_count"):
            continue
        d = stat[k]
        d["launches"] += 1
        d["ns"] += e - s
        ov = 0
        for a0, a1 in applies:
            if a0 < e and a1 > s:
                ov += min(e, a1) - max(s, a0)
        d["overlap_ns"] += ov
        d["overlapped_launches"] += ov > 0
    out = {k: {"launches": v["launches"], "overlapped_launches": v["overlapped_launches"],
               "avg_us": round(v["ns"] / max(v["launches"], 1) / 1e3, 2),
               "overlapped_share_of_time": round(v["overlap_ns"] / max(v["ns"], 1), 3)} for k, v in stat.items()}
    # one pipelined call's sequence: the last 14 launches of the trace, with start offsets
    tail = rows[-14:]
    t0 = tail[0][0] if tail else 0
    out["last_launches"] = [{"kernel": short(n), "start_us": round((s - t0) / 1e3, 2), "dur_us": round((e - s) / 1e3, 2)}
                            for s, e, n in tail]
    js = json.dumps(out, indent=1)
    print(js)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js + "\n")


if __name__ == "__main__":
    main()
