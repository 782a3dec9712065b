"""Per-kernel launch statistics of a rocprofv3 --kernel-trace run, from its SQLite output
(rocprofv3 on this image writes results.db; the `kernels` view has one row per dispatch).
Writes the same columns as rocprofv3's kernel_stats.csv.
usage: python tools/kernel_stats.py RUN.db [out.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, (end - start) from kernels").fetchall()
    con.close()
    per = {}
    for name, ns in rows:
        per.setdefault(name, []).append(ns)
    total = sum(sum(v) for v in per.values()) or 1
    out = []
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        out.append({"Name": name, "Calls": len(v), "TotalDurationNs": sum(v), "AverageNs": sum(v) / len(v),
                    "Percentage": 100.0 * sum(v) / total, "MinNs": min(v), "MaxNs": max(v)})
    return out


if __name__ == "__main__":
    res = stats(sys.argv[1])
    f = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.DictWriter(f, fieldnames=list(res[0].keys()))
    w.writeheader()
    w.writerows(res)
