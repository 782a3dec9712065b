"""The C3 call's kernel timeline from a rocprofv3 --kernel-trace database: per walked call
(a call starts at its walk_head dispatch), each kernel's duration and the idle gap before
it, averaged over the calls after the first `skip`; the call's span (walk_head start to the
next call's walk_head start) against the sum of its kernels' durations shows how much of a
step is launch gaps rather than kernel time.
usage: python tools/c3_timeline.py RUN.db [--skip 5] > timeline.json"""
import argparse
import json
import re
import sqlite3


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name.replace("psx::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--skip", type=int, default=5)
    args = ap.parse_args()
    con = sqlite3.connect(args.db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    con.close()
    starts = [i for i, r in enumerate(rows) if "walk_head" in r[0]]
    calls = []
    for a, b in zip(starts, starts[1:]):
        seq = rows[a:b]
        span = rows[b][1] - seq[0][1]
        ks = []
        prev_end = None
        for name, s, e in seq:
            ks.append((short(name), (e - s) / 1e3, (s - prev_end) / 1e3 if prev_end is not None else 0.0))
            prev_end = e
        calls.append((span / 1e3, ks))
    calls = calls[args.skip:]
    if not calls:
        print(json.dumps({"error": "no walked calls", "kernels": len(rows)}))
        return
    # the most common kernel sequence
    sig = {}
    for span, ks in calls:
        sig.setdefault(tuple(k[0] for k in ks), []).append((span, ks))
    seq, group = max(sig.items(), key=lambda kv: len(kv[1]))
    n = len(group)
    out = {"calls": len(calls), "calls_with_this_sequence": n,
           "span_us_mean": round(sum(s for s, _ in group) / n, 2),
           "kernel_us_sum_mean": round(sum(sum(k[1] for k in ks) for _, ks in group) / n, 2),
           "sequence": []}
    for i, name in enumerate(seq):
        out["sequence"].append({"kernel": name,
                                "us_mean": round(sum(ks[i][1] for _, ks in group) / n, 2),
                                "gap_before_us_mean": round(sum(ks[i][2] for _, ks in group) / n, 2)})
    out["gap_us_sum_mean"] = round(out["span_us_mean"] - out["kernel_us_sum_mean"], 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
