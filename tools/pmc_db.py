"""Summarise a rocprofv3 --pmc SQLite output (pmc_results.db): per psx kernel, the mean
of every collected counter per dispatch.  Usage: python tools/pmc_db.py DB [DB...]"""
import collections
import json
import re
import sqlite3
import sys


def summarise(db, prefix="psx::"):
    con = sqlite3.connect(db)
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for name, counter, value, disp in con.execute(
            "select name, counter_name, counter_value, dispatch_id from pmc_events"):
        if not name.startswith(prefix) and prefix not in name[:80]:
            continue
        short = re.sub(r"\(.*$", "", name)[:90]
        acc[short][counter].append(value)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"dispatches": max(len(v) for v in cs.values())}
            for k, cs in acc.items()}


if __name__ == "__main__":
    out = {db: summarise(db) for db in sys.argv[1:]}
    print(json.dumps(out, indent=1))
