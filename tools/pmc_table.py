#!/usr/bin/env python3
"""Per-kernel average of every counter in rocprofv3 --pmc databases.
usage: pmc_table.py <db> [<db> ...]"""
import sqlite3
import sys
from collections import defaultdict

rows = defaultdict(dict)
dur = {}
for db in sys.argv[1:]:
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    cn = "counter_name" if "counter_name" in cols else None
    q = (f"select kernel_name, {cn}, avg(value), avg(duration) from counters_collection "
         f"group by kernel_name, {cn}")
    for k, n, v, d in c.execute(q):
        rows[k][n] = v
        dur[k] = d
    c.close()
for k in sorted(rows, key=lambda k: -dur[k])[:10]:
    print(f"{k[:60]}  dur_ns={dur[k]:.0f}")
    for n, v in sorted(rows[k].items()):
        print(f"    {n:24s} {v:16.0f}")
