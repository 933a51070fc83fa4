#!/usr/bin/env python3
"""Per-kernel SQ counters per launch from a rocprofv3 --pmc database, as the
JSON bench.py reads for roofline.valu.
usage: pmc_json.py <run_results.db> <out.json> --source <name> --git <rev>"""
import argparse
import json
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("out")
ap.add_argument("--source", required=True)
ap.add_argument("--git", required=True)
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = c.execute("select kernel_name, counter_name, avg(value), avg(duration) "
                 "from counters_collection group by kernel_name, counter_name").fetchall()
c.close()
ker = {}
for k, n, v, d in rows:
    ker.setdefault(k, {"avg_us_profiled": round(d / 1e3, 3)})[n] = v
with open(a.out, "w") as f:
    json.dump({"source": a.source, "git": a.git, "unit": "per launch", "kernels": ker}, f, indent=1)
