#!/usr/bin/env python3
"""Idle-time breakdown of a kernel trace (tools/gpu.sh trace / prof):

    python tools/timeline.py gpurun_out/TAG [--tail 0.7]

Over the last `tail` fraction of the traced span (the timed frames of a
long bench run): each stream's kernel count, busy time (union of its
kernels), the time any kernel runs, and each stream's idle gaps grouped by
the kernel pair around them -- where a stream waits on the host, an event
or another stream."""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_json import open_db, short  # noqa: E402


def union(iv):
    iv = sorted(iv)
    if not iv:
        return 0
    tot, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ce - cs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tagdir")
    ap.add_argument("--tail", type=float, default=0.7)
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    c = open_db(os.path.join(a.tagdir, "trace"))
    rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    t0, t1 = min(r[1] for r in rows), max(r[2] for r in rows)
    lo = t1 - a.tail * (t1 - t0)
    rows = [r for r in rows if r[1] >= lo]
    span = (t1 - lo) / 1e6
    by = collections.defaultdict(list)
    for n, s, e, st in rows:
        by[st].append((s, e, short(n)))
    print(f"window {span:.1f} ms (last {a.tail:.0%} of the trace); any kernel running "
          f"{union([(s, e) for _, s, e, _ in rows]) / 1e6:.1f} ms")
    for st, v in sorted(by.items(), key=lambda x: -len(x[1])):
        busy = union([(s, e) for s, e, _ in v]) / 1e6
        top = collections.Counter(x[2] for x in v).most_common(2)
        gaps = collections.Counter()
        for x, y in zip(v, v[1:]):
            g = y[0] - x[1]
            if g > 0:
                gaps[(x[2][:34], y[2][:34])] += g
        print(f"stream {st}: {len(v)} kernels, busy {busy:.1f} ms, idle {span - busy:.1f} ms "
              f"({', '.join(n[:30] for n, _ in top)})")
        for (p, q), g in gaps.most_common(a.top):
            print(f"    {g / 1e6:7.2f} ms  {p}  ->  {q}")


if __name__ == "__main__":
    main()
