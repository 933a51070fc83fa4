"""Per-kernel summary of a rocprofv3 kernel trace (the SQLite results.db of
rocprofv3 >= 1.0 or a *_kernel_trace.csv[.gz]):

    python tools/trace_summary.py gpurun_out/TAG/trace [--frames N]

Prints total / count / mean per kernel (sorted by total), the busy sum and
the trace span; --frames divides the totals per coded frame."""
import argparse
import collections
import csv
import glob
import gzip
import os
import sqlite3


def load(d):
    dbs = glob.glob(os.path.join(d, "*.db")) + glob.glob(os.path.join(d, "*.db.gz"))
    if dbs:
        path = dbs[0]
        if path.endswith(".gz"):  # tools/gpu.sh prof compresses the results
            import tempfile
            tmp = tempfile.NamedTemporaryFile(suffix=".db", delete=False)
            with gzip.open(path, "rb") as f:
                tmp.write(f.read())
            tmp.close()
            path = tmp.name
        c = sqlite3.connect(path)
        return [(n, int(s), int(e), int(sc)) for n, s, e, sc in
                c.execute("select name, start, end, scratch_size from kernels")]
    f = glob.glob(os.path.join(d, "*kernel_trace.csv*"))[0]
    op = gzip.open if f.endswith(".gz") else open
    return [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             int(r.get("Scratch_Size", 0) or 0)) for r in csv.DictReader(op(f, "rt"))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--frames", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = load(a.dir)
    agg = collections.defaultdict(lambda: [0, 0.0, 0])
    for n, s, e, sc in rows:
        k = n.replace("(anonymous namespace)::", "").split("(")[0][:70]
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e6
        agg[k][2] = max(agg[k][2], sc)
    span = (max(r[2] for r in rows) - min(r[1] for r in rows)) / 1e6
    busy = sum(v[1] for v in agg.values())
    print(f"dispatches {len(rows)}  span {span:.2f} ms  busy-sum {busy:.2f} ms  "
          f"(per frame: {busy / a.frames:.3f} ms over {a.frames:g} frames)")
    print(f"{'ms/frame':>9} {'launches/frame':>14} {'us/launch':>9} {'scratch':>7}  kernel")
    for k, (c, ms, sc) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{ms / a.frames:9.3f} {c / a.frames:14.1f} {ms / c * 1000:9.1f} {sc:7d}  {k}")


if __name__ == "__main__":
    main()
