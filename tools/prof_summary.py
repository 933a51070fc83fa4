#!/usr/bin/env python3
"""Summarise rocprofv3 output databases into a committed markdown file.

usage: prof_summary.py <prof_dir> <out.md> [--bench <bench.log>]

<prof_dir> holds trace/run_results.db (--kernel-trace --stats) and
optionally fetch/ and write/ (separate --pmc FETCH_SIZE / WRITE_SIZE passes).
Per kernel: calls, average / total duration, share of GPU time, and the HBM
bytes per launch from the PMC passes.  FETCH_SIZE is also shown doubled:
MI355X_MICROARCH.md ("HBM") measures that gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced streaming read; for other access widths the
counter is uncalibrated, so both columns are kept.
"""
import argparse
import json
import os
import sqlite3


def short(name, n=70):
    name = name.replace("rv::", "")
    return name if len(name) <= n else name[: n - 3] + "..."


def top_kernels(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage "
                     "from top_kernels order by total_duration desc").fetchall()
    c.close()
    return rows


def pmc(db):
    if not os.path.exists(db):
        return {}
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, count(*), avg(value), avg(duration) "
                     "from counters_collection group by kernel_name").fetchall()
    c.close()
    return {r[0]: (r[1], r[2], r[3]) for r in rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("out")
    ap.add_argument("--bench")
    ap.add_argument("--title", default="")
    ap.add_argument("--traffic-json", help="also write per-kernel HBM bytes per launch "
                    "(FETCH_SIZE x2 + WRITE_SIZE, bytes) for bench.py's roofline.traffic")
    a = ap.parse_args()
    tk = top_kernels(os.path.join(a.prof_dir, "trace", "run_results.db"))
    fe = pmc(os.path.join(a.prof_dir, "fetch", "run_results.db"))
    wr = pmc(os.path.join(a.prof_dir, "write", "run_results.db"))
    lines = [f"# rocprofv3 summary {a.title}".rstrip(), ""]
    if a.bench and os.path.exists(a.bench):
        with open(a.bench) as f:
            js = [ln for ln in f if ln.startswith("{")]
        if js:
            b = json.loads(js[-1])
            lines += ["Bench line of the same build (un-profiled run):", "", "```json",
                      json.dumps(b), "```", ""]
    lines += ["Kernel trace (`rocprofv3 --kernel-trace --stats`), durations in microseconds.",
              "HBM bytes per launch from separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` "
              "passes (KB as reported; FETCHx2 = the gfx950 streaming-read correction).", "",
              "| kernel | calls | avg us | total us | % | FETCH KB | FETCHx2 KB | WRITE KB |",
              "|---|---|---|---|---|---|---|---|"]
    for name, calls, tot, avg, pct in tk:
        f = fe.get(name)
        w = wr.get(name)
        fs = f"{f[1]:.1f}" if f else "-"
        f2 = f"{2 * f[1]:.1f}" if f else "-"
        ws = f"{w[1]:.1f}" if w else "-"
        lines.append(f"| `{short(name)}` | {calls} | {avg:.2f} | {tot:.1f} | "
                     f"{pct:.1f} | {fs} | {f2} | {ws} |")
    lines += ["", "Calibration (tools/ubench/pmc_cal.hip, 1 GiB streams on this pool): FETCH_SIZE "
              "reports 1/2 of the bytes read at byte, dword and dwordx4 widths alike; WRITE_SIZE "
              "reports the bytes written exactly. So HBM bytes = 2 x FETCH + WRITE."]
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    if a.traffic_json:
        import subprocess
        rev = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True,
                             text=True).stdout.strip()
        tj = {"source": os.path.basename(a.out), "git": rev, "unit": "bytes per launch",
              "kernels": {}}
        for name, calls, tot, avg, pct in tk:
            f_, w_ = fe.get(name), wr.get(name)
            if f_ and w_:
                tj["kernels"][name] = {"fetch": 2 * f_[1] * 1024, "write": w_[1] * 1024,
                                       "hbm_bytes": 2 * f_[1] * 1024 + w_[1] * 1024,
                                       "avg_us": avg}
        with open(a.traffic_json, "w") as f:
            json.dump(tj, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
