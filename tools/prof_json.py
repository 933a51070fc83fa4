#!/usr/bin/env python3
"""Summarise one `tools/gpu.sh prof TAG CFG` run (kernel trace + FETCH_SIZE /
WRITE_SIZE / SQ passes of `bench.py --steps S --warmup W`) into the JSON
bench.py prices its roofline from and a markdown table:

    python tools/prof_json.py gpurun_out/TAG profiles/rNN_prof_CFG.json \
        --frames 11 --bench gpurun_out/TAG/trace.log --md profiles/rNN_prof_CFG.md

Per kernel (all launches of the run): launches and milliseconds per coded
frame, mean microseconds per launch, HBM bytes per launch (2 x FETCH_SIZE +
WRITE_SIZE: MI355X_MICROARCH.md's gfx950 correction, calibrated in
tools/ubench/pmc_cal.hip), the SQ ratios.  The F4 candidate kernels
(rdo_quad_kernel MODE 0 / 1) are also split into their round-0 launch (the
full evaluation whose candidates bench.py counts; identified as the launch
on the same queue right before the round's score_wave_kernel over every
superblock) and the MV-stack rounds' re-evaluations.  Inputs may be
gzip-compressed (tools/gpu.sh prof compresses what it returns).
"""
import argparse
import collections
import gzip
import json
import os
import shutil
import subprocess
import sqlite3
import tempfile

ROUND0_OF = ("rdo_quad_kernel<unsigned char, 0>", "rdo_quad_kernel<unsigned char, 1>",
             "rdo_quad_kernel<unsigned short, 0>", "rdo_quad_kernel<unsigned short, 1>",
             "rdo_quad_list_kernel<unsigned char, 0, 0>", "rdo_quad_list_kernel<unsigned char, 1, 1>",
             "rdo_quad_list_kernel<unsigned short, 0, 0>", "rdo_quad_list_kernel<unsigned short, 1, 1>")


def open_db(d):
    for name in ("run_results.db", "run_results.db.gz"):
        p = os.path.join(d, name)
        if os.path.exists(p):
            if p.endswith(".gz"):
                tmp = tempfile.NamedTemporaryFile(suffix=".db", delete=False)
                with gzip.open(p, "rb") as f:
                    shutil.copyfileobj(f, tmp)
                tmp.close()
                p = tmp.name
            return sqlite3.connect(p)
    return None


def short(name):
    name = name.replace("(anonymous namespace)::", "")  # rv_mvref.hip's kernels
    return name.split("(")[0].replace("void ", "").strip() or "(unnamed)"


def classify(rows):
    """rows: (dispatch, name, queue, grid, start, dur) in start order ->
    {dispatch: 'round0' | 'rounds'} for the ROUND0_OF kernels."""
    last = {}
    cls = {}
    full_score = max((g for _, n, _, g, _, _ in rows if "score_wave_kernel" in n), default=0)
    for d, n, q, g, s, du in rows:
        sn = short(n)
        if any(k in sn for k in ROUND0_OF):
            cls[d] = "rounds"
            last[(q, sn)] = d
        elif "score_wave_kernel" in n and g == full_score:
            for (qq, sn2), d2 in list(last.items()):
                if qq == q:
                    cls[d2] = "round0"
                    del last[(qq, sn2)]
    return cls


def trace(c):
    rows = c.execute("select dispatch_id, name, stream_id, grid_x, start, end - start "
                     "from kernels order by start").fetchall()
    return rows


def pmc(c, counters):
    rows = c.execute("select dispatch_id, kernel_name, queue_id, grid_size, start, duration, "
                     "counter_name, value from counters_collection order by start").fetchall()
    disp = {}
    for d, n, q, g, s, du, cn, v in rows:
        disp.setdefault(d, [d, n, q, g, s, du, {}])[6][cn] = v
    return list(disp.values())


def _union(iv):
    """Total length of the union of [start, end) intervals (sorted by start)."""
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def timed_window(tr):
    """The trace between bench.py's two rv_trace_marker_kernel launches (its
    timed region), or the whole trace without them."""
    ms = sorted(s for _, n, _, _, s, _ in tr if "rv_trace_marker_kernel" in n)
    if len(ms) < 2:
        return tr, False
    return [t for t in tr if ms[0] < t[4] < ms[-1] and "rv_trace_marker_kernel" not in t[1]], True


def occupancy(tr):
    """How busy the device and each stream were over the trace: the fraction
    of the span some kernel ran (any stream), each stream's own fraction
    (a stream near 1.0 is a serial chain of kernels: its latency, not the
    chip, bounds it), and the mean number of kernels in flight."""
    iv = sorted((s, s + du) for _, _, _, _, s, du in tr)
    t0, t1 = iv[0][0], max(e for _, e in iv)
    span = t1 - t0
    per = collections.defaultdict(list)
    for _, _, q, _, s, du in tr:
        per[q].append((s, s + du))
    streams = {}
    names = collections.defaultdict(lambda: collections.Counter())
    for _, n, q, _, s, du in tr:
        names[q][short(n)] += du
    for q, v in per.items():
        v.sort()
        streams[str(q)] = {"busy_frac": round(_union(v) / span, 4), "launches": len(v),
                           "top": [k for k, _ in names[q].most_common(3)]}
    # each stream's idle gaps between its kernels, by length (fraction of
    # the span): short ones are dispatch, long ones waits (events, host)
    edges = [5e3, 20e3, 100e3, 1e6]  # ns
    for q, v in per.items():
        hist = [0] * (len(edges) + 1)
        end = v[0][1]
        for s, e in v[1:]:
            if s > end:
                gap = s - end
                hist[sum(gap >= x for x in edges)] += gap
            end = max(end, e)
        streams[str(q)]["gaps_frac"] = dict(zip(["<5us", "5-20us", "20-100us", "0.1-1ms", ">1ms"],
                                                [round(h / span, 4) for h in hist]))
    # device-idle stretches (no kernel anywhere), charged to the stream whose
    # kernel ends them: the chain the device waited on
    idle = collections.defaultdict(int)
    owner = sorted((s, s + du, q) for _, _, q, _, s, du in tr)
    end = owner[0][1]
    for s, e, q in owner[1:]:
        if s > end:
            idle[str(q)] += s - end
        end = max(end, e)
    return {"any_kernel_frac": round(_union(iv) / span, 4),
            "mean_kernels_in_flight": round(sum(e - s for s, e in iv) / span, 3),
            "idle_ended_by": {q: round(v / span, 4) for q, v in
                              sorted(idle.items(), key=lambda x: -x[1])},
            "streams": dict(sorted(streams.items(), key=lambda x: -x[1]["busy_frac"]))}


def quantiles(v):
    v = sorted(v)
    q = lambda f: round(v[min(len(v) - 1, int(f * len(v)))], 2)
    return {"p10": q(0.1), "p50": q(0.5), "p90": q(0.9), "max": round(v[-1], 2),
            "top10pct_time_frac": round(sum(v[int(0.9 * len(v)):]) / sum(v), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tagdir")
    ap.add_argument("out")
    ap.add_argument("--frames", type=float, required=True, help="coded frames the run coded")
    ap.add_argument("--bench", help="the traced run's log (its bench line is recorded)")
    ap.add_argument("--md")
    a = ap.parse_args()
    ct = open_db(os.path.join(a.tagdir, "trace"))
    tr = trace(ct)
    cls = classify([(d, n, q, g, s, du) for d, n, q, g, s, du in tr])
    ker = collections.OrderedDict()
    for d, n, q, g, s, du in tr:
        k = ker.setdefault(short(n), {"launches": 0, "us": 0.0, "round0": [0, 0.0],
                                      "rounds": [0, 0.0], "durs": []})
        k["launches"] += 1
        k["durs"].append(du / 1e3)
        k["us"] += du / 1e3
        if d in cls:
            k[cls[d]][0] += 1
            k[cls[d]][1] += du / 1e3
    span = (max(s + du for _, _, _, _, s, du in tr) - min(s for _, _, _, _, s, _ in tr)) / 1e6
    win, marked = timed_window(tr)
    occ = occupancy(win)
    occ["window"] = "bench.py's timed region (marker kernels)" if marked else "the whole trace"
    # PMC passes: bytes per launch (all launches, and round 0 of the F4 kernels)
    traffic = collections.defaultdict(lambda: {"fetch": [0, 0.0], "write": [0, 0.0],
                                               "fetch0": [0, 0.0], "write0": [0, 0.0]})
    sq = collections.defaultdict(lambda: collections.defaultdict(float))
    for pas, cn in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        c = open_db(os.path.join(a.tagdir, pas))
        if not c:
            continue
        rows = pmc(c, [cn])
        cl = classify([(d, n, q, g, s, du) for d, n, q, g, s, du, _ in rows])
        for d, n, q, g, s, du, vals in rows:
            t = traffic[short(n)]
            kb = vals.get(cn, 0.0)
            t[pas][0] += 1
            t[pas][1] += kb
            if cl.get(d) == "round0":
                t[pas + "0"][0] += 1
                t[pas + "0"][1] += kb
    c = open_db(os.path.join(a.tagdir, "sq"))
    if c:
        for d, n, q, g, s, du, vals in pmc(c, []):
            for cn, v in vals.items():
                sq[short(n)][cn] += v
    out = {"source": os.path.basename(a.out), "tagdir": os.path.basename(a.tagdir.rstrip("/")),
           # PROF_GIT: the commit the profiled tree is (the GPU box has no .git)
           "git": os.environ.get("PROF_GIT") or subprocess.run(
               ["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip(),
           "frames": a.frames, "span_ms": round(span, 3),
           "busy_ms_per_frame": round(sum(k["us"] for k in ker.values()) / 1e3 / a.frames, 4),
           "occupancy": occ,
           "hbm_bytes_rule": "2 x FETCH_SIZE + WRITE_SIZE (KB x 1024; MI355X_MICROARCH.md, "
                             "tools/ubench/pmc_cal.hip)",
           "kernels": {}}
    if a.bench and os.path.exists(a.bench):
        with open(a.bench) as f:
            js = [ln for ln in f if ln.startswith("{")]
        if js:
            b = json.loads(js[-1])
            out["bench_line"] = {k: b.get(k) for k in ("value", "ms_per_step", "steps", "warmup")}
    for name, k in sorted(ker.items(), key=lambda x: -x[1]["us"]):
        e = {"launches_per_frame": round(k["launches"] / a.frames, 3),
             "ms_per_frame": round(k["us"] / 1e3 / a.frames, 4),
             "avg_us": round(k["us"] / k["launches"], 3)}
        if k["us"] / 1e3 / a.frames >= 0.1:  # the heavy kernels: launch duration spread (us)
            e["dur_us"] = quantiles(k["durs"])
        if k["round0"][0]:
            e["round0"] = {"launches": k["round0"][0],
                           "avg_us": round(k["round0"][1] / k["round0"][0], 3)}
            e["rounds"] = {"launches": k["rounds"][0],
                           "avg_us": round(k["rounds"][1] / max(1, k["rounds"][0]), 3),
                           "ms_per_frame": round(k["rounds"][1] / 1e3 / a.frames, 4)}
        t = traffic.get(name)
        if t and t["fetch"][0] and t["write"][0]:
            e["hbm_bytes_per_launch"] = round((2 * t["fetch"][1] / t["fetch"][0] +
                                               t["write"][1] / t["write"][0]) * 1024)
            if t["fetch0"][0] and t["write0"][0]:
                e["round0"]["hbm_bytes_per_launch"] = round(
                    (2 * t["fetch0"][1] / t["fetch0"][0] + t["write0"][1] / t["write0"][0]) * 1024)
        s = sq.get(name)
        if s and s.get("SQ_WAVE_CYCLES"):
            wc = s["SQ_WAVE_CYCLES"]
            e["sq"] = {"wait_any_over_wave_cycles": round(s.get("SQ_WAIT_ANY", 0) / wc, 4),
                       "active_inst_over_wave_cycles": round(s.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4),
                       "valu_insts_per_launch": round(s.get("SQ_INSTS_VALU", 0) / k["launches"]),
                       "waves_per_launch": round(s.get("SQ_WAVES", 0) / k["launches"], 1)}
        out["kernels"][name] = e
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    if a.md:
        lines = [f"# Kernel profile `{out['tagdir']}` (git {out['git']})", "",
                 f"`bench.py` traced by `tools/gpu.sh prof`: {a.frames:g} coded frames, trace span "
                 f"{span:.1f} ms, kernel busy time {out['busy_ms_per_frame']:.3f} ms per frame "
                 "(summed over streams: the twin instance and the lookahead engine overlap).", "",
                 f"Occupancy ({occ['window']}): some kernel in flight {occ['any_kernel_frac']:.1%} of the span, "
                 f"{occ['mean_kernels_in_flight']:.2f} kernels in flight on average; busiest "
                 "streams (fraction of the span with a kernel of theirs running): " +
                 ", ".join(f"{q}: {v['busy_frac']:.1%}" for q, v in
                           list(occ["streams"].items())[:6]), ""]
        if "bench_line" in out:
            lines += [f"Bench line of the traced run: `{json.dumps(out['bench_line'])}`", ""]
        lines += ["| kernel | ms/frame | launches/frame | avg us | HBM B/launch | round 0 avg us | "
                  "round 0 HBM B | wait/wave-cyc |", "|---|---|---|---|---|---|---|---|"]
        for name, e in out["kernels"].items():
            r0 = e.get("round0", {})
            lines.append(f"| `{name}` | {e['ms_per_frame']:.4f} | {e['launches_per_frame']:.2f} | "
                         f"{e['avg_us']:.2f} | {e.get('hbm_bytes_per_launch', '-')} | "
                         f"{r0.get('avg_us', '-')} | {r0.get('hbm_bytes_per_launch', '-')} | "
                         f"{e.get('sq', {}).get('wait_any_over_wave_cycles', '-')} |")
        with open(a.md, "w") as f:
            f.write("\n".join(lines) + "\n")
    print(json.dumps({k: out[k] for k in ("frames", "span_ms", "busy_ms_per_frame")}))
    for name, e in list(out["kernels"].items())[:12]:
        print(f"{e['ms_per_frame']:8.4f} {e['avg_us']:9.2f}  {name}  {e.get('round0', '')}")


if __name__ == "__main__":
    main()
