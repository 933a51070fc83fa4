#!/usr/bin/env python3
"""bench.py -- encode hot-path replay throughput on MI355X.

Metric (BASELINE.json): encoded frames/sec (+ Mpixels/sec) of the speed-10
hot path of one stream (config D: speed 6), frames resident in HBM, vs the
host CPU running the same schedule.  A "step" = one coded frame of the replay
driver: F0 pyramid, F1 1/4-res full search, F2 the four
half-res quadrant searches, FL the lookahead's 16x16 searches, F3 full-res
diamond + sub-pel (speed 6: also every 32x32, 16x16 and 8x8 block, and the
partition decision), F4 every RDO inter candidate (NEARESTMV / NEAR0MV /
GLOBALMV / NEWMV x reference, skip and non-skip: MC, distortion, diff + fwd
DCT, quantize, estimate_rate, inverse + add) with rav1e's rd cost and
argmin, F6 the winners' reconstruction, F5 8x8 importance SATD, F8 the
committed coefficients' entropy coding (write_coeffs_lv_map: device tokens, a
host range coder beside the next frames; --no-entropy skips it), F7 the
reconstruction becomes a reference.  Frames run in the reorder pyramid's
coding order (me_range_scale 4, 2, 1, 1), the input advances every frame.

N = 1: 2160p 8-bit 4:2:0 speed 10 with BASELINE config C's tiling (8 tile
columns), the metric's configuration, on one GPU.  N > 1
(torch.distributed.run, one process per GPU): the SAME stream, tile
columns split over the ranks (config C: one 8-SB tile column per GPU at
N = 8); after every frame the ranks all-gather the reconstruction over RCCL
(rv_replay_frame).  `value` = frames of the stream / max-over-ranks time
("scaling": "strong").  --config picks the other BASELINE shapes.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
# Hardware queues per process: HIP's default 4, set explicitly before HIP
# initialises.  The three replay instances, their frame-edge / entropy
# streams and the lookahead engine share them; more queues measured slower
# (2160p, 96 frames: 205 fps at 4, 188 at 6, 161 at 8, r04hq -- the more
# streams run side by side, the more the rounds' latency-bound kernels
# lose to the others' work).  RAV1E_BENCH_HW_QUEUES: another count (A/B).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RAV1E_BENCH_HW_QUEUES", "4")
sys.path.insert(0, ROOT)

# name: (width, height, xdec, ydec, bit_depth, tiling kwargs, BASELINE config, speed)
CONFIGS = {
    "360p": (640, 360, 1, 1, 8, {}, "A", 10),
    "1080p": (1920, 1080, 1, 1, 8, {}, "B", 10),
    "2160p": (3840, 2160, 1, 1, 8, {"tile_cols": 8}, "C", 10),
    "2160p10": (3840, 2160, 1, 1, 10, {}, "D", 6),
    "2160p444": (3840, 2160, 0, 0, 8, {"tiles": 4}, "E", 10),
}
TIMING_STRIDE = 4  # in GOPs
IMP_WINDOW = 40  # rdo_lookahead_frames default (src/api/config.rs:158)
_T0 = time.time()


def progress(msg):
    """one line per bench phase on stderr (a long silent run looks hung)"""
    print(f"[bench {time.time() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)
CPU_FRAMES = 8  # coded frames of the CPU baseline / parity stream with a window
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: 8.0 TB/s spec
# VALU issue peaks, G wave64 instructions/s over 256 CUs at 2.4 GHz: the
# guide's 2 cycles per wave instruction per SIMD (MI355X_MICROARCH.md "Wave
# scheduling"), and the rate measured on MI355X for the integer SAD / dot /
# mul24 instructions these kernels are built from (tools/ubench/valu_rates.hip,
# its output committed as profiles/valu_rates.txt; read at run time)
VALU_PEAK_GUIDE = 256 * 4 * 2.4 / 2
VALU_RATES = os.path.join(ROOT, "profiles", "valu_rates.txt")
INT_OPS = ("v_sad_u8", "v_dot4_i32_i8", "v_dot2_i32_i16", "v_mad_i32_i24")


def valu_peak_int():
    """Mean measured issue rate of INT_OPS (wave-instr / cycle / CU) x 256
    CUs x 2.4 GHz, and the file it came from; None if the file is absent."""
    if not os.path.exists(VALU_RATES):
        return None
    rates = {}
    with open(VALU_RATES) as f:
        for line in f:
            parts = line.split()
            if len(parts) > 4 and parts[0] in INT_OPS and parts[4] == "wave-instr/cycle/CU":
                rates[parts[0]] = float(parts[3])
    if len(rates) != len(INT_OPS):
        return None
    per_cu = sum(rates.values()) / len(rates)
    return {"G_per_s": round(per_cu * 256 * 2.4, 1), "wave_instr_per_cycle_per_cu": round(per_cu, 4),
            "ops": rates, "source": "profiles/valu_rates.txt"}
# FL runs on a second stream by default: "FL_on_main_stream" is then the
# fork alone, and "FL_lookahead_span" the lookahead's own span, overlapped
# with F3/F4 (RAV1E_HIP_REPLAY_SERIAL=1: both on one stream)
STAGES = ["F0_pyramid", "F1_full_search", "F2_half_res_quadrants", "FL_on_main_stream",
          "F3_diamond_fullpel", "F3_diamond_subpel", "F4_rdo_single_ref", "F4_rdo_compound",
          "F4_argmin_and_mv_stack_rounds", "F6_commit", "F6b_intra_screen_rdo", "F5_importance_satd",
          "F7_pad_exchange", "FL_lookahead_span", "EDGE_levels_span", "F8_entropy_tokens"]
# speed 6: the 32x32 / 16x16 / 8x8 searches run inside the sub-pel stage,
# their candidates inside F4, the partition decision with the argmin
STAGES6 = ["F0_pyramid", "F1_full_search", "F2_half_res_quadrants", "FL_on_main_stream",
           "F3_diamond_fullpel", "F3_subpel_and_level_me", "F4_rdo_single_ref_all_levels",
           "F4_rdo_compound_all_levels", "F4_argmin_partition", "F6_commit_leaves",
           "F6b_intra_screen_rdo", "F5_importance_satd", "F7_pad_exchange", "FL_lookahead_span",
           "EDGE_levels_span", "F8_entropy_tokens"]


def coarse_windows(W, H, R, scale, tiling, group):
    """(nx, ny) of every F1 job: estimate_motion_ss4's window
    (src/me.rs:1023-1075), as the replay builds it (tile-relative
    adjust_bo)."""
    w_in_b, h_in_b = 2 * ((W + 7) >> 3), 2 * ((H + 7) >> 3)
    tws, ths = tiling["tile_width_sb"], tiling["tile_height_sb"]
    gx0, gy0, gw, gh = group

    def tdiv8(v):
        return int(v / 8)
    out = []
    for sb in range(gw * gh):
        fx, fy = gx0 + sb % gw, gy0 + sb // gw
        t0x, t0y = fx - fx % tws, fy - fy % ths
        mi_w = min(W - t0x * 64, tws * 64) >> 2
        mi_h = min(H - t0y * 64, ths * 64) >> 2
        bx, by = (fx - t0x) * 16, (fy - t0y) * 16
        bx, by = max(min(bx, mi_w - 16), 0), max(min(by, mi_h - 16), 0)
        fbx, fby = bx + t0x * 16, by + t0y * 16
        mr = [-fbx * 32 - 640, (w_in_b - fbx - 16) * 32 + 640,
              -fby * 32 - 640, (h_in_b - fby - 16) * 32 + 640]
        rx, ry = 192 * scale, 64 * scale
        x_lo = fbx + (max(-rx, tdiv8(mr[0])) >> 2)
        x_hi = fbx + (min(rx, tdiv8(mr[1])) >> 2)
        y_lo = fby + (max(-ry, tdiv8(mr[2])) >> 2)
        y_hi = fby + (min(ry, tdiv8(mr[3])) >> 2)
        out.append((max(0, x_hi - x_lo + 1), max(0, y_hi - y_lo + 1)))
    return out * R


# rocprofv3 kernel names of the bench's kernel classes (u8 / u16 builds)
ROCPROF_NAMES = {
    "full_search": "fs16_sea_kernel_{pxs}",
    "diamond_fullpel_64": "ds_fast_kernel<{px}, 64, 64, false>",
    "diamond_subpel_64": "ds_fast_kernel<{px}, 64, 64, true>",  # (+ ds_f2_f3_kernel: fused rounds)
    "rdo_candidates": "rdo_quad_list_kernel<{px}, 0, 0>",
    "rdo_compound": "rdo_quad_list_kernel<{px}, 1, 1>",
    "rdo_commit": "rdo_quad_kernel<{px}, 2>",
}


def _prof_json(args):
    """The newest committed kernel profile of this config
    (profiles/rNN_prof_<config>.json, tools/prof_json.py over a
    `tools/gpu.sh prof` run of this bench)."""
    import glob
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_prof_{args.config}.json")))
    # profiles/prof_current.json names the current one per config (tags do
    # not sort by time)
    cur = os.path.join(ROOT, "profiles", "prof_current.json")
    if os.path.exists(cur):
        with open(cur) as f:
            name = json.load(f).get(args.config)
        if name and os.path.exists(os.path.join(ROOT, "profiles", name)):
            fs = [os.path.join(ROOT, "profiles", name)]
    if args.refs != 2 or not fs:
        return None
    with open(fs[-1]) as f:
        return json.load(f)


def _kernels_trace(pj):
    """Every kernel of the committed trace of this bench, per coded frame
    (all launches: round 0, the MV-stack rounds, the lookahead engine, the
    twin), up to 95 % of the busy time; busy time is summed over streams,
    which overlap, so it may exceed the step."""
    ks = list(pj["kernels"].items())
    busy = pj["busy_ms_per_frame"]
    out, acc = {}, 0.0
    for k, v in ks:
        if acc >= 0.95 * busy:
            break
        out[k] = {"ms_per_frame": v["ms_per_frame"], "launches_per_frame": v["launches_per_frame"]}
        acc += v["ms_per_frame"]
    bl = pj.get("bench_line") or {}
    return {"source": pj["source"], "git": pj["git"], "busy_ms_per_frame": busy,
            "listed_ms_per_frame": round(acc, 4),
            "traced_run_ms_per_step": bl.get("ms_per_step"),
            "busy_over_step": round(busy / bl["ms_per_step"], 3) if bl.get("ms_per_step") else None,
            "kernels": out}


def timed_run(engine, group, steps, warmup, sync=None, finish=None, before=None, start=None,
              mark=None):
    """W untimed frames (the key frame first), then exactly K timed coded
    frames bracketed by a barrier and a device sync on both sides; returns
    (max-over-ranks seconds, result words of the last frame).  `engine` is a
    HipReplay / TileParallel (the product) or, in the multi-rank CPU tests,
    the oracle's CpuReplay behind a TileParallel.  before(): after the
    warmup, outside the timing (probes reset); start(): the first thing
    inside the timing (the lookahead engine released); mark(): an empty
    marker kernel right before t0 and after t1 (a kernel trace's timed
    region, tools/prof_json.py)."""
    drain = getattr(engine, "drain", None)  # PairedReplay: frames issued from a second thread
    for i in range(warmup):
        engine.frame()
        progress(f"warmup frame {i} issued")
    if warmup:
        engine.results()  # drains the stream
    progress(f"warmup: {warmup} frames")
    if before:
        before()
    group.barrier()
    if sync:
        sync()
    if mark:
        mark()
    t0 = time.perf_counter()
    if start:
        start()
    for _ in range(steps):
        engine.frame()
    if drain:
        drain()
    if sync:
        sync()  # device-wide: every frame on every stream has finished
    if finish:
        finish()  # the host's share of the frames (F8's range coder) has finished too
    t1 = time.perf_counter()
    if mark:
        mark()
    progress(f"timed: {steps} frames in {t1 - t0:.3f} s")
    group.barrier()
    # the verification checksums are not part of a frame: outside the timing
    words = engine.results()
    return group.max(t1 - t0), words


def cpu_baseline_and_parity(args, hip_inputs, W, H, xdec, ydec, bd, nref, tiling, n_inputs,
                            speed=10, flags=0, imp_window=0):
    """The CPU baseline and the full-size parity check, from one CPU run.

    The CPU replay (oracle/orc_replay.c: the same schedule over the oracle's
    restatements; the build for this host's ISA level) codes the stream's
    first frames (the key frame, then >= one GOP) on every host thread this
    process may use, timed, keeping each frame's result words.  A fresh GPU
    replay then codes the same frames and its words must equal the CPU's,
    frame by frame: the bench's own full-size bit-exactness check.  A
    bounded 1-thread sample (the first superblocks of one GOP) is timed
    beside it.  With an importance window both code a stream of CPU_FRAMES
    coded frames (the window shrinks at its end, as rav1e's does at the end
    of a stream)."""
    import rav1e_amd as R
    from rav1e_amd import replay as RP
    from tests import oracle_lib as O  # the checker / CPU baseline only
    L, isa = O.baseline_lib()
    threads = O.cpu_share()
    ts = (tiling["tile_width_sb"], tiling["tile_height_sb"])
    nin = len(hip_inputs)
    db = bool(flags & RP.RV_REPLAY_DEBLOCK)
    cd = bool(flags & RP.RV_REPLAY_CDEF)
    ent = bool(flags & RP.RV_REPLAY_ENTROPY)
    sti = bool(flags & RP.RV_REPLAY_MVREF_STANDIN)
    lrf = bool(flags & RP.RV_REPLAY_LRF)
    limit = CPU_FRAMES + 1 if imp_window else 0
    c = O.CpuReplay(W, H, xdec, ydec, bd, nref, tile_size=ts, n_inputs=nin, threads=threads, L=L,
                    speed=speed, deblock=db, cdef=cd, entropy=ent, mvref_standin=sti,
                    imp_window=imp_window, imp_limit=limit, lrf=lrf)
    for i in range(nin):
        c.set_input(i, hip_inputs[i])
    c.frame()  # the key frame (a copy), untimed
    progress("CPU replay: started")
    cpu_words, cpu_ent = [], []
    n, tc0 = 0, time.perf_counter()
    while n < 4 or (time.perf_counter() - tc0 < args.cpu_seconds and n < nin - 6 and
                    (not limit or n < CPU_FRAMES)):
        c.frame()
        n += 1
        cpu_words.append(c.results())  # a memcpy + sums; kept inside the timing
        if ent:
            cpu_ent.append(c.entropy_stats()[:3])
    tc = time.perf_counter() - tc0
    progress(f"CPU replay: {n} frames in {tc:.1f} s")
    c.close()
    # 1 thread: the first 1/8 of the superblocks of one GOP
    nsb = ((W + 63) // 64) * ((H + 63) // 64)
    lim = max(1, nsb // 8)
    c1 = O.CpuReplay(W, H, xdec, ydec, bd, nref, tile_size=ts, n_inputs=nin, threads=1, L=L,
                     speed=speed, deblock=db, cdef=cd, entropy=ent, mvref_standin=sti,
                     imp_window=imp_window, imp_limit=5 if imp_window else 0)
    for i in range(nin):
        c1.set_input(i, hip_inputs[i])
    c1.frame()
    t1 = time.perf_counter()
    for _ in range(4):
        c1.frame(lim)
    t1 = time.perf_counter() - t1
    c1.close()
    fps1 = 4 * (lim / nsb) / t1
    progress("CPU one-thread sample done")
    cpu = {"value": round(n / tc, 4), "unit": "frames/s", "cores": threads, "kind": "port",
           "isa": isa,
           "cores_note": "the GPU box's per-GPU CPU share (16 threads; the harness sizes worker "
                         "pools to it), not every physical core of the host as SURVEY.md §8d "
                         "asks; a scalar C restatement of the schedule, not rav1e's SIMD path",
           "sample": f"the first {n} coded {args.config} frames of the same stream and schedule "
                     f"(after the key frame), oracle/orc_replay.c -O3 -march={isa} on "
                     f"{threads} host threads",
           "mpix_per_s": round(n / tc * W * H / 1e6, 3),
           "one_thread": {"value": round(fps1, 5), "unit": "frames/s",
                          "sample": f"first {lim} of {nsb} superblocks of each frame of one GOP, "
                                    f"scaled to whole frames"}}
    # the GPU replay over the same frames, word for word
    g = RP.HipReplay(W, H, xdec, ydec, bd, nref, tile_size=ts, n_inputs=n_inputs,
                     flags=flags & (RP.RV_REPLAY_SPEED6 | RP.RV_REPLAY_DEBLOCK |
                                    RP.RV_REPLAY_CDEF | RP.RV_REPLAY_ENTROPY |
                                    RP.RV_REPLAY_MVREF_STANDIN | RP.RV_REPLAY_LRF),
                     imp_window=imp_window, imp_limit=limit)
    g.synth_inputs(0)
    g.frame()
    bad = []
    for i in range(n):
        g.frame()
        gw = g.results()
        d = np.nonzero(gw != cpu_words[i])[0]
        if d.size:
            bad.append({"frame": i, "n_diff": int(d.size), "first": int(d[0])})
        if ent and g.entropy_stats()[:3] != cpu_ent[i]:
            bad.append({"frame": i, "entropy": "coefficient bytes differ"})
    g.close()
    R._check(R.lib().rv_device_sync(), "rv_device_sync")
    progress(f"GPU parity pass: {n} frames, {len(bad)} mismatches")
    parity = {"frames": n, "words": int(sum(w.size for w in cpu_words)),
              "bit_exact": not bad, "vs": "oracle/orc_replay.c (CPU replay)",
              **({"importance_window": imp_window, "stream_frames": limit} if imp_window else {})}
    if ent:
        parity["coefficient_bytes"] = int(sum(e[0] for e in cpu_ent))
    if bad:
        parity["mismatches"] = bad[:8]
    return cpu, parity


# The lookahead engine's kernels (rocprofv3 names) and how a rank's share of
# them scales at N ranks: the searches and the 8x8 importance data run on the
# rank's own tile group (1 / N), the window's target lists and propagation
# over the whole frame on every rank
LA_KERNELS_PER_GROUP = ("ds_grp_kernel<{px}, 16, false, false>", "la_check_kernel",
                        "fs16_sea_kernel_{pxs}", "pyramid_kernel<{px}>", "box_sums_kernel<{px}>",
                        "data_kernel<{px}>")
LA_KERNELS_WHOLE_FRAME = ("pass_kernel", "csr_scan_kernel", "csr_scatter_kernel", "csr_order_kernel",
                          "keys_kernel", "zero_kernel", "final_kernel")


def emulate_ranks(n, W, H, xdec, ydec, bd, nref, tiling, flags, gops=6, imp_window=0, pj=None):
    """The N-rank tile-group split on ONE GPU: config's n tile groups as n
    HipReplay instances (the ranks), each frame coded group by group with
    the GPU to itself, the all-gather emulated by device copies into every
    group's receive buffer (RCCL's layout), then every group's import
    (unpack, loop filters, pad).  Per group: the wall time of its frame
    (frame() to a device sync: every stream of the group -- F0 .. F8, the
    frame-edge levels, the side streams); averaged over the frames past GOP 4.
    The groups' lookahead engines run ahead (inputs declared in place: the
    window's part exchange needs every group's engine), so their per-frame
    work is not in that span; it is added from the committed kernel trace of
    the one-GPU bench: the rank's share of the search kernels (1 / N) and
    all of the whole-frame importance propagation.  The projected N-rank step
    = the slowest group + that lookahead share + the slowest import + the
    all-gather at an assumed xGMI rate.  At N > 1 every rank codes its frames
    one after another (PipelinedReplay is one-GPU only), which this models."""
    import ctypes as C

    import rav1e_amd as R
    from rav1e_amd import replay as RP
    L = R.lib()
    ts = (tiling["tile_width_sb"], tiling["tile_height_sb"])
    rects = RP.tile_groups(tiling, n)
    gop = len(RP.GOP_SCALES)
    frames = 1 + gops * gop
    nin = frames + 8 + (imp_window + 37 if imp_window else 0)
    gs = [RP.HipReplay(W, H, xdec, ydec, bd, nref, group=r, tile_size=ts, n_inputs=nin,
                       flags=flags, imp_window=imp_window) for r in rects]
    # the importance window: each group's engine computes its blocks' part,
    # the parts meet in an in-process hub (the ranks' RCCL all-gather)
    hub = RP.LaHub(n) if imp_window else None
    sync = lambda: R._check(L.rv_device_sync(), "rv_device_sync")  # noqa: E731
    for k, g in enumerate(gs):
        g.synth_inputs(0)
        g.set_groups(rects, k, None)
        if hub:
            g.set_la_exchange(hub=hub)
            g.set_inputs_ready(nin)  # the groups code one after another here
        g.set_timing(1, 1)
    bufs = [g.exchange_buffers() for g in gs]
    nb = bufs[0][2]
    span = [[] for _ in gs]
    imp = [[] for _ in gs]
    progress(f"emulated ranks: {n} groups")
    stage = [[] for _ in gs]
    for f in range(frames):
        timed = f > 4 * gop  # past GOP 4: every me_range_scale once per GOP
        order = range(n - 1, -1, -1) if os.environ.get("RAV1E_BENCH_EMU_REVERSE") else range(n)
        for k in order:  # (reversed: A/B of the first group's position)
            g = gs[k]
            t0 = time.perf_counter()
            g.frame()
            sync()
            if timed:
                span[k].append((time.perf_counter() - t0) * 1e3)
                stage[k].append(float(g.stage_ms()[:13].sum()))
        if f == 0:
            continue  # the key frame: every group copied its own input
        for k in range(n):
            for j in range(n):
                R._check(L.rv_memcpy_d2d(C.c_void_p(bufs[k][1] + j * nb), C.c_void_p(bufs[j][0]),
                                         nb, None), "rv_memcpy_d2d")
        sync()
        for k, g in enumerate(gs):
            t0 = time.perf_counter()
            g.import_()
            sync()
            if timed:
                imp[k].append((time.perf_counter() - t0) * 1e3)
    progress("emulated ranks: done")
    cnts = [[int(v) for v in g.counters()] for g in gs]
    for g in gs:
        g.close()
    if hub:
        hub.close()
    per = [sum(s) / len(s) for s in span]
    per_stage = [sum(s) / len(s) for s in stage]
    imp_ms = max(sum(s) / len(s) for s in imp)
    xgmi_gbs = 64.0  # assumed all-gather algorithm bandwidth per rank (RCCL over xGMI)
    ag_ms = (n - 1) * nb / (xgmi_gbs * 1e9) * 1e3
    la_ms, la_src = 0.0, None
    if imp_window and pj:
        pxn = "unsigned short" if bd > 8 else "unsigned char"
        fmt = dict(px=pxn, pxs="u16" if bd > 8 else "u8")
        grp = sum(v["ms_per_frame"] for k, v in pj["kernels"].items()
                  if any(nm.format(**fmt) in k for nm in LA_KERNELS_PER_GROUP))
        whole = sum(v["ms_per_frame"] for k, v in pj["kernels"].items()
                    if any(nm in k for nm in LA_KERNELS_WHOLE_FRAME))
        la_ms = grp / n + whole
        la_src = {"source": pj["source"], "git": pj["git"], "search_ms_per_frame": round(grp, 4),
                  "whole_frame_ms_per_frame": round(whole, 4),
                  "rule": "searches / N + the whole-frame propagation, from the one-GPU trace"}
    proj = max(per) + la_ms + imp_ms + ag_ms
    return {"ranks": n, "groups_sb": [list(r) for r in rects],
            "group_frame_ms": [round(v, 4) for v in per], "max_group_ms": round(max(per), 4),
            "group_stage_sum_ms": [round(v, 4) for v in per_stage],
            "lookahead_ms_per_rank": round(la_ms, 4), "lookahead_model": la_src,
            "import_ms_max": round(imp_ms, 4), "exchange_bytes_per_group": int(nb),
            "allgather_ms_model": round(ag_ms, 4),
            "allgather_model": f"(n-1) x bytes_per_group at an assumed {xgmi_gbs:g} GB/s",
            "projected_ms_per_step": round(proj, 4),
            "projected_frames_per_s": round(1e3 / proj, 2),
            "frames_averaged": len(span[0]),
            # per group, over all its frames: MV-stack rounds and re-evaluated
            # superblocks per frame, outer passes, lookahead rounds
            "group_rounds_per_frame": [round(c[14] / max(1, c[16]), 2) for c in cnts],
            "group_reevaluated_sb_per_frame": [round(c[15] / max(1, c[16]), 1) for c in cnts],
            "group_lookahead_rounds_per_frame": [round(c[18] / max(1, c[16]), 2) for c in cnts],
            "group_order": "groups code each frame in index order (group 0 first)",
            "importance_window": imp_window,
            "method": "one GPU, groups run one after another (wall clock of each group's "
                      "frame to a device sync, frames past GOP 4; import wall clock incl. "
                      "launch), device-copy all-gather; each rank codes its frames serially"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 96 frames: a steady-state sample (24 GOPs; the lookahead engine's lead
    # is capped at the window at the start of the timing, see below)
    ap.add_argument("--steps", type=int, default=96)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="2160p", choices=sorted(CONFIGS))
    ap.add_argument("--refs", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--speed", type=int, choices=(6, 10), default=None,
                    help="schedule (default: the config's BASELINE speed)")
    ap.add_argument("--loop-filters", choices=("all", "cdef", "deblock", "none"), default="all",
                    help="the in-loop filters every coded frame runs before it becomes a "
                         "reference: rav1e's deblocking (fast levels at speed >= 8, "
                         "sse_optimize below), CDEF (cdef_preset is always true, "
                         "src/api/config.rs:421-423) and loop restoration (enable_restoration "
                         "on 4:2:0 / 4:4:4, src/encoder.rs:229-230, 2789-2806; one tile group: "
                         "off with several ranks) -- the default; 'cdef' / 'deblock' / 'none' "
                         "for A/B")
    ap.add_argument("--emulate-ranks", type=int, default=8,
                    help="N > 1 (single-GPU runs): also code the N-rank tile-group split as N "
                         "replays on this GPU and report the projected N-rank step (0: off)")
    ap.add_argument("--serial-levels", action="store_true",
                    help="one instance codes every frame (default on one GPU: the level-2 "
                         "frames run on a twin instance concurrently with levels 0 / 1)")
    ap.add_argument("--mv-stack", choices=("exact", "standin"), default="exact",
                    help="speed 10: rav1e's find_mvrefs stacks in coding-order rounds (default), or "
                         "the neighbour-NEWMV stand-in (A/B of the rounds' cost)")
    ap.add_argument("--no-entropy", action="store_true",
                    help="skip stage F8 (the coefficients' entropy coding: device tokens + "
                         "the host range coder); default: every frame's coefficients are coded")
    ap.add_argument("--exhaustive-fs", action="store_true",
                    help="F1 coarse search without successive elimination (same results)")
    ap.add_argument("--imp-window", type=int, default=IMP_WINDOW,
                    help="rdo_lookahead_frames: block importances propagated over that many "
                         "coded frames ahead (rav1e's default 40; 0: importance 0, bias 0.65); "
                         "with several GPUs each rank computes its tile group's lookahead part "
                         "and the parts are all-gathered (the propagation reads the whole frame)")
    args = ap.parse_args()
    # a stalled run names where it stalled (every thread's stack on stderr)
    import faulthandler
    faulthandler.dump_traceback_later(120, repeat=True, file=sys.stderr)

    import rav1e_amd as R  # load the HIP library before anything else
    from rav1e_amd import replay as RP
    from rav1e_amd.ranks import RankGroup, TileParallel, rank_info
    R.lib()
    info = rank_info()
    rank, world = info.rank, info.world
    group = RankGroup(info)
    R.require_device(info.local_rank % max(1, R.lib().rv_device_count()))

    W, H, xdec, ydec, bd, tkw, cfg_name, speed = CONFIGS[args.config]
    speed = args.speed or speed
    nref = args.refs
    tiling = RP.tiling_for(W, H, **tkw)
    ts = (tiling["tile_width_sb"], tiling["tile_height_sb"])
    rects = RP.tile_groups(tiling, world)
    imp_window = args.imp_window
    # every display the run codes, the lookahead's W frames beyond, and the
    # engine's ring slack (RW = W + 29: it may run that far past the oldest
    # frame in flight).  The stream is unbounded (imp_limit 0): every frame's
    # window reaches W frames ahead, so the engine's lookahead of frames past
    # the run is inside the timed region, as in a streaming encode, and it
    # never runs out of inputs before the last timed frame
    n_inputs = args.warmup + args.steps + 8 + (imp_window + 29 + 8 if imp_window else 0)
    deblock = args.loop_filters in ("all", "cdef", "deblock")
    cdef = args.loop_filters in ("all", "cdef")
    # loop restoration: 4:2:2 has none (enable_restoration,
    # src/encoder.rs:229-230); with tile groups each rank decides its own
    # units and they travel with its reconstruction
    lrf = args.loop_filters == "all" and not (xdec == 1 and ydec == 0)
    flags = (RP.RV_REPLAY_EXHAUSTIVE_FS if args.exhaustive_fs else 0) | \
        (RP.RV_REPLAY_SPEED6 if speed == 6 else 0) | (RP.RV_REPLAY_DEBLOCK if deblock else 0) | \
        (RP.RV_REPLAY_CDEF if cdef else 0) | (0 if args.no_entropy else RP.RV_REPLAY_ENTROPY) | \
        (RP.RV_REPLAY_MVREF_STANDIN if args.mv_stack == "standin" else 0) | \
        (RP.RV_REPLAY_LRF if lrf else 0)
    hip = RP.HipReplay(W, H, xdec, ydec, bd, nref, group=rects[rank], tile_size=ts,
                       n_inputs=n_inputs, flags=flags, imp_window=imp_window,
                       imp_limit=0)
    hip.synth_inputs(0)  # the stream's frames, resident in HBM before the timing
    # The lookahead engine's lead: during the warmup it runs only the W
    # frames each coded frame's window needs (no inputs declared ready), so
    # at the start of the timing it is exactly W frames ahead of the encode.
    # The first thing inside the timing declares every input in place, and
    # from then on it runs as far ahead as its ring allows, as rav1e computes
    # a frame's lookahead when the frame arrives.  So every timed frame's own
    # lookahead (frame n + W's, for n's window) is computed inside the timing:
    # the line reports that count (>= steps), and no lookahead done before
    # the timing flatters it.
    ready = bool(imp_window) and os.environ.get("RAV1E_BENCH_NO_READY") != "1"
    comm = RP.RcclComm(group) if world > 1 else None
    eng = TileParallel(hip, rects, rank, group, comm)
    paired = world == 1 and not args.serial_levels
    if paired:
        # three instances (PipelinedReplay: 2160p 205-206 vs 189-193 fps for
        # two, r04p4); RAV1E_BENCH_INSTANCES=2: PairedReplay (A/B)
        eng = (RP.PairedReplay(hip) if os.environ.get("RAV1E_BENCH_INSTANCES") == "2"
               else RP.PipelinedReplay(hip))
    sea = bd <= 10 and not args.exhaustive_fs  # the replay's F1 path
    # HIP events on a sample of frames: every TIMING_STRIDE-th GOP
    gop = len(RP.GOP_SCALES)
    (eng if paired else hip).set_timing(TIMING_STRIDE, gop)
    ent = not args.no_entropy
    # RAV1E_BENCH_NO_PROBE=1: no kernel probe (A/B of the probe's own cost)
    probe = (world == 1 and speed == 10 and hasattr(eng, "set_kernel_probe")
             and os.environ.get("RAV1E_BENCH_NO_PROBE") != "1")
    la_cnt = {}

    def before():
        if probe:  # the F3 sub-pel kernel probe over the timed frames
            eng.set_kernel_probe(True)
        if imp_window:
            la_cnt["t0"] = int((eng if paired else hip).counters()[20])

    def start():
        if ready:
            hip.set_inputs_ready(n_inputs)

    dt, words = timed_run(eng, group, args.steps, args.warmup,
                          sync=lambda: R._check(R.lib().rv_device_sync(), "rv_device_sync"),
                          finish=eng.entropy_stats if ent else None, before=before, start=start,
                          mark=lambda: R._check(R.lib().rv_trace_marker(None), "rv_trace_marker"))
    if imp_window:
        la_cnt["t1"] = int((eng if paired else hip).counters()[20])
    kp = eng.kernel_probe() if probe else None
    if os.environ.get("RAV1E_HIP_DS_PHASES") == "1":  # diagnostic: the rounds' sub-pel phases
        R._check(R.lib().rv_ds_phase_dump(), "rv_ds_phase_dump")
    if os.environ.get("RAV1E_HIP_RDO_PHASES") == "1":  # diagnostic: the rounds' F4 phases
        R._check(R.lib().rv_rdo_phase_dump(), "rv_rdo_phase_dump")
    ent_stats = eng.entropy_stats() if ent else None

    # per-kernel times over the instrumented frames of the timed region
    nonkey = range(args.warmup - 1, args.warmup - 1 + args.steps)
    k = min(sum(1 for f in nonkey if (f // gop) % TIMING_STRIDE == 0), 64)
    k = max(k, 1)
    if paired:  # the instrumented frames of each instance in the timed region
        inst = [f for f in nonkey if (f // gop) % TIMING_STRIDE == 0]
        if hasattr(eng, "stage_ms_sum_frames"):
            ssum, kn = eng.stage_ms_sum_frames(inst)
            ms = ssum / max(1, kn)
        else:
            kp = min(sum(1 for f in inst if eng.on_primary(f)), 64)
            kt = min(sum(1 for f in inst if not eng.on_primary(f)), 64)
            ms = eng.stage_ms_sum(kp, kt) / max(1, kp + kt)
        cnt = [int(v) for v in eng.counters()]
    else:
        ms = hip.stage_ms_sum(k) / k  # per frame
        cnt = [int(v) for v in hip.counters()]
    ev_full, ev_sub, ev_frames, n_single, n_comp = cnt[:5]
    ev_frames = max(1, ev_frames)
    gx0, gy0, gw, gh = rects[rank]
    nsb = gw * gh
    px = 2 if bd > 8 else 1
    # algorithmic bytes per frame of each kernel class; the
    # SEA search also reads the box-sum tables: per 4-wide x 8-tall tile of
    # candidates, 20 rows of 16 B (paired u32 4x8 sums, rv_me.hip)
    fs_bytes = sum(sum((nx + 15) * (ny + 15) * px + 256 * px + 56 +
                       (((nx + 3) // 4) * ((ny + 7) // 8) * 20 * 16 if sea else 0)
                       for nx, ny in coarse_windows(W, H, nref, s, tiling, rects[rank]))
                   for s in RP.GOP_SCALES) / 4.0
    nj = nsb * nref
    cw, ch = 64 >> xdec, 64 >> ydec
    ntx_c = (cw // 32) * (ch // 32)
    # F4 per evaluated candidate (the measured counts): luma (64+7)^2 window
    # (two for compound) + 64x64 source + 3 result words; per chroma 32x32
    # transform block the same at 32 (U and V)
    ns, nc = n_single / ev_frames, n_comp / ev_frames
    rdo_bytes = float(ns * ((71 * 71 + 64 * 64) * px + 24) +
                      2 * ntx_c * ns * ((39 * 39 + 32 * 32) * px + 24))
    comp_bytes = float(nc * ((2 * 71 * 71 + 64 * 64) * px + 24) +
                       2 * ntx_c * nc * ((2 * 39 * 39 + 32 * 32) * px + 24))
    # commit: one candidate per superblock, + levels and the reconstruction
    commit_bytes = float(nsb * ((71 * 71 + 2 * 64 * 64) * px + 4096 + 16) +
                         2 * nsb * ntx_c * ((39 * 39 + 2 * 32 * 32) * px + 4096))
    level_cands = {}
    if speed == 6:
        # the 32x32 / 16x16 / 8x8 candidates: B x B luma ((B+7)^2 window + source),
        # bc x bc per chroma plane, 3 result words each; compound reads two windows
        for l in (1, 2, 3):
            B = 64 >> l
            bc = B >> xdec
            s1, c1 = cnt[5 + 2 * (l - 1)] / ev_frames, cnt[6 + 2 * (l - 1)] / ev_frames
            level_cands[f"{B}x{B}"] = {"single_ref": round(s1, 1), "compound": round(c1, 1)}
            rdo_bytes += s1 * (((B + 7) ** 2 + B * B) * px + 24 +
                               2 * (((bc + 7) ** 2 + bc * bc) * px + 24))
            comp_bytes += c1 * ((2 * (B + 7) ** 2 + B * B) * px + 24 +
                                2 * ((2 * (bc + 7) ** 2 + bc * bc) * px + 24))
    kernels = {
        "full_search": dict(ms=float(ms[1]), bytes=fs_bytes),
        "diamond_fullpel_64": dict(ms=float(ms[4]),
                                   bytes=nj * (64 * 64 * px + 80) + ev_full / ev_frames * 64 * 64 * px),
        "diamond_subpel_64": dict(ms=float(ms[5]),
                                  bytes=nj * (64 * 64 * px + 80) + ev_sub / ev_frames * 71 * 71 * px),
        "rdo_candidates": dict(ms=float(ms[6]), bytes=rdo_bytes),
        "rdo_compound": dict(ms=float(ms[7]), bytes=comp_bytes),
        "rdo_commit": dict(ms=float(ms[9]), bytes=commit_bytes),
    }
    pj = _prof_json(args)
    pk = valu_peak_int()
    pxn = "unsigned short" if bd > 8 else "unsigned char"

    def trace_entry(kernel):
        """the kernel's entry in the committed trace + PMC summary of this bench"""
        nm = ROCPROF_NAMES.get(kernel, "?").format(px=pxn, pxs="u16" if bd > 8 else "u8")
        return next((v for k, v in pj["kernels"].items() if nm in k), None) if pj else None

    def valu_of(te, avg_s, hbm_frac):
        """VALU rate of a kernel: its SQ_INSTS_VALU per launch (the committed SQ
        pass of the same bench) over the live launch duration"""
        sq = te.get("sq") if te else None
        if not sq:
            return None, None
        achv = sq["valu_insts_per_launch"] / avg_s / 1e9
        v = {"achieved": round(achv, 1), "unit": "G wave64 VALU instr/s",
             "peak_guide": VALU_PEAK_GUIDE, "frac_guide": round(achv / VALU_PEAK_GUIDE, 4),
             "insts_per_launch": sq["valu_insts_per_launch"],
             "waves_per_launch": sq.get("waves_per_launch"), "source": pj["source"], "git": pj["git"]}
        if pk:
            v.update(peak_int_measured=pk["G_per_s"], frac_int_measured=round(achv / pk["G_per_s"], 4),
                     peak_int_source=pk["source"])
        wait = sq["wait_any_over_wave_cycles"]
        lim = {"resource": ("latency: waves parked on s_waitcnt / barriers" if wait > 0.3 else
                            "VALU issue" if achv / VALU_PEAK_GUIDE > 0.6 else "mixed issue / latency"),
               "SQ_WAIT_ANY_over_WAVE_CYCLES": wait,
               "SQ_ACTIVE_INST_ANY_over_WAVE_CYCLES": sq["active_inst_over_wave_cycles"],
               "valu_frac_guide": round(achv / VALU_PEAK_GUIDE, 4), "hbm_frac": hbm_frac,
               "source": pj["source"]}
        return v, lim

    def family_entry(sub):
        """Every instance of a kernel in the committed trace (template
        instances are traced as separate names; `sub`: a name substring or a
        tuple of them) aggregated per coded frame: ms, launches, mean launch,
        and HBM bytes / SQ ratios weighted by launches."""
        if not pj:
            return None
        subs = sub if isinstance(sub, tuple) else (sub,)
        es = [v for k, v in pj["kernels"].items() if any(x in k for x in subs)]
        if not es:
            return None
        lpf = sum(e["launches_per_frame"] for e in es)
        mpf = sum(e["ms_per_frame"] for e in es)
        out = {"ms_per_frame": round(mpf, 4), "launches_per_frame": round(lpf, 3),
               "avg_us": round(mpf * 1e3 / lpf, 3), "instances": len(es)}
        if all(e.get("hbm_bytes_per_launch") for e in es):
            out["hbm_bytes_per_launch"] = round(sum(e["hbm_bytes_per_launch"] * e["launches_per_frame"]
                                                    for e in es) / lpf)
        if all(e.get("sq") for e in es):
            w = [e["launches_per_frame"] / lpf for e in es]
            out["sq"] = {k: round(sum(wi * e["sq"][k] for wi, e in zip(w, es)), 4)
                         for k in ("wait_any_over_wave_cycles", "active_inst_over_wave_cycles",
                                   "valu_insts_per_launch", "waves_per_launch")}
        return out

    def attach_trace(roof, te, bytes_l, avg_s, ach):
        if not te:
            return
        roof["trace"] = {"source": pj["source"], "git": pj["git"], "avg_us": te["avg_us"],
                         "launches_per_frame": te["launches_per_frame"],
                         "ms_per_frame": te["ms_per_frame"],
                         "frac_from_trace": round(bytes_l / (te["avg_us"] * 1e-6) / 1e9 /
                                                  HBM_PEAK_GBS, 5),
                         "live_over_trace_duration": round(avg_s * 1e6 / te["avg_us"], 3)}
        if te.get("instances"):
            roof["trace"]["instances_aggregated"] = te["instances"]
        if te.get("hbm_bytes_per_launch"):
            roof["traffic"] = {"bytes_per_launch": te["hbm_bytes_per_launch"],
                               "source": pj["source"], "git": pj["git"],
                               "over_algorithmic": round(te["hbm_bytes_per_launch"] / bytes_l, 3),
                               "rule": pj.get("hbm_bytes_rule")}
        v, lim = valu_of(te, avg_s, round(ach / HBM_PEAK_GBS, 5))
        if v:
            roof["valu"], roof["limiter"] = v, lim

    roofs = {}
    if kp is not None and kp[0] > 0:
        # F3's sub-pel search: the batched MC + distortion kernel north_star
        # names (every candidate a 6-tap put_8tap of its 71 x 71 window, then
        # SAD against the source) -- ds_fast_kernel<64, 64, sub-pel> for round
        # 0 and a run's first round, and inside ds_f2_f3_kernel (fused behind
        # F2 || F3 full-pel) for the later MV-stack rounds.  Live: every such
        # launch of the instrumented timed frames; its units: the sub-pel
        # candidate evaluations those launches counted.  The fused launches'
        # F2 and full-pel searches are not counted: achieved is a lower bound.
        nl = float(kp[0])
        # the launch's duration: its span on the device clock (the first
        # workgroup's start to the last one's end, what rocprofv3 times);
        # the HIP event pairs around it also hold the dispatch and the
        # records (reported beside it)
        ev_s = kp[1] / nl / 1e3
        avg_s = kp[4] / nl / 1e3 if len(kp) > 4 and kp[4] > 0 else ev_s
        cand_b = (71 * 71 + 64 * 64) * px + 4  # fused MC + dist candidate
        bytes_l = kp[2] / nl * cand_b
        ach = bytes_l / avg_s / 1e9
        roof = {"kernel": "diamond_subpel_64",
                "name": f"ds_fast_kernel<{pxn}, 64, 64, true> + ds_f2_f3_kernel<{pxn}> (fused rounds)",
                "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                "avg_launch_ms": round(avg_s * 1e3, 5),
                "avg_launch_ms_hip_events": round(ev_s * 1e3, 5),
                "duration": "device clock (wall_clock64) span of every probed launch: first "
                            "workgroup start to last workgroup end; HIP event pairs on the "
                            "launch's stream beside it",
                "algorithmic_bytes_per_launch": round(bytes_l),
                "per_unit": {"unit": "candidate (MC + SAD of one sub-pel MV)", "bytes": cand_b,
                             "rule": "(64+7)^2 b window + 64^2 b source + 4 (SURVEY.md §8d)"},
                "units_per_launch": round(kp[2] / nl, 1), "jobs_per_launch": round(kp[3] / nl, 1),
                "launches_probed": int(nl),
                "launch": "every launch holding F3 sub-pel searches (round 0, each run's first "
                          "round, the fused F2 || F3 launches of the later MV-stack rounds) of "
                          "the instrumented timed frames; the fused launches' F2 and full-pel "
                          "searches are not counted (achieved is a lower bound)"}
        attach_trace(roof, family_entry((f"ds_fast_kernel<{pxn}, 64, 64, true>",
                                         f"ds_f2_f3_kernel<{pxn}>")), bytes_l, avg_s, ach)
        roofs["diamond_subpel_64"] = roof
    if kp is not None and len(kp) >= 12 and kp[5] > 0:
        # F4, rdo_quad_list_kernel: every inter candidate's fused chain (MC,
        # distortion, fht, quantise, rate, inverse, distortion) over the
        # compacted lists, round 0's single-reference and compound launches
        # and each MV-stack round's pair.  Units: the candidates and chroma
        # transform blocks the launches counted (device-side, per launch).
        nl = float(kp[5])
        ev_s = kp[6] / nl / 1e3
        avg_s = kp[7] / nl / 1e3 if kp[7] > 0 else ev_s
        per = {"luma_single": (71 * 71 + 64 * 64) * px + 24,
               "luma_compound": (2 * 71 * 71 + 64 * 64) * px + 24,
               "chroma_single": (39 * 39 + 32 * 32) * px + 24,
               "chroma_compound": (2 * 39 * 39 + 32 * 32) * px + 24}
        # (the chroma counts are per plane: U and V each)
        units = dict(zip(per, (kp[8], kp[9], 2 * kp[10], 2 * kp[11])))
        bytes_l = sum(units[k] * per[k] for k in per) / nl
        ach = bytes_l / avg_s / 1e9
        roof = {"kernel": "rdo_candidates_list", "name": f"rdo_quad_list_kernel<{pxn}, *, *>",
                "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                "avg_launch_ms": round(avg_s * 1e3, 5),
                "avg_launch_ms_hip_events": round(ev_s * 1e3, 5),
                "duration": "device clock (wall_clock64) span of every probed launch: first "
                            "workgroup start to last workgroup end; HIP event pairs on the "
                            "launch's stream beside it",
                "algorithmic_bytes_per_launch": round(bytes_l),
                "per_unit": {"unit": "candidate transform block (its MC window(s) + source + 3 "
                                     "result words)", "bytes": per,
                             "rule": "luma (64+7)^2 b window (two for compound) + 64^2 b source "
                                     "+ 24; chroma per 32x32 block the same at 32 (SURVEY.md §8d: "
                                     "fused MC + distortion candidate)"},
                "units_per_launch": {k: round(v / nl, 1) for k, v in units.items()},
                "launches_probed": int(nl),
                "launch": "every F4 list launch (round 0's single and compound, each MV-stack "
                          "round's pair) of the instrumented timed frames"}
        attach_trace(roof, family_entry(f"rdo_quad_list_kernel<{pxn}"), bytes_l, avg_s, ach)
        roofs["rdo_candidates_list"] = roof
    if roofs:
        # the line prices the kernel with the most milliseconds per frame in
        # the committed trace (every template instance of a kernel summed:
        # rocprofv3 names them apart), or live when there is no trace
        def weight(r):
            t = r.get("trace")
            return t["ms_per_frame"] if t else r["avg_launch_ms"] * r["launches_probed"]
        order = sorted(roofs.values(), key=weight, reverse=True)
        roof = dict(order[0])
        roof["chosen_by"] = ("the most ms per coded frame in the committed trace (all template "
                             "instances of the kernel)" if "trace" in roof else
                             "the most probed ms (no committed trace)")
        if len(order) > 1:
            roof["other"] = order[1]
    if not roofs:
        # no probe (speed 6, several ranks): the frame's full F4 evaluation
        # (round 0), from its HIP-event stage span
        dom = "rdo_candidates" if kernels["rdo_candidates"]["bytes"] > 0 else \
            max(kernels, key=lambda n: kernels[n]["ms"])
        kd = kernels[dom]
        avg_s = kd["ms"] / 1e3
        ach = kd["bytes"] / avg_s / 1e9
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                "avg_launch_ms": round(kd["ms"], 5),
                "algorithmic_bytes_per_launch": round(kd["bytes"]),
                "launch": "the frame's full evaluation (round 0), HIP events on its stream"}
        te = trace_entry(dom)
        if te and te.get("round0"):
            r0 = te["round0"]
            roof["trace"] = {"source": pj["source"], "git": pj["git"], "round0_avg_us": r0["avg_us"],
                             "frac_from_trace": round(kd["bytes"] / (r0["avg_us"] * 1e-6) / 1e9 /
                                                      HBM_PEAK_GBS, 5),
                             "live_over_trace_duration": round(kd["ms"] * 1e3 / r0["avg_us"], 3)}
            if r0.get("hbm_bytes_per_launch"):
                roof["traffic"] = {"bytes_per_launch": r0["hbm_bytes_per_launch"],
                                   "source": pj["source"], "git": pj["git"],
                                   "over_algorithmic": round(r0["hbm_bytes_per_launch"] / kd["bytes"], 3)}
    fps = args.steps / dt  # frames of the one stream

    emu = None
    n_emu = min(args.emulate_ranks, tiling["cols"] * tiling["rows"])  # one tile group per rank
    if rank == 0 and world == 1 and n_emu > 1:
        emu = emulate_ranks(n_emu, W, H, xdec, ydec, bd, nref, tiling, flags,
                            imp_window=imp_window, pj=pj)

    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the CPU codes the same frames: the GPU's inputs, downloaded
        inputs = [hip.get_input(i) for i in range(min(22 + imp_window, n_inputs))]
        if paired:
            eng.close()
        hip.close()  # the parity pass below builds a fresh GPU replay
        cpu, parity = cpu_baseline_and_parity(args, inputs, W, H, xdec, ydec, bd, nref,
                                              tiling, n_inputs, speed, flags, imp_window)

    if rank == 0:
        line = {
            "metric": "encoded frames/sec + Mpixels/sec, 4K 8-bit speed=10, 1/2/4/8 GPU vs host CPU",
            "value": round(fps, 3), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "u16" if bd > 8 else "u8", "data": "synthetic",
            "config": {"workload": f"{args.config} {bd}-bit "
                                   f"{'4:2:0' if xdec else '4:4:4'} speed={speed} hot-path replay of one "
                                   f"stream (BASELINE config {cfg_name}), "
                                   f"{tiling['cols']}x{tiling['rows']} tiles over {world} GPU(s), "
                                   f"{nref} refs, reorder-pyramid coding order"
                                   f"{'' if args.no_entropy else ', coefficients entropy-coded'}",
                       "width": W, "height": H, "refs": nref, "speed": speed,
                       "deblock": deblock, "cdef": cdef, "loop_restoration": lrf,
                       "tiles": [tiling["cols"], tiling["rows"]],
                       "parallelism": f"tile-groups{world}",
                       "frame_concurrency": (("levels 0/1 + 4g+1 on the primary, 4g+3 on a "
                                              "twin (2 instances)")
                                             if paired and isinstance(eng, RP.PairedReplay) else
                                             ("level 0 + 4g+1, level 1, 4g+3 on three instances "
                                              "(own streams and host threads, device events)")
                                             if paired else "serial"),
                       "candidates_per_sb": f"{4 * nref} inter modes x (skip, non-skip)",
                       **({"mv_stack": ("rav1e's find_mvrefs over the coded blocks, coding-order "
                                        "rounds" if args.mv_stack == "exact" else
                                        "stand-in: the neighbours' search MVs (A/B)")}
                          if speed == 10 else {}),
                       **({"partition": "64x64 .. 8x8 top-down NONE vs SPLIT, every level "
                                        "searched and scored"} if speed == 6 else {})},
            "mpix_per_s": round(fps * W * H / 1e6, 3),
            "inputs": {"residency": "every input frame is generated in HBM (rv_replay_synth_inputs) "
                                    "before the timed region; the timed region moves no pixels "
                                    "over PCIe",
                       "upload_bytes_per_frame": int(W * H * px + 2 * ((W + xdec) >> xdec) *
                                                     ((H + ydec) >> ydec) * px),
                       "note": "a streaming encoder would upload that many bytes per frame "
                               "(rv_replay_set_input; ~0.3 ms at 2160p 8-bit over a ~40 GB/s "
                               "host link), overlappable with the lookahead engine's W-frame "
                               "lead; not measured here"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity,
            "gpu_vs_cpu": round(fps / cpu["value"], 2) if cpu else None,
            "stage_ms": {n: round(float(v), 4) for n, v in zip(STAGES6 if speed == 6 else STAGES, ms)},
            "kernels_ms": {n: round(v["ms"], 4) for n, v in kernels.items()},
            **({"kernels_trace": _kernels_trace(pj)} if pj else {}),
            "full_search_path": "successive elimination" if sea else "exhaustive",
            "diamond_evals_per_frame": [round(ev_full / ev_frames, 1),
                                        round(ev_sub / ev_frames, 1)],
            "rdo_candidates_per_frame": {"single_ref": round(ns, 1), "compound": round(nc, 1),
                                         "variants": "skip + non-skip each",
                                         **({"levels": level_cands} if level_cands else {})},
            **({"mv_stacks": {
                "what": "speed 10: rav1e's find_mvrefs stacks (NEAREST / NEAR / GLOBAL candidates, "
                        "the search's rate predictors) in coding-order rounds: round 0 evaluates "
                        "every superblock, a later round the ones whose stacks changed",
                "rounds_per_frame": round(cnt[14] / max(1, cnt[16]), 3),
                "reevaluated_sb_per_frame": round(cnt[15] / max(1, cnt[16]), 2),
                "outer_passes_per_frame": round(cnt[17] / max(1, cnt[16]), 3) if len(cnt) > 17
                else None,
                "round_bound": "tws + 2 ths - 2 evaluation rounds per run (DESIGN.md §3)"}}
               if speed == 10 and len(cnt) > 16 else {}),
            "importances": ({
                "window": imp_window,
                "what": "compute_block_importances over rdo_lookahead_frames coded frames: every "
                        "frame's lookahead (F0 pyramids, F1, F2L / FL with their EPZS rounds) runs "
                        "that many frames ahead on a lookahead engine (own host thread, stream and "
                        "round ring), then the window's propagation (per-frame target lists, one "
                        "pass per frame and reference) and log2; the frame's RDO bias reads them",
                "stream": "unbounded: each frame's window reaches W frames past it, so the "
                          "engine's lookahead runs W frames ahead of the timed frames",
                "lookahead_frames": cnt[20] if len(cnt) > 20 else None,
                "lookahead_frames_in_timed_region": (la_cnt["t1"] - la_cnt["t0"]
                                                     if "t1" in la_cnt else None),
                "engine_lead_at_start": ("the window (W frames): no input declared ready before "
                                         "the timing" if ready else "not capped"),
                "lookahead_rounds_per_frame": round(cnt[18] / max(1, cnt[20]), 3)
                if len(cnt) > 20 else None,
                **({"ranks": "each rank's engine computes its tile group's lookahead part; the "
                             "parts are all-gathered over RCCL on the encode stream before the "
                             "frames whose window needs them, so every rank propagates over the "
                             "whole frame"} if world > 1 else {})} if imp_window else
                {"window": 0, "what": "importance 0 (bias 0.65)"}),
            "intra_per_frame": {"screened_superblocks": round(cnt[11] / ev_frames, 2),
                                "intra_winners": round(cnt[12] / ev_frames, 2),
                                "rounds": round(cnt[13] / ev_frames, 2),
                                "modes_per_screen": "13 predicted + SATD, 3 RDO x (chroma "
                                                    "mode, DC)"},
            **({"entropy": {
                "stage": "F8: coefficients of every coded frame (write_coeffs_lv_map) tokenized on "
                         "the GPU, range-coded on a host thread per replay instance beside the "
                         "next frames; inside the timed region",
                "frames": int(ent_stats[3]),
                "coefficient_bytes_per_frame": round(ent_stats[4] / max(1, ent_stats[3]), 1),
                "coefficient_kbit_per_frame": round(ent_stats[4] * 8 / 1e3 / max(1, ent_stats[3]), 3),
                "scope": "coefficient syntax only (no mode / MV / partition symbols, headers)"}}
               if ent else {}),
            **({"emulated_ranks": emu} if emu else {}),
        }
        print(json.dumps(line), flush=True)
    if paired:
        eng.close()
    hip.close()
    if comm:
        comm.close()
    group.close()


if __name__ == "__main__":
    main()
