#!/usr/bin/env python3
"""bench.py -- encode hot-path replay throughput on MI355X.

Metric (BASELINE.json): encoded frames/sec (+ Mpixels/sec) of the speed-10
hot path, frames resident in HBM, vs the host CPU running the same schedule.
A "step" = one frame of the replay driver (DESIGN.md "Replay driver"):
F0 downsample, F1 1/4-res full search, F2 1/2-res diamond, F3 full-res
diamond + sub-pel, F4 RDO candidates (MC, diff+fwd DCT, coefficient
stand-in, inverse DCT + add, distortion), F5 8x8 importance SATD.
Frames cycle through the reorder pyramid's me_range_scale (4, 2, 1, 1).

N = 1: the configuration BASELINE.json's metric is quoted on -- 4K (2160p)
8-bit 4:2:0 speed 10, one tile on one GPU (it fits one GPU; --config picks
the other shapes of `configs`, e.g. 1080p = configs[1]).
N > 1 (torch.distributed.run, one process per GPU): every rank runs its own
2160p tile stream (rav1e_amd/ranks.py) -- tiles are independent units in
the replay, so there is no data-path collective; `value` = frames of all
ranks / max-over-ranks time ("scaling": "weak").  torch.distributed (gloo)
carries only the barrier and the max-time reduction.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {  # name: (width, height, xdec, ydec, bit_depth)
    "360p": (640, 360, 1, 1, 8),
    "1080p": (1920, 1080, 1, 1, 8),
    "2160p": (3840, 2160, 1, 1, 8),
    "2160p10": (3840, 2160, 1, 1, 10),
    "2160p444": (3840, 2160, 0, 0, 8),
}
TIMING_STRIDE = 4  # in GOPs
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: 8.0 TB/s spec
# v_sad_u8 issue peak: a wave64 VALU op takes 4 cycles on a SIMD (64 lanes
# per CU-cycle over 4 SIMDs; tools/ubench/valu_rates.hip measures 0.87 of
# it), 4 |a-b| per lane-op for u8, 2 for v_sad_u16
SAD_PEAK_PX = 256 * 64 * 2.4e9 * 4
VALU_PEAK_GIPS = 256 * 4 * 2.4 / 4  # G wave64 VALU instructions/s


def coarse_windows(W, H, R, scale, tile=(0, 0, 0, 0)):
    """(nx, ny) of every F1 job: estimate_motion_ss4's window
    (src/me.rs:1023-1075), as the replay builds it."""
    w_in_b, h_in_b = 2 * ((W + 7) >> 3), 2 * ((H + 7) >> 3)
    sbc, sbr = (W + 63) // 64, (H + 63) // 64
    tx0, ty0, tw, th = tile
    tw, th = tw or sbc - tx0, th or sbr - ty0
    vis_w = min(W - tx0 * 64, tw * 64)
    vis_h = min(H - ty0 * 64, th * 64)
    mi_w, mi_h = vis_w >> 2, vis_h >> 2

    def tdiv8(v):
        return int(v / 8)
    out = []
    for sb in range(tw * th):
        bx, by = (sb % tw) * 16, (sb // tw) * 16
        bx, by = max(min(bx, mi_w - 16), 0), max(min(by, mi_h - 16), 0)
        fbx, fby = bx + tx0 * 16, by + ty0 * 16
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
    "full_search_exhaustive": "fs16_kernel<{px}>",
    "diamond_fullpel_64": "ds_fast_kernel<{px}, 64, 64, false>",
    "diamond_subpel_64": "ds_fast_kernel<{px}, 64, 64, true>",
    "rdo_candidates": "rdo_quad_kernel<{px}>",
    "rdo_candidates_zero_mv": "rdo_quad_kernel<{px}>",
}


def measured_traffic(args, kernel, bd):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    passes (profiles/traffic_<config>.json: 2 x FETCH_SIZE + WRITE_SIZE, see
    tools/prof_summary.py), for the workload it was measured on; None
    otherwise."""
    path = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if args.refs != 2 or not os.path.exists(path):
        return None
    with open(path) as f:
        tj = json.load(f)
    if kernel == "full_search" and args.exhaustive_fs:
        kernel = "full_search_exhaustive"
    want = ROCPROF_NAMES.get(kernel, "?").format(px="unsigned short" if bd > 8 else "unsigned char",
                                                 pxs="u16" if bd > 8 else "u8")
    for name, v in tj["kernels"].items():
        if want in name:
            return {"bytes_per_launch": round(v["hbm_bytes"]), "source": tj["source"],
                    "git": tj["git"]}
    return None


def measured_valu(args, kernel, bd):
    """Wave64 VALU instructions per launch of `kernel` (SQ_INSTS_VALU) from the
    committed rocprofv3 SQ counter pass profiles/valu_<config>.json
    (tools/pmc_json.py); None when the workload has no committed pass."""
    path = os.path.join(ROOT, "profiles", f"valu_{args.config}.json")
    if args.refs != 2 or not os.path.exists(path):
        return None
    with open(path) as f:
        tj = json.load(f)
    if kernel == "full_search" and args.exhaustive_fs:
        kernel = "full_search_exhaustive"
    want = ROCPROF_NAMES.get(kernel, "?").format(px="unsigned short" if bd > 8 else "unsigned char",
                                                 pxs="u16" if bd > 8 else "u8")
    for name, v in tj["kernels"].items():
        if want in name:
            return v["SQ_INSTS_VALU"], tj
    return None


def timed_run(engine, group, steps, warmup, scales=None, sync=None):
    """W untimed frames, then exactly K timed frames bracketed by a barrier
    and a device sync on both sides; returns (max-over-ranks seconds, result
    words of the last frame).  `engine` is a HipReplay (the product) or, in
    the multi-rank CPU tests, the oracle's CpuReplay."""
    from rav1e_amd import replay as RP
    scales = scales or RP.GOP_SCALES
    for i in range(warmup):
        engine.frame(scales[i % len(scales)])
    if warmup:
        engine.results()  # drains the stream
    group.barrier()
    if sync:
        sync()
    t0 = time.perf_counter()
    for i in range(steps):
        engine.frame(scales[(warmup + i) % len(scales)])
    if sync:
        sync()  # device-wide: every frame on every stream has finished
    t1 = time.perf_counter()
    group.barrier()
    # the verification checksums are not part of a frame: outside the timing
    words = engine.results()
    return group.max(t1 - t0), words


def cpu_baseline_and_parity(args, frames, W, H, xdec, ydec, bd, nref, scales):
    """The CPU baseline and the full-size parity check, from one CPU run.

    The CPU replay (oracle/orc_replay.c: the same schedule over the oracle's
    restatements; the build for this host's ISA level) runs frames 0..n-1 of
    the bench's workload on every host thread this process may use, timed,
    keeping each frame's result words.  A fresh GPU replay then runs the same
    n frames and its words must equal the CPU's, frame by frame: the bench's
    own full-size bit-exactness check.  A bounded 1-thread sample (the first
    superblocks of one GOP) is timed beside it."""
    import rav1e_amd as R
    from rav1e_amd import replay as RP
    from tests import oracle_lib as O  # the checker / CPU baseline only
    L, isa = O.baseline_lib()
    threads = O.cpu_share()
    c = O.CpuReplay(W, H, xdec, ydec, bd, nref, threads=threads, L=L)
    for s, f in enumerate(frames):
        c.set_frame(s, f)
    cpu_words = []
    n, tc0 = 0, time.perf_counter()
    while n < len(scales) or (time.perf_counter() - tc0 < args.cpu_seconds and n < 16):
        c.frame(scales[n % len(scales)])
        n += 1
        cpu_words.append(c.results())  # a memcpy; kept inside the timing
    tc = time.perf_counter() - tc0
    c.close()
    # 1 thread: the first 1/8 of the superblocks of one GOP
    nsb = ((W + 63) // 64) * ((H + 63) // 64)
    lim = max(1, nsb // 8)
    c1 = O.CpuReplay(W, H, xdec, ydec, bd, nref, threads=1, L=L)
    for s, f in enumerate(frames):
        c1.set_frame(s, f)
    t1 = time.perf_counter()
    for i in range(len(scales)):
        c1.frame(scales[i], lim)
    t1 = time.perf_counter() - t1
    c1.close()
    fps1 = len(scales) * (lim / nsb) / t1
    cpu = {"value": round(n / tc, 4), "unit": "frames/s", "cores": threads, "kind": "port",
           "isa": isa,
           "sample": f"{n} full {args.config} frames (scales {[scales[i % len(scales)] for i in range(n)]}) "
                     f"of the same replay schedule, oracle/orc_replay.c -O3 -march={isa} on "
                     f"{threads} host threads",
           "mpix_per_s": round(n / tc * W * H / 1e6, 3),
           "one_thread": {"value": round(fps1, 5), "unit": "frames/s",
                          "sample": f"first {lim} of {nsb} superblocks of each frame of one GOP "
                                    f"(scales {list(scales)}), scaled to whole frames"}}
    # the GPU replay over the same frames, word for word
    g = RP.HipReplay(W, H, xdec, ydec, bd, nref)
    for s, f in enumerate(frames):
        g.set_frame(s, f)
    bad = []
    for i in range(n):
        g.frame(scales[i % len(scales)])
        gw = g.results()
        d = np.nonzero(gw != cpu_words[i])[0]
        if d.size:
            bad.append({"frame": i, "n_diff": int(d.size), "first": int(d[0])})
    g.close()
    R._check(R.lib().rv_device_sync(), "rv_device_sync")
    parity = {"frames": n, "words": int(sum(w.size for w in cpu_words)),
              "bit_exact": not bad, "vs": "oracle/orc_replay.c (CPU replay)"}
    if bad:
        parity["mismatches"] = bad[:8]
    return cpu, parity


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--config", default="2160p", choices=sorted(CONFIGS))
    ap.add_argument("--refs", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--split-rdo", action="store_true",
                    help="F4 luma and chroma candidate kernels on two concurrent streams")
    ap.add_argument("--side-rdo", action="store_true",
                    help="zero-MV RDO candidates on a second stream, concurrent with F0-F3")
    ap.add_argument("--exhaustive-fs", action="store_true",
                    help="F1 coarse search without successive elimination (same results)")
    args = ap.parse_args()

    import rav1e_amd as R  # load the HIP library before anything else
    from rav1e_amd import replay as RP
    from rav1e_amd.ranks import RankGroup, rank_info
    R.lib()
    info = rank_info()
    rank, world = info.rank, info.world
    group = RankGroup(info)
    R.require_device(info.local_rank % max(1, R.lib().rv_device_count()))

    W, H, xdec, ydec, bd = CONFIGS[args.config]
    nref = args.refs
    frames = [RP.synth_frame(W, H, info.frame_offset + t, xdec, ydec, bd) for t in range(nref + 1)]
    hip = RP.HipReplay(W, H, xdec, ydec, bd, nref,
                       flags=(RP.RV_REPLAY_SIDE_RDO if args.side_rdo else 0) |
                       (RP.RV_REPLAY_SPLIT_RDO if args.split_rdo else 0) |
                       (RP.RV_REPLAY_EXHAUSTIVE_FS if args.exhaustive_fs else 0))
    sea = bd <= 10 and not args.exhaustive_fs  # the replay's F1 path
    for s, f in enumerate(frames):
        hip.set_frame(s, f)
    scales = RP.GOP_SCALES
    # HIP events on a sample of frames: every TIMING_STRIDE-th GOP records
    # them (whole GOPs, so every me_range_scale is equally represented)
    gop = len(scales)
    hip.set_timing(TIMING_STRIDE, gop)
    dt, words = timed_run(hip, group, args.steps, args.warmup, scales, sync=lambda: R._check(R.lib().rv_device_sync(), "rv_device_sync"))

    # per-kernel times over the instrumented frames of the timed region
    k = min(sum(1 for f in range(args.warmup, args.warmup + args.steps)
                if (f // gop) % TIMING_STRIDE == 0), 64)
    k = max(k, 1)
    ms = hip.stage_ms_sum(k) / k  # per frame
    ev_full, ev_sub, ev_frames = (int(v) for v in hip.counters())
    ev_frames = max(1, ev_frames)
    nsb = ((W + 63) // 64) * ((H + 63) // 64)
    px = 2 if bd > 8 else 1
    # algorithmic bytes per frame of each kernel class; the
    # SEA search also reads the box-sum tables: per 4-wide x 8-tall tile of
    # candidates, 20 rows of 16 B (paired u32 4x8 sums, rv_me.hip)
    fs_bytes = sum(sum((nx + 15) * (ny + 15) * px + 256 * px + 56 +
                       (((nx + 3) // 4) * ((ny + 7) // 8) * 20 * 16 if sea else 0)
                       for nx, ny in coarse_windows(W, H, nref, s)) for s in scales) / 4.0
    fs_ops = sum(sum(nx * ny * 256 for nx, ny in coarse_windows(W, H, nref, s))
                 for s in scales) / 4.0
    nj = nsb * nref
    nctx = nsb * 2 * nref
    cw, ch = 64 >> xdec, 64 >> ydec
    ntx_c = (cw // 32) * (ch // 32)
    csub = (cw // (min(cw, 8) >> xdec)) * (ch // (min(ch, 8) >> ydec))
    rdo_bytes = float(nctx * (71 * 71 * px + 64 * 64 * px + 4 * 32 * 32 + 64 * 64 * px +
                              64 * 40 + 16 + 24) +
                      2 * nctx * ((cw + 7) * (ch + 7) * px + 2 * cw * ch * px +
                                  4 * ntx_c * 32 * 32 + 8 * csub + 16 + 24 * ntx_c))
    kernels = {
        "full_search": dict(ms=float(ms[1]), launches=1, bytes=fs_bytes, sad_px=fs_ops),
        "diamond_fullpel_64": dict(ms=float(ms[6]), launches=1,
                                   bytes=nj * (64 * 64 * px + 80) +
                                   ev_full / ev_frames * 64 * 64 * px),
        "diamond_subpel_64": dict(ms=float(ms[7]), launches=1,
                                  bytes=nj * (64 * 64 * px + 80) +
                                  ev_sub / ev_frames * 71 * 71 * px),
        # F4: one fused launch over every candidate; with --side-rdo two launches
        # (sub-pel-MV candidates on the replay stream, zero-MV candidates on a
        # second stream concurrent with F0-F3), each half of the candidates
        "rdo_candidates": dict(ms=float(ms[8]), launches=1,
                               bytes=rdo_bytes / 2 if args.side_rdo else rdo_bytes),
    }
    if args.side_rdo:
        kernels["rdo_candidates_zero_mv"] = dict(ms=float(ms[9]), launches=1, bytes=rdo_bytes / 2)
    dom = max(kernels, key=lambda n: kernels[n]["ms"])
    kd = kernels[dom]
    launch_s = kd["ms"] / 1e3 / kd["launches"]
    ach = kd["bytes"] / kd["launches"] / launch_s / 1e9
    roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5),
            "traffic": measured_traffic(args, dom, bd),
            "avg_launch_ms": round(kd["ms"] / kd["launches"], 5),
            "algorithmic_bytes_per_launch": round(kd["bytes"] / kd["launches"])}
    mv = measured_valu(args, dom, bd)
    if mv:
        # VALU issue roofline: one wave64 VALU instruction per 4 cycles per
        # SIMD (1024 SIMDs at 2.4 GHz); instructions per launch from the
        # committed SQ_INSTS_VALU pass, time from this run's HIP events
        achv = mv[0] / launch_s / 1e9
        roof["valu"] = {"achieved": round(achv, 1), "peak": VALU_PEAK_GIPS,
                        "unit": "G wave64 VALU instr/s", "frac": round(achv / VALU_PEAK_GIPS, 4),
                        "insts_per_launch": round(mv[0]), "source": mv[1]["source"],
                        "git": mv[1]["git"]}
    if dom == "full_search" and not sea:
        achv = kd["sad_px"] / (kd["ms"] / 1e3) / 1e12
        peak = SAD_PEAK_PX / (2 if bd > 8 else 1)
        roof["valu"] = {"achieved": round(achv, 3), "peak": round(peak / 1e12, 1),
                        "unit": "T |a-b|/s (v_sad_u8 / v_sad_u16)",
                        "frac": round(achv * 1e12 / peak, 4)}
    fps = world * args.steps / dt

    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        hip.close()  # the parity pass below builds a fresh GPU replay
        cpu, parity = cpu_baseline_and_parity(args, frames, W, H, xdec, ydec, bd, nref, scales)

    if rank == 0:
        line = {
            "metric": "encoded frames/sec + Mpixels/sec, 4K 8-bit speed=10, 1/2/4/8 GPU vs host CPU",
            "value": round(fps, 3), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u16" if bd > 8 else "u8", "data": "synthetic",
            "config": {"workload": f"{args.config} {bd}-bit "
                                   f"{'4:2:0' if xdec else '4:4:4'} speed=10 hot-path replay, "
                                   f"1 tile per GPU, {nref} refs, GOP scales (4,2,1,1)",
                       "width": W, "height": H, "refs": nref, "parallelism": f"tiles{world}"},
            "mpix_per_s": round(fps * W * H / 1e6, 3),
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity,
            "gpu_vs_cpu": round(fps / cpu["value"], 2) if cpu else None,
            "stage_ms": {n: round(float(v), 4) for n, v in
                         zip(["F0_downsample", "F1_full_search", "F2_diamond_half",
                              "F3_diamond_full_subpel", "F4_rdo", "F5_importance_satd"], ms[:6])},
            "kernels_ms": {n: round(v["ms"], 4) for n, v in kernels.items()},
            "full_search_path": "successive elimination" if sea else "exhaustive",
            "diamond_evals_per_frame": [round(ev_full / ev_frames, 1),
                                        round(ev_sub / ev_frames, 1)],
            "checksum": int(words[-3]) & 0xFFFFFFFF,
        }
        print(json.dumps(line), flush=True)
    hip.close()
    group.close()


if __name__ == "__main__":
    main()
