#!/usr/bin/env python3
"""Per-me_range_scale stage times of the replay (development aid):
python tools/stage_scales.py [--config 1080p] [--flags N] -> one line per scale."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1080p")
    ap.add_argument("--flags", type=int, nargs="*", default=[0])
    ap.add_argument("--frames", type=int, default=24)
    args = ap.parse_args()
    import rav1e_amd as R
    from rav1e_amd import replay as RP
    from bench import CONFIGS
    R.lib()
    R.require_device(0)
    W, H, xdec, ydec, bd = CONFIGS[args.config]
    frames = [RP.synth_frame(W, H, t, xdec, ydec, bd) for t in range(3)]
    for fl in args.flags:
        hip = RP.HipReplay(W, H, xdec, ydec, bd, 2, flags=fl)
        for s, f in enumerate(frames):
            hip.set_frame(s, f)
        hip.set_timing(1, 1)
        for scale in (4, 2, 1):
            for _ in range(4):
                hip.frame(scale)
            hip.results()
            for _ in range(args.frames):
                hip.frame(scale)
            hip.results()
            ms = hip.stage_ms_sum(args.frames) / args.frames
            print(f"flags={fl} scale={scale} " +
                  " ".join(f"{v * 1e3:.1f}" for v in ms[:9]), flush=True)
        hip.close()


if __name__ == "__main__":
    main()
