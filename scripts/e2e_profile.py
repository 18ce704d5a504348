"""Where an end-to-end frame's host time goes (bench.end_to_end's loop at C3).

  python scripts/e2e_profile.py [--frames 32] [--sync]

Wraps DPVO.__call__'s stages with host timers (perf_counter, no extra
synchronisation unless --sync, which synchronises after every stage so the
numbers become GPU+host time per stage) and prints the per-frame mean of each.
"""
import argparse
import json
import os
import sys
import time
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "wild-video-3d-reconstruction_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--buffer", type=int, default=2048)
    ap.add_argument("--sync", action="store_true")
    ap.add_argument("--graphed", action="store_true", help="cfg.GRAPH_UPDATE")
    args = ap.parse_args()
    import bench
    from dpvo.synthetic import image_stream, steady_state_tracker
    total = args.frames + args.warmup
    cfgd = bench.CONFIGS["C3"]
    over = dict(cfgd["overrides"])
    if args.graphed:
        over["GRAPH_UPDATE"] = True
    slam = steady_state_tracker(cfgd["preset"], buffer=args.buffer, n=args.buffer - 8 - total, seed=0,
                                iterations=cfgd["iterations"], **over)
    intr = torch.tensor([320.0, 320.0, 320.0, 240.0], device=slam.device)
    imgs = [img for _, img in image_stream(total, device=slam.device)]
    acc = defaultdict(float)
    on = [False]

    def wrap(obj, name, label):
        f = getattr(obj, name)

        def g(*a, **k):
            t = time.perf_counter()
            r = f(*a, **k)
            if args.sync:
                torch.cuda.synchronize()
            if on[0]:
                acc[label] += time.perf_counter() - t
            return r
        setattr(obj, name, g)

    wrap(slam.network.patchify, "forward", "patchify")
    wrap(slam, "append_factors", "append_factors")
    wrap(slam, "update", "update")
    wrap(slam, "remove_factors", "remove_factors")
    inner = slam.keyframe
    kept = [0, 0]

    def keyframe():
        drop = (kept[0] + kept[1]) % 2 == 0
        slam.cfg.KEYFRAME_THRESH = float("inf") if drop else -1.0
        n0 = slam.n
        t = time.perf_counter()
        inner()
        if args.sync:
            torch.cuda.synchronize()
        if on[0]:
            acc["keyframe (incl. remove_factors)"] += time.perf_counter() - t
        kept[int(slam.n == n0)] += 1
    slam.keyframe = keyframe
    t_first = slam.n
    with torch.no_grad():
        for k, img in enumerate(imgs):
            if k == args.warmup:
                torch.cuda.synchronize()
                on[0] = True
                t0 = time.perf_counter()
            slam(t_first + k, img, None, None, intr)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    per = {k: round(v / args.frames * 1e3, 3) for k, v in acc.items()}
    per["frame"] = round(dt / args.frames * 1e3, 3)
    per["other (prelude, edges)"] = round(per["frame"] - sum(v for k, v in per.items()
                                                              if k not in ("frame", "remove_factors")), 3)
    print(json.dumps({"sync": args.sync, "graphed": args.graphed, "ms_per_frame": per, "kept": kept}))


if __name__ == "__main__":
    main()
