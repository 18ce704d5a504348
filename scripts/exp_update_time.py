"""The update operator (DPVO.update's network call) and the whole update() at
C3, HIP events over back-to-back updates from one seeded steady state -- for
A/B runs of experiment builds (DPVO_HOT_LIB=exp/<name>/libdpvo_hot.so
DPVO_DIAG=1).  Prints the mean update() time and a digest of the state after
a fixed number of updates (equal digests = same bits).

  python scripts/exp_update_time.py [--reps 20] [--tag name]
"""
import argparse
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default=os.environ.get("DPVO_HOT_LIB", "product"))
    ap.add_argument("--preset", default="dpvo_2k")
    ap.add_argument("--buffer", type=int, default=2048)
    ap.add_argument("--set", action="append", default=[],
                    help="NAME=0|1: a class-level switch of dpvo.net.Update (e.g. FUSE_GRU_RES=0)")
    args = ap.parse_args()
    from dpvo.net import Update
    for kv in args.set:
        k, v = kv.split("=")
        assert hasattr(Update, k), k
        setattr(Update, k, bool(int(v)))
        args.tag += f" {k}={v}"
    from dpvo.synthetic import steady_state_tracker
    slam = steady_state_tracker(args.preset, buffer=args.buffer, seed=0)
    with torch.no_grad():
        for _ in range(3):
            slam.update()
        torch.cuda.synchronize()
        h = hashlib.sha256()
        for t in (slam.pg.poses_, slam.pg.patches_, slam.pg.net, slam.pg.target, slam.pg.weight):
            h.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())
        ts = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                slam.update()
            b.record()
            torch.cuda.synchronize()
            ts.append(round(a.elapsed_time(b) / args.reps, 4))
    print(json.dumps({"tag": args.tag, "edges": slam.pg.ii.numel(), "update_ms": ts,
                      "state_sha_after_3": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
