"""altcorr (the per-edge matrix-core kernel, window group-by order) at C3,
HIP events over back-to-back launches -- for A/B runs of experiment builds
(DPVO_HOT_LIB=exp/<name>/libdpvo_hot.so DPVO_DIAG=1).

  python scripts/exp_corr_time.py [--reps 40] [--tag name]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--tag", default=os.environ.get("DPVO_HOT_LIB", "product"))
    ap.add_argument("--preset", default="dpvo_2k")
    ap.add_argument("--buffer", type=int, default=2048)
    args = ap.parse_args()
    import update_ops
    from dpvo.synthetic import steady_state_tracker
    slam = steady_state_tracker(args.preset, buffer=args.buffer, seed=0)
    with torch.no_grad():
        coords = slam.reproject()
        ctx, jslot, _, _, order = update_ops.window_group_by(
            slam.pg.ii, slam.pg.jj, slam.pg.kk, slam.M, slam.n - 64, slam.M * slam.pmem, slam.pmem,
            flag=slam._ba_status, jj_order=True)
        fn = lambda: slam.corr(coords, slots=(ctx, jslot), order=order)  # noqa: E731
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / args.reps)
        out = fn()
        torch.cuda.synchronize()
    import hashlib
    digest = hashlib.sha256(out.contiguous().view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"tag": args.tag, "edges": slam.pg.ii.numel(), "corr_ms": [round(t, 4) for t in ts],
                      "out_sha": digest}), flush=True)


if __name__ == "__main__":
    main()
