"""altcorr at C3: the per-edge matrix-core kernel (edges in the window
group-by's target-frame order) against the LDS-staged kernel (its own
(frame, cell) binning included), HIP events over back-to-back launches.

  python scripts/bench_corr_stage.py [--reps 30] [--buffer 2048]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]

import torch  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--buffer", type=int, default=2048)
    ap.add_argument("--preset", default="dpvo_2k")
    args = ap.parse_args()
    import update_ops
    from dpvo.synthetic import steady_state_tracker
    slam = steady_state_tracker(args.preset, buffer=args.buffer, seed=0)
    with torch.no_grad():
        coords = slam.reproject()
        ctx, jslot, _, _, order = update_ops.window_group_by(
            slam.pg.ii, slam.pg.jj, slam.pg.kk, slam.M, slam.n - 64, slam.M * slam.pmem, slam.pmem,
            flag=slam._ba_status, jj_order=True)
        slam.cfg.STAGED_CORR = False
        ref = slam.corr(coords, slots=(ctx, jslot), order=order).clone()
        t_mfma = timeit(lambda: slam.corr(coords, slots=(ctx, jslot), order=order), args.reps)
        slam.cfg.STAGED_CORR = True
        got = slam.corr(coords, slots=(ctx, jslot)).clone()
        t_stage = timeit(lambda: slam.corr(coords, slots=(ctx, jslot)), args.reps)
    same = torch.equal(got.view(torch.int16), ref.view(torch.int16))
    # fallback share: the binned count from the workspace (offs[nb - 1]) is internal; restate the rule
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from test_gpu_corr_stage import binned_fraction
    frac = binned_fraction(coords.cpu(), ctx.cpu(), jslot.cpu(), slam.M * slam.pmem, slam.pmem)
    print(json.dumps({"edges": slam.pg.ii.numel(), "mfma_ms": round(t_mfma, 4), "staged_ms": round(t_stage, 4),
                      "speedup": round(t_mfma / t_stage, 3), "bit_identical": same,
                      "staged_fraction": round(frac, 4)}), flush=True)


if __name__ == "__main__":
    main()
