"""A/B of the fused update operator's switches at C3 (or C2): net.update as
DPVO.update calls it, HIP events over back-to-back calls, the variants
interleaved over several rounds on one box (box-to-box spread is ~3-5 %).

  python scripts/ab_update_op.py [--preset dpvo_2k --buffer 2048] [--flag FUSE_AGG_ADD]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="dpvo_2k")
    ap.add_argument("--buffer", type=int, default=2048)
    ap.add_argument("--flag", default="FUSE_AGG_ADD")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import update_ops
    from dpvo.net import Update
    from dpvo.synthetic import steady_state_tracker
    slam = steady_state_tracker(args.preset, buffer=args.buffer, seed=0)
    with torch.no_grad():
        coords = slam.reproject()
        ctx, jslot, kk_g, ij_g, order = update_ops.window_group_by(
            slam.pg.ii, slam.pg.jj, slam.pg.kk, slam.M, slam.n - 64, slam.M * slam.pmem, slam.pmem,
            flag=slam._ba_status, jj_order=True)
        with torch.autocast("cuda", enabled=True):
            corr = slam.corr(coords, slots=(ctx, jslot), order=order)

            def call():
                return slam.network.update(slam.pg.net, slam.imap, corr, None, slam.pg.ii, slam.pg.jj, slam.pg.kk,
                                           inp_idx=ctx, index_bounds=(slam.N * slam.M, slam.N), kk_groups=kk_g,
                                           ij_groups=ij_g)

            outs = {}
            times = {False: [], True: []}
            for r in range(args.rounds):
                for v in (False, True):
                    setattr(Update, args.flag, v)
                    for _ in range(2):
                        call()
                    torch.cuda.synchronize()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(args.reps):
                        net, (d, w, _) = call()
                    b.record()
                    torch.cuda.synchronize()
                    times[v].append(a.elapsed_time(b) / args.reps)
                    outs[v] = (net.clone(), d.clone(), w.clone())
    same = all(torch.equal(x, y) for x, y in zip(outs[False], outs[True]))
    print(json.dumps({"flag": args.flag, "edges": slam.pg.ii.numel(),
                      "off_ms": [round(t, 4) for t in times[False]], "on_ms": [round(t, 4) for t in times[True]],
                      "off_median": round(float(np.median(times[False])), 4),
                      "on_median": round(float(np.median(times[True])), 4), "bit_identical": same}), flush=True)


if __name__ == "__main__":
    main()
