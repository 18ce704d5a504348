"""Experiment: the per-edge matrix-core altcorr visiting the edges in
(target frame, 8x8 level-1 cell) order instead of the window group-by's
target-frame order -- does L1 / L2 locality between the concurrently
processed edges' boxes shorten it?  (order computed with torch here; timing
of the kernel only)"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import torch  # noqa: E402


def timeit(fn, reps=20):
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
    import cuda_corr
    import update_ops
    from dpvo import altcorr
    from dpvo.synthetic import steady_state_tracker
    slam = steady_state_tracker("dpvo_2k", buffer=2048, seed=0)
    res = {}
    with torch.no_grad():
        coords = slam.reproject()
        ctx, jslot, _, _, order = update_ops.window_group_by(
            slam.pg.ii, slam.pg.jj, slam.pg.kk, slam.M, slam.n - 64, slam.M * slam.pmem, slam.pmem,
            flag=slam._ba_status, jj_order=True)
        table = slam._gmap_table(mfma=True)
        run = lambda o: altcorr.corr_pyramid_mfma(table, slam.gmap.shape[1], slam.pyramid, coords, ctx, jslot, order=o)
        ref = run(order).clone()
        c = coords[0, :, :, 1, 1]
        cy = torch.div(torch.floor(c[:, 1]).long() + 1, 8, rounding_mode="floor").clamp(-1, 13) + 1
        cx = torch.div(torch.floor(c[:, 0]).long() + 1, 8, rounding_mode="floor").clamp(-1, 17) + 1
        for name, key in (("frame", jslot), ("frame_cell", jslot * 1000 + cy * 20 + cx),
                          ("frame_row_band", jslot * 1000 + cy * 20 + cx // 2)):
            o = torch.argsort(key, stable=True).int().contiguous()
            res[name] = round(timeit(lambda: run(o)), 4)
            assert torch.equal(run(o), ref)
        res["window_group_by_order"] = round(timeit(lambda: run(order)), 4)
        res["no_order"] = round(timeit(lambda: run(None)), 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
