"""Where the staged altcorr differs from the per-edge kernel (debug aid):
per edge class (staged / fallback), the differing edges, which level, how far."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_gpu_altcorr import dpvo_sized_inputs  # noqa: E402
from test_gpu_corr_stage import both  # noqa: E402


def rule(coords, ii, jj, N1, N2, H=96, W=128):
    c = coords[0].numpy().astype(np.float32)
    x, y = c[:, 0].reshape(len(c), -1), c[:, 1].reshape(len(c), -1)
    fin = (np.abs(x) < 1e6).all(1) & (np.abs(y) < 1e6).all(1)
    with np.errstate(invalid="ignore"):
        f = lambda v, s: np.floor(np.nan_to_num(v / np.float32(s))).astype(np.int64)
        fy, fx, gy, gx = f(y, 1), f(x, 1), f(y, 4), f(x, 4)
    cy, cx = (fy.min(1) + 1) >> 3, (fx.min(1) + 1) >> 3
    ok = fin & (fy.max(1) - fy.min(1) <= 4) & (fx.max(1) - fx.min(1) <= 4)
    ok &= (cy >= -1) & (cy < (H + 7) // 8 + 1) & (cx >= -1) & (cx < (W + 7) // 8 + 1)
    ok &= (fy.max(1) <= 8 * cy + 8) & (fx.max(1) <= 8 * cx + 8)
    ok &= (gy.min(1) >= 2 * cy - 1) & (gy.max(1) <= 2 * cy + 2) & (gx.min(1) >= 2 * cx - 1) & (gx.max(1) <= 2 * cx + 2)
    ok &= (ii.numpy() >= 0) & (ii.numpy() < N1) & (jj.numpy() >= 0) & (jj.numpy() < N2)
    return ok, cy, cx, fy, fx


for seed in (0, 1):
    inp = dpvo_sized_inputs(seed)
    got, ref = both(*inp)
    g, r = got[0].cpu().numpy(), ref[0].cpu().numpy()
    diff = (g.view(np.uint16) != r.view(np.uint16))
    bad = diff.any(1)
    ok, cy, cx, fy, fx = rule(inp[5], inp[3], inp[4], 64, 6)
    print(f"seed {seed}: E={len(bad)} staged={ok.sum()} bad staged={int((bad & ok).sum())} "
          f"bad fallback={int((bad & ~ok).sum())}")
    for e in np.nonzero(bad)[0][:6]:
        d = diff[e]
        lev1, lev2 = int(d[0::2].sum()), int(d[1::2].sum())
        err = np.abs(g[e].astype(np.float64) - r[e].astype(np.float64)).max()
        print(f"  edge {e}: staged={bool(ok[e])} cell=({cy[e]},{cx[e]}) fy[{fy[e].min()},{fy[e].max()}] "
              f"fx[{fx[e].min()},{fx[e].max()}] jj={int(inp[4][e])} lvl1 diffs {lev1} lvl2 diffs {lev2} "
              f"max {err:.3g} got0 {g[e][:4]} ref0 {r[e][:4]}")
