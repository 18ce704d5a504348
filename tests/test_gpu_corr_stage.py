"""The LDS-staged matrix-core correlation (csrc/corrstage.hip, DPVO.corr's
default path since round 5) against the per-edge matrix-core kernel
(csrc/corrmfma.hip), bit for bit.

Both compute every edge's row with the same arithmetic (the same MFMA
channel order, the same fp32 bilinear epilogue); the staged kernel only reads
the box pixels from an LDS copy of the edge's (target frame, level-1 cell)
region instead of from the feature maps.  So the bar is bit identity, on the
edge cases (integer, far-outside, saturating, widely spread, non-finite
coordinates, bad indices), on cells crowded past one pass of the workgroup's
waves, and on the whole C3 update (E = 95,424).  The accuracy of the rows
themselves against the oracle is tests/test_gpu_corr_mfma.py's."""
import numpy as np
import pytest
import torch

from test_gpu_altcorr import channel_last, dev, dpvo_sized_inputs

pytestmark = pytest.mark.gpu


def both(gmap, f1, f2, ii, jj, coords, out=None):
    import cuda_corr
    d = dev()
    table = cuda_corr.pack_mfma(gmap.to(d))
    pyr = [channel_last(f1.to(d)), channel_last(f2.to(d))]
    args = (table, gmap.shape[1], pyr, coords.to(d), ii.to(d), jj.to(d))
    ref = cuda_corr.forward_pyramid_mfma(*args)
    got = cuda_corr.forward_pyramid_staged(*args, out=out)
    torch.cuda.synchronize()
    return got, ref


def bits_equal(a, b):
    return np.array_equal(a.cpu().numpy().view(np.uint16), b.cpu().numpy().view(np.uint16))


def binned_fraction(coords, ii, jj, N1, N2, H=96, W=128, scales=(1.0, 4.0)):
    """The staged kernel's binning rule (cs_bin_kernel) restated in numpy:
    the fraction of edges whose level-1 box fits its cell's 17 x 17 region and
    whose level-2 box fits the 11 x 11 one."""
    c = coords[0].numpy().astype(np.float32)               # [E, 2, 3, 3]
    x, y = c[:, 0].reshape(len(c), -1), c[:, 1].reshape(len(c), -1)
    fin = (np.abs(x) < 1e6).all(1) & (np.abs(y) < 1e6).all(1)
    with np.errstate(invalid="ignore"):
        f = lambda v, s: np.floor(np.nan_to_num(v / np.float32(s))).astype(np.int64)
        fy, fx, gy, gx = f(y, scales[0]), f(x, scales[0]), f(y, scales[1]), f(x, scales[1])
    cy, cx = (fy.min(1) + 1) >> 3, (fx.min(1) + 1) >> 3
    ncy, ncx = (H + 7) // 8 + 2, (W + 7) // 8 + 2
    ok = fin & (fy.max(1) - fy.min(1) <= 4) & (fx.max(1) - fx.min(1) <= 4)
    ok &= (cy >= -1) & (cy < ncy - 1) & (cx >= -1) & (cx < ncx - 1)
    ok &= (fy.max(1) <= 8 * cy + 8) & (fx.max(1) <= 8 * cx + 8)
    ok &= (gy.min(1) >= 2 * cy - 1) & (gy.max(1) <= 2 * cy + 2) & (gx.min(1) >= 2 * cx - 1) & (gx.max(1) <= 2 * cx + 2)
    ok &= (ii.numpy() >= 0) & (ii.numpy() < N1) & (jj.numpy() >= 0) & (jj.numpy() < N2)
    return float(ok.mean())


@pytest.mark.parametrize("seed", [0, 1])
def test_staged_equals_mfma_with_edge_cases(seed):
    inp = dpvo_sized_inputs(seed)
    got, ref = both(*inp)
    assert bits_equal(got, ref)
    frac = binned_fraction(inp[5], inp[3], inp[4], 64, 6)
    assert 0.8 < frac < 1.0, frac          # most edges staged, the edge cases fall back


@pytest.mark.parametrize("spread", [1.4, 1.8, 2.3])
def test_staged_equals_mfma_wide_boxes(spread):
    inp = dpvo_sized_inputs(7, E=1200, spread=spread, edge_cases=False)
    got, ref = both(*inp)
    assert bits_equal(got, ref)


def test_staged_nonfinite_bad_indices_and_rows():
    gmap, f1, f2, ii, jj, coords = dpvo_sized_inputs(2, E=200, edge_cases=False)
    coords[0, :10, 0, 1, 1] = float("nan")
    coords[0, 10:20, 1, 0, 0] = float("inf")
    ii[20:30] = 10_000
    jj[30:40] = -1
    jj[40:45] = 6               # one past the ring
    buf = torch.zeros(200, 896, dtype=torch.float16, device=dev())
    got, ref = both(gmap, f1, f2, ii, jj, coords, out=buf[:, :882][None])
    assert torch.equal(buf[:, 882:], torch.zeros_like(buf[:, 882:]))   # pad columns untouched
    assert bits_equal(got, ref)
    assert np.all(got[0, 20:45].cpu().numpy() == 0)


def test_staged_crowded_cells_and_empty():
    """Hundreds of edges in a few cells (many passes of the 8 waves over one
    staged region, bins split between workgroups) and cells at the map's
    borders and corners (regions partly outside: zero pixels)."""
    g = torch.Generator().manual_seed(11)
    gmap, f1, f2, ii, jj, coords = dpvo_sized_inputs(3, E=3000, edge_cases=False)
    centres = torch.tensor([[3.5, 2.2], [60.3, 40.7], [126.4, 94.6], [0.2, 95.1], [127.9, 0.3]])
    pick = torch.randint(0, len(centres), (3000,), generator=g)
    off = torch.stack(torch.meshgrid(torch.arange(3.) - 1, torch.arange(3.) - 1, indexing="ij")[::-1], 0)
    c = centres[pick] + 0.3 * torch.rand(3000, 2, generator=g)
    coords = (c[:, :, None, None] + off[None] + 0.05 * torch.randn(3000, 2, 3, 3, generator=g))[None].contiguous()
    jj = torch.randint(0, 2, (3000,), generator=g)
    got, ref = both(gmap, f1, f2, ii, jj, coords)
    assert bits_equal(got, ref)
    import cuda_corr
    d = dev()
    e0 = cuda_corr.forward_pyramid_staged(cuda_corr.pack_mfma(gmap.to(d)), gmap.shape[1],
                                          [channel_last(f1.to(d)), channel_last(f2.to(d))], coords[:, :0].to(d),
                                          ii[:0].to(d), jj[:0].to(d))
    assert e0.shape == (1, 0, 882)


def test_tracker_corr_c3_staged_equals_mfma():
    """DPVO.corr at C3 (2048-KF buffer, n = 2040, E = 95,424) as update()
    calls it: the staged rows equal the per-edge kernel's on every edge, and
    nearly every edge is staged (the synthetic steady state)."""
    import cuda_corr
    import update_ops
    from dpvo.synthetic import steady_state_tracker
    slam = steady_state_tracker("dpvo_2k", buffer=2048, seed=4)
    E = slam.pg.ii.numel()
    assert E == 95424
    with torch.no_grad():
        coords = slam.reproject()
        ctx, jslot, _, _, order = update_ops.window_group_by(
            slam.pg.ii, slam.pg.jj, slam.pg.kk, slam.M, slam.n - 64, slam.M * slam.pmem, slam.pmem,
            flag=slam._ba_status, jj_order=True)
        slam.cfg.STAGED_CORR = False
        ref = slam.corr(coords, slots=(ctx, jslot), order=order).clone()
        slam.cfg.STAGED_CORR = True
        got = slam.corr(coords, slots=(ctx, jslot)).clone()
    torch.cuda.synchronize()
    assert bits_equal(got, ref)
    frac = binned_fraction(coords.cpu(), ctx.cpu(), jslot.cpu(), slam.M * slam.pmem, slam.pmem)
    print(f"C3: {100 * frac:.1f} % of the edges staged")
    assert frac > 0.9
    # and a second call reusing the cached workspace gives the same rows
    with torch.no_grad():
        again = slam.corr(coords, slots=(ctx, jslot)).clone()
    assert torch.equal(again, got)
    del cuda_corr
