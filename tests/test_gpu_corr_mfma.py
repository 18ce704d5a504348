"""The matrix-core correlation (csrc/corrmfma.hip, DPVO.corr's default path)
against the oracle.

It is NOT bit-identical to the reference: the reference accumulates the 128
channel products of every window pixel in fp16 (correlation_kernel.cu:121-131,
each add rounded to binary16) and rounds each bilinear op to fp16; this
kernel accumulates in fp32 on the matrix cores and rounds once.  The bar is
therefore accuracy against the oracle's exact arithmetic (fp16 inputs, fp64
accumulation, mode F16_ACC64): every output within the final fp16 rounding
of exact (2^-11 relative, plus 2e-5 absolute for the fp32 accumulation), and
the fp16-chain reference itself no closer to exact than this kernel (RMS).  The tracker-level effect on
poses / depths / points is bounded in tests/test_gpu_configs.py."""
import numpy as np
import pytest
import torch

from oracle import oracle
from test_gpu_altcorr import channel_last, dev, dpvo_sized_inputs

pytestmark = pytest.mark.gpu
RTOL, ATOL = 4.9e-4, 2e-5


def run_mfma(gmap, f1, f2, ii, jj, coords):
    import cuda_corr
    d = dev()
    table = cuda_corr.pack_mfma(gmap.to(d))
    out = cuda_corr.forward_pyramid_mfma(table, gmap.shape[1], [channel_last(f1.to(d)), channel_last(f2.to(d))],
                                         coords.to(d), ii.to(d), jj.to(d))
    return out.cpu().numpy()


def oracle_modes(gmap, f1, f2, ii, jj, coords):
    args = (gmap.numpy(), [f1.numpy(), f2.numpy()], coords.numpy(), ii.numpy(), jj.numpy())
    exact = oracle.corr_pyramid(*args, mode=oracle.F16_ACC64)
    ref16 = oracle.corr_pyramid(*args)
    return exact, ref16


def check(got, exact, ref16):
    g = got.astype(np.float64)
    fin = np.isfinite(exact)
    # non-finite exactly where the exact result is (NaN / inf coordinates)
    assert np.array_equal(np.isfinite(g), fin)
    err = np.abs(g[fin] - exact[fin])
    bad = err > RTOL * np.abs(exact[fin]) + ATOL
    assert not bad.any(), f"{bad.sum()} outputs off, worst {err.max():.3g}"
    rms = lambda x: float(np.sqrt(np.mean(x * x)))
    ref_err = rms(ref16.astype(np.float64)[fin] - exact[fin])
    assert rms(g[fin] - exact[fin]) <= ref_err + 1e-7
    return rms(g[fin] - exact[fin]), ref_err


@pytest.mark.parametrize("seed", [0, 1])
def test_mfma_corr_accuracy_with_edge_cases(seed):
    """Integer, far-outside, saturating and widely spread coordinates (the
    per-pixel window fallback) beside ordinary ones."""
    inp = dpvo_sized_inputs(seed)
    got = run_mfma(*inp)
    assert got.shape == (1, inp[-1].shape[1], 882)
    mine, ref = check(got, *oracle_modes(*inp))
    print(f"rms error vs exact: mfma {mine:.3g}, reference fp16 chain {ref:.3g}")


@pytest.mark.parametrize("spread", [1.4, 1.8, 2.3])
def test_mfma_corr_wide_boxes(spread):
    inp = dpvo_sized_inputs(7, E=1200, spread=spread, edge_cases=False)
    check(run_mfma(*inp), *oracle_modes(*inp))


def test_mfma_corr_nonfinite_and_bad_indices():
    gmap, f1, f2, ii, jj, coords = dpvo_sized_inputs(2, E=200, edge_cases=False)
    coords[0, :10, 0, 1, 1] = float("nan")
    coords[0, 10:20, 1, 0, 0] = float("inf")
    ii[20:30] = 10_000          # patch index outside the ring: zero features
    jj[30:40] = -1              # frame index outside the ring: zero map
    got = run_mfma(gmap, f1, f2, ii, jj, coords)
    exact, ref16 = oracle_modes(gmap, f1, f2, ii, jj, coords)
    assert np.all(got[0, 20:40] == 0) and np.all(exact[0, 20:40] == 0)
    check(got, exact, ref16)


def test_mfma_corr_empty_and_strided_rows():
    import cuda_corr
    d = dev()
    gmap, f1, f2, ii, jj, coords = dpvo_sized_inputs(4, E=300, edge_cases=False)
    table = cuda_corr.pack_mfma(gmap.to(d))
    buf = torch.zeros(300, 896, dtype=torch.float16, device=d)
    out = cuda_corr.forward_pyramid_mfma(table, gmap.shape[1], [channel_last(f1.to(d)), channel_last(f2.to(d))],
                                         coords.to(d), ii.to(d), jj.to(d), out=buf[:, :882][None])
    assert torch.equal(buf[:, 882:], torch.zeros_like(buf[:, 882:]))   # pad columns untouched
    ref = run_mfma(gmap, f1, f2, ii, jj, coords)
    assert np.array_equal(out.cpu().numpy(), ref)
    e0 = cuda_corr.forward_pyramid_mfma(table, gmap.shape[1], [channel_last(f1.to(d)), channel_last(f2.to(d))],
                                        coords[:, :0].to(d), ii[:0].to(d), jj[:0].to(d))
    assert e0.shape == (1, 0, 882)


def test_tracker_corr_mfma_vs_exact_kernel():
    """DPVO.corr at C3 size (E = 95,424): the default matrix-core path against
    the bit-exact fp16-chain kernel (cfg.EXACT_CORR), on every edge."""
    from dpvo.synthetic import steady_state_tracker
    slam = steady_state_tracker("dpvo_2k", buffer=72, seed=3)
    with torch.no_grad():
        coords = slam.reproject()
        fast = slam.corr(coords).float().clone()
        slam.cfg.EXACT_CORR = True
        exact16 = slam.corr(coords).float().clone()
        slam.cfg.EXACT_CORR = False
    d = (fast - exact16).abs()
    scale = exact16.abs().mean().item()
    # the two differ by the reference's fp16 accumulation error: a few fp16 ulps
    assert d.max().item() < 0.1, d.max().item()
    assert d.mean().item() < 0.02 * scale


def test_edge_order_is_a_grouped_permutation_and_changes_nothing():
    """cuda_corr.edge_order(jj) groups the edges by target frame (a counting
    sort); visiting the edges in that order gives the same rows bit for bit."""
    import cuda_corr
    d = dev()
    gmap, f1, f2, ii, jj, coords = dpvo_sized_inputs(5, E=2000)
    jj[:7] = 99     # outside the ring: grouped last
    order = cuda_corr.edge_order(jj.to(d), 6)
    o = order.cpu().numpy()
    assert np.array_equal(np.sort(o), np.arange(2000))
    keys = np.where(jj.numpy() < 6, jj.numpy(), 6)[o]
    assert np.all(np.diff(keys) >= 0)
    table = cuda_corr.pack_mfma(gmap.to(d))
    args = (table, gmap.shape[1], [channel_last(f1.to(d)), channel_last(f2.to(d))], coords.to(d), ii.to(d), jj.to(d))
    a = cuda_corr.forward_pyramid_mfma(*args)
    b = cuda_corr.forward_pyramid_mfma(*args, order=order)
    assert torch.equal(a, b)


def test_tracker_corr_c3_window_order_vs_oracle_exact():
    """DPVO.corr at C3 (2048-KF buffer, n = 2040, E = 95,424) exactly as
    update() calls it -- ring slots and the visiting order from the per-update
    window group-by (dpvo_window_group_by, jj_order) -- against the oracle's
    exact mode (fp16 inputs, fp64 sums) on a 480-edge sample, at the
    small-size bound: every output within the final fp16 rounding, RMS no
    worse than the reference's fp16 chain."""
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
        corr = slam.corr(coords, slots=(ctx, jslot), order=order)
    torch.cuda.synchronize()
    assert int(slam._ba_status.item()) == 0
    o = order.cpu().numpy()
    assert np.array_equal(np.sort(o), np.arange(E))
    sel = np.unique(np.concatenate([np.linspace(0, E - 1, 400).astype(np.int64), o[:40], o[-40:]]))
    c = coords[0].cpu().numpy()[sel][None]
    fm = [slam.fmap1_.contiguous().cpu().numpy(), slam.fmap2_.contiguous().cpu().numpy()]
    args = (slam.gmap.cpu().numpy(), fm, c, ctx.cpu().numpy()[sel], jslot.cpu().numpy()[sel])
    exact = oracle.corr_pyramid(*args, mode=oracle.F16_ACC64)
    ref16 = oracle.corr_pyramid(*args)
    mine, ref = check(corr[0].cpu().numpy()[sel][None], exact, ref16)
    print(f"C3 tracker order, {len(sel)} edges: rms vs exact {mine:.3g} (reference fp16 chain {ref:.3g})")
