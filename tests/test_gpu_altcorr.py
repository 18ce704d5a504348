"""altcorr on the GPU (through the C ABI) vs the oracle / golden vectors.

Bar: bit-exact.  The reference accumulates in c10::Half with per-op
rounding; the HIP kernel emulates that exactly, so every fp16 output bit must
match the oracle (which itself matches the torch-f16 restatement bitwise).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import oracle

pytestmark = pytest.mark.gpu


def dev():
    return torch.device("cuda:0")


def channel_last(t):
    """Same logical NCHW tensor, channel-contiguous storage (the fast path)."""
    return t.permute(0, 1, 3, 4, 2).contiguous().permute(0, 1, 4, 2, 3)


def bits(a):
    return np.asarray(a).view(np.uint16)


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLDEN, "altcorr_ref.npz"))


@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
@pytest.mark.parametrize("level", [1, 2])
def test_forward_golden(gold, layout, level):
    import cuda_corr
    d = dev()
    g = torch.from_numpy(gold["gmap"]).view(torch.float16).to(d)
    f = torch.from_numpy(gold["fmap1" if level == 1 else "fmap2"]).view(torch.float16).to(d)
    if layout == "nhwc":
        f = channel_last(f)
    c = torch.from_numpy(gold["coords"]).to(d) / (1 if level == 1 else 4)
    out, = cuda_corr.forward(g, f, c, torch.from_numpy(gold["ii"]).to(d), torch.from_numpy(gold["jj"]).to(d), 3)
    assert out.shape == (1, 48, 7, 7, 3, 3)
    ref = gold["corr_l1" if level == 1 else "corr_l2"]
    assert np.array_equal(bits(out.contiguous().cpu().numpy()), bits(ref))


@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
def test_pyramid_golden(gold, layout):
    import cuda_corr
    d = dev()
    g = torch.from_numpy(gold["gmap"]).view(torch.float16).to(d)
    f1 = torch.from_numpy(gold["fmap1"]).view(torch.float16).to(d)
    f2 = torch.from_numpy(gold["fmap2"]).view(torch.float16).to(d)
    if layout == "nhwc":
        f1, f2 = channel_last(f1), channel_last(f2)
    c = torch.from_numpy(gold["coords"]).to(d)
    out = cuda_corr.forward_pyramid(g, [f1, f2], c, torch.from_numpy(gold["ii"]).to(d),
                                    torch.from_numpy(gold["jj"]).to(d), 3, [1, 4])
    assert np.array_equal(bits(out.cpu().numpy()), bits(gold["corr_stacked"]))


def test_odd_shapes_generic_path(gold):
    """radius 1, 5x5 patches, C=40, batch 2: the generic kernel."""
    import cuda_corr
    d = dev()
    g = torch.from_numpy(gold["b_gmap"]).view(torch.float16).to(d)
    f = torch.from_numpy(gold["b_fmap"]).view(torch.float16).to(d)
    out, = cuda_corr.forward(g, f, torch.from_numpy(gold["b_coords"]).to(d), torch.from_numpy(gold["b_ii"]).to(d),
                             torch.from_numpy(gold["b_jj"]).to(d), 1)
    assert np.array_equal(bits(out.contiguous().cpu().numpy()), bits(gold["b_corr"]))


def dpvo_sized_inputs(seed, E=1500, spread=1.0, edge_cases=True):
    """DPVO-shaped: C=128, 96x128 level-1 map, 3x3 patches, coords from a
    patch-grid + noise; includes out-of-image, far-away, integer and widely
    spread (non-shared-box) coordinates."""
    g = torch.Generator().manual_seed(seed)
    N1, C, N2, H, W = 64, 128, 6, 96, 128
    gmap = (0.25 * torch.randn(1, N1, C, 3, 3, generator=g)).half()
    f1 = (0.25 * torch.randn(1, N2, C, H, W, generator=g)).half()
    f2 = torch.nn.functional.avg_pool2d(f1[0].float(), 4, 4).half()[None]
    ii = torch.randint(0, N1, (E,), generator=g)
    jj = torch.randint(0, N2, (E,), generator=g)
    base = torch.stack([torch.rand(E, generator=g) * (W + 20) - 10, torch.rand(E, generator=g) * (H + 20) - 10], -1)
    off = torch.stack(torch.meshgrid(torch.arange(3.) - 1, torch.arange(3.) - 1, indexing="ij")[::-1], 0)
    coords = base[:, :, None, None] + spread * off[None] + 0.2 * torch.randn(E, 2, 3, 3, generator=g)
    if edge_cases:
        coords[:20] = torch.floor(coords[:20])                       # integer coordinates
        coords[20:40] = coords[20:40] * 4.0                          # wide spread -> fallback windows
        coords[40:50] = coords[40:50] + 1e6                          # far outside, saturating floor
        coords[50:60] = -coords[50:60] - 1e4
    return gmap, f1, f2, ii, jj, coords[None].float().contiguous()


@pytest.mark.parametrize("seed", [0, 1])
def test_pyramid_dpvo_sized_bitexact(seed):
    import cuda_corr
    d = dev()
    gmap, f1, f2, ii, jj, coords = dpvo_sized_inputs(seed)
    out = cuda_corr.forward_pyramid(gmap.to(d), [channel_last(f1.to(d)), channel_last(f2.to(d))], coords.to(d),
                                    ii.to(d), jj.to(d), 3, [1, 4])
    ref = oracle.corr_pyramid(gmap.numpy(), [f1.numpy(), f2.numpy()], coords.numpy(), ii.numpy(), jj.numpy())
    got = bits(out.cpu().numpy())
    assert got.shape == ref.shape == (1, coords.shape[1], 882)
    assert np.array_equal(got, bits(ref))


@pytest.mark.parametrize("spread", [1.4, 1.8, 2.3])
def test_pyramid_wide_boxes_bitexact(spread):
    """Scaled patches (perspective between distant frames): floor spreads of
    3-4 px take the 11x11 / 12x12 shared box, wider ones the per-pixel windows."""
    import cuda_corr
    d = dev()
    gmap, f1, f2, ii, jj, coords = dpvo_sized_inputs(7, E=1200, spread=spread, edge_cases=False)
    out = cuda_corr.forward_pyramid(gmap.to(d), [channel_last(f1.to(d)), channel_last(f2.to(d))], coords.to(d),
                                    ii.to(d), jj.to(d), 3, [1, 4])
    ref = oracle.corr_pyramid(gmap.numpy(), [f1.numpy(), f2.numpy()], coords.numpy(), ii.numpy(), jj.numpy())
    assert np.array_equal(bits(out.cpu().numpy()), bits(ref))


def test_fast_and_generic_paths_agree():
    import cuda_corr
    d = dev()
    gmap, f1, _, ii, jj, coords = dpvo_sized_inputs(3, E=700)
    a, = cuda_corr.forward(gmap.to(d), f1.to(d), coords.to(d), ii.to(d), jj.to(d), 3)            # NCHW: generic
    b, = cuda_corr.forward(gmap.to(d), channel_last(f1.to(d)), coords.to(d), ii.to(d), jj.to(d), 3)  # fast
    assert torch.equal(a.contiguous().view(torch.int16), b.contiguous().view(torch.int16))


def test_fp32_and_fp64_match_oracle():
    import cuda_corr
    d = dev()
    gmap, f1, _, ii, jj, coords = dpvo_sized_inputs(4, E=200, edge_cases=False)
    for dt, tol in ((torch.float32, 0.0), (torch.float64, 0.0)):
        g32, f32 = gmap.to(dt), f1.to(dt)
        out, = cuda_corr.forward(g32.to(d), f32.to(d), coords.to(d), ii.to(d), jj.to(d), 3)
        ref = oracle.corr_forward(g32.numpy(), f32.numpy(), coords.numpy(), ii.numpy(), jj.numpy(), 3)
        np.testing.assert_allclose(out.contiguous().cpu().numpy(), ref.transpose(0, 1, 3, 2, 4, 5), rtol=0, atol=tol)


def test_empty_and_invalid_indices():
    import cuda_corr
    d = dev()
    gmap, f1, f2, ii, jj, coords = dpvo_sized_inputs(5, E=64, edge_cases=False)
    out = cuda_corr.forward_pyramid(gmap.to(d), [channel_last(f1.to(d))], coords[:, :0].contiguous().to(d),
                                    ii[:0].to(d), jj[:0].to(d), 3, [1])
    assert out.shape == (1, 0, 441)
    ii = ii.clone(); ii[:5] = 10_000   # out-of-range patch index -> zeros (reference: undefined)
    out = cuda_corr.forward_pyramid(gmap.to(d), [channel_last(f1.to(d))], coords.to(d), ii.to(d), jj.to(d), 3, [1])
    assert torch.count_nonzero(out[0, :5]) == 0


def test_patchify_matches_oracle():
    import cuda_corr
    d = dev()
    g = torch.Generator().manual_seed(0)
    for dt, r, C in ((torch.float16, 1, 128), (torch.float32, 0, 384), (torch.float32, 1, 3)):
        net = torch.randn(1, C, 24, 32, generator=g).to(dt)
        coords = torch.stack([torch.randint(-2, 34, (1, 50), generator=g),
                              torch.randint(-2, 26, (1, 50), generator=g)], -1).float()
        coords[0, :10] += 0.5
        out, = cuda_corr.patchify_forward(net.to(d), coords.to(d), r)
        ref = oracle.patchify_forward(net.numpy(), coords.numpy(), r)
        assert np.array_equal(out.cpu().numpy(), ref)


def test_corr_backward_matches_autograd_reference():
    """Gradients of the generic fp32 forward, against a dense torch recomputation."""
    import cuda_corr
    d = dev()
    gmap, f1, _, ii, jj, coords = dpvo_sized_inputs(6, E=40, edge_cases=False)
    g32 = gmap.float().to(d).requires_grad_(True)
    f32 = f1[:, :, :, :24, :32].float().contiguous().to(d).requires_grad_(True)
    c = (coords.to(d) / 4).contiguous()
    out, = cuda_corr.forward(g32.detach(), f32.detach(), c, ii.to(d), jj.to(d), 3)
    grad = torch.randn_like(out)
    g1, g2 = cuda_corr.backward(g32.detach(), f32.detach(), c, ii.to(d), jj.to(d), grad, 3)
    # finite-difference-free check: the forward is bilinear in (gmap, fmap):
    # <grad, corr(g, f)> = <g1, g> = <g2, f>
    s = (grad * out).sum().double()
    assert torch.allclose((g1 * g32.detach()).sum().double(), s, rtol=1e-3)
    assert torch.allclose((g2 * f32.detach()).sum().double(), s, rtol=1e-3)


def test_nan_coordinates_follow_reference_conversion():
    """NaN coords: (int)floor(NaN) is 0 on the reference's GPU (cvt.rzi.s32), the
    bilinear weights are NaN; compare with NaN == NaN (payload bits may differ)."""
    import cuda_corr
    d = dev()
    gmap, f1, f2, ii, jj, coords = dpvo_sized_inputs(6, E=128, edge_cases=False)
    coords[0, :4] = float("nan")                 # whole edges
    coords[0, 4:8, 0, 1, 1] = float("nan")       # one patch pixel's x
    coords[0, 8:12, 1, 0, 2] = float("inf")      # +inf y
    out = cuda_corr.forward_pyramid(gmap.to(d), [channel_last(f1.to(d)), channel_last(f2.to(d))], coords.to(d),
                                    ii.to(d), jj.to(d), 3, [1, 4]).cpu().float().numpy()
    ref = oracle.corr_pyramid(gmap.numpy(), [f1.numpy(), f2.numpy()], coords.numpy(), ii.numpy(),
                              jj.numpy()).astype(np.float32)
    assert np.array_equal(np.isnan(out), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.array_equal(out[ok], ref[ok])


def test_packed_table_path_is_identical():
    """dpvo_corr_pack + forward with the table == forward packing internally (bit-exact)."""
    import cuda_corr
    d = dev()
    gmap, f1, f2, ii, jj, coords = dpvo_sized_inputs(7, E=500)
    args = (gmap.to(d), [channel_last(f1.to(d)), channel_last(f2.to(d))], coords.to(d), ii.to(d), jj.to(d), 3, [1, 4])
    a = cuda_corr.forward_pyramid(*args)
    tab = cuda_corr.pack(gmap.to(d))
    b = cuda_corr.forward_pyramid(*args, table=tab)
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
