"""The DPVO tracker (dpvo/dpvo.py mirror) on the GPU: the hot-path pieces of
one update against the oracle, and the full frame-by-frame API."""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def slam():
    from dpvo.synthetic import steady_state_tracker
    return steady_state_tracker("dpvo_2k", buffer=72, seed=0)


def test_steady_state_shapes(slam):
    n, M = slam.n, slam.M
    assert n == 64 and M == 192
    assert slam.pg.ii.numel() == 497 * M
    assert torch.unique(slam.pg.kk).numel() == 23 * M


def test_update_pieces_match_oracle(slam):
    """reproject -> corr (bit-exact on an edge sample) -> BA -> point cloud."""
    from dpvo import fastba
    from dpvo import projective_ops as pops
    from dpvo.lietorch import SE3
    with torch.no_grad():
        coords = slam.reproject()
        poses = slam.pg.poses_.cpu().numpy()
        patches = slam.pg.patches_.view(-1, 3, 3, 3).cpu().numpy()
        intr = slam.pg.intrinsics_.cpu().numpy()
        ii, jj, kk = (t.cpu().numpy() for t in (slam.pg.ii, slam.pg.jj, slam.pg.kk))
        ref = oracle.transform(poses, patches, intr, ii, jj, kk)[0].transpose(0, 3, 1, 2)
        np.testing.assert_allclose(coords[0].cpu().numpy(), ref, rtol=1e-5, atol=5e-3)

        corr = slam.corr(coords)
        sel = np.linspace(0, len(ii) - 1, 300).astype(np.int64)
        c_np = coords[0].cpu().numpy()[sel][None]
        want = oracle.corr_pyramid(slam.gmap.cpu().numpy(), [slam.fmap1_.contiguous().cpu().numpy(),
                                                              slam.fmap2_.contiguous().cpu().numpy()],
                                   c_np, kk[sel] % (slam.M * slam.pmem), jj[sel] % slam.pmem)
        assert np.array_equal(corr[0].cpu().numpy()[sel].view(np.uint16), want[0].view(np.uint16))

        g = torch.Generator(device=slam.device).manual_seed(5)
        target = coords[..., 1, 1] + torch.randn(1, len(ii), 2, generator=g, device=slam.device)
        weight = torch.rand(1, len(ii), 2, generator=g, device=slam.device)
        t0, t1 = slam.n - 10, slam.n
        rp, rq, st = oracle.ba_forward(poses, patches, intr, target.cpu().numpy(), weight.cpu().numpy(), 1e-4,
                                       ii, jj, kk, t0, t1, 2)
        assert st == 0
        fastba.BA(slam.poses, slam.patches, slam.intrinsics, target, weight, slam._lmbda, slam.pg.ii, slam.pg.jj,
                  slam.pg.kk, t0, t1, 2)
        gp = slam.pg.poses_.cpu().numpy()
        gq = slam.pg.patches_.view(-1, 3, 3, 3).cpu().numpy()
        assert np.linalg.norm(gp - rp) <= 1e-3 * np.linalg.norm(rp)
        assert np.linalg.norm(gq[:, 2] - rq[:, 2]) <= 1e-3 * np.linalg.norm(rq[:, 2])

        m = slam.pg.m
        pc = pops.point_cloud_centre(SE3(slam.poses), slam.patches[:, :m], slam.intrinsics, slam.ix[:m])
        want = oracle.point_cloud_centre(gp, gq[:m], intr, slam.ix[:m].cpu().numpy())
        np.testing.assert_allclose(pc.cpu().numpy(), want, rtol=1e-4, atol=1e-4)


def test_update_runs_and_moves_the_window(slam):
    with torch.no_grad():
        p0 = slam.pg.poses_.clone()
        d0 = slam.pg.patches_[..., 2, 1, 1].clone()
        for _ in range(3):
            slam.update()
        torch.cuda.synchronize()
    moved = (slam.pg.poses_ - p0).abs().amax(dim=1)
    assert moved[: slam.n - 10].max() == 0          # outside the optimisation window: fixed
    assert moved[slam.n - 10: slam.n].max() > 0     # inside: optimised
    assert torch.isfinite(slam.pg.points_[: slam.pg.m]).all()
    assert (slam.pg.patches_[..., 2, 1, 1] != d0).any()


def test_frame_by_frame_api():
    """__call__ -> init (12 updates) -> update + keyframe per frame -> terminate."""
    from dpvo.config import make_cfg
    from dpvo.dpvo import DPVO
    from dpvo.net import VONet
    from dpvo.synthetic import image_stream
    torch.manual_seed(0)
    net = VONet()
    with torch.no_grad():
        net.update.d[1].weight.mul_(40.0)  # random weights: make the motion probe pass
    cfg = make_cfg("fast", BUFFER_SIZE=64)
    intr = torch.tensor([320.0, 320.0, 320.0, 240.0], device="cuda")
    with torch.no_grad():
        slam = DPVO(cfg, net, ht=384, wd=512)
        for t, img in image_stream(24):
            slam(t, img, None, None, intr)
        assert slam.is_initialized
        poses, tstamps = slam.terminate()
    assert poses.shape == (24, 7) and np.isfinite(poses).all()
    assert len(tstamps) == 24
