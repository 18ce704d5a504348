"""The per-frame bookkeeping ops of DPVO.__call__ / keyframe() that replace
Python-level compositions: the DAMPED_LINEAR motion model and the keyframe's
relative pose (lietorch calls in the reference), and the edge append
(aranges + meshgrids + concatenations)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def random_poses(n, seed):
    from dpvo.lietorch import SE3
    g = torch.Generator().manual_seed(seed)
    xi = torch.cat([0.5 * torch.randn(n, 3, generator=g), 0.3 * torch.randn(n, 3, generator=g)], -1)
    return SE3.exp(xi.cuda()).data.contiguous()


@pytest.mark.parametrize("seed,s", [(0, 0.5), (1, 1.0), (2, 0.0), (3, 2.5)])
def test_pose_extrapolate_equals_the_lietorch_composition(seed, s):
    from dpvo import projective_ops as pops
    from dpvo.lietorch import SE3
    poses = random_poses(8, seed)
    n = 5
    P1, P2 = SE3(poses[n - 1]), SE3(poses[n - 2])
    want = (SE3.exp(s * (P1 * P2.inv()).log()) * P1).data
    got = poses.clone()
    pops.pose_extrapolate(got, n, s)
    torch.testing.assert_close(got[n], want, rtol=0, atol=2e-6)
    assert torch.equal(got[:n], poses[:n]) and torch.equal(got[n + 1:], poses[n + 1:])


def test_pose_relative_equals_the_lietorch_composition():
    from dpvo import projective_ops as pops
    from dpvo.lietorch import SE3
    poses = random_poses(4, 7)
    got = pops.pose_relative(poses[2], poses[1]).data
    want = (SE3(poses[2]) * SE3(poses[1]).inv()).data
    torch.testing.assert_close(got, want, rtol=0, atol=2e-6)


def reference_append(ii, jj, kk, ix, n, M, r):
    """dpvo.py:756-769 + append_factors, as torch ops"""
    from dpvo.utils import flatmeshgrid
    dev = kk.device
    kf, jf = flatmeshgrid(torch.arange(M * max(n - r, 0), M * max(n - 1, 0), device=dev),
                          torch.arange(n - 1, n, device=dev), indexing="ij")
    kb, jb = flatmeshgrid(torch.arange(M * max(n - 1, 0), M * max(n, 0), device=dev),
                          torch.arange(max(n - r, 0), n, device=dev), indexing="ij")
    k = torch.cat([kf, kb])
    return torch.cat([ii, ix[k]]), torch.cat([jj, torch.cat([jf, jb])]), torch.cat([kk, k])


@pytest.mark.parametrize("n,M,r,E", [(1, 4, 13, 0), (2, 4, 13, 5), (12, 8, 13, 40), (40, 96, 13, 9000),
                                     (70, 192, 13, 0), (30, 16, 1, 7)])
def test_append_edges_equals_the_reference_construction(n, M, r, E):
    import update_ops
    g = torch.Generator().manual_seed(n)
    ii = torch.randint(0, 100, (E,), generator=g).cuda()
    jj = torch.randint(0, 100, (E,), generator=g).cuda()
    kk = torch.randint(0, 1000, (E,), generator=g).cuda()
    ix = torch.arange(128, device="cuda").repeat_interleave(M)   # index_: frame f's M patches map to f
    got = update_ops.append_edges(ii, jj, kk, ix, n, M, r)
    want = reference_append(ii, jj, kk, ix, n, M, r)
    for a, b in zip(got, want):
        assert torch.equal(a, b)


def test_append_edges_errors():
    import update_ops
    x = torch.zeros(3, dtype=torch.int64, device="cuda")
    with pytest.raises(RuntimeError, match="same length"):
        update_ops.append_edges(x, x[:2], x, x, 5, 4, 13)
    with pytest.raises(RuntimeError, match="PATCH_LIFETIME"):
        update_ops.append_edges(x, x, x, x, 0, 4, 13)
    with pytest.raises(RuntimeError):
        update_ops.append_edges(x.cpu(), x.cpu(), x.cpu(), x.cpu(), 5, 4, 13)
