"""dpvo_window_group_by (DPVO.update's per-update grouping in four launches)
== dpvo_window_keys followed by dpvo_group_by(key_kk) and dpvo_group_by(key_ij):
the same slots, flag and both CSRs, bit for bit."""
import pytest
import torch
from tests_helpers import same

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("poisoned")]


def separate(ii, jj, kk, M, base, ring, frames, flag=None):
    import update_ops
    key_kk, key_ij, ctx, jslot = update_ops.window_keys(ii, jj, kk, M, base, ring, frames, flag=flag)
    kk_g = update_ops.group_by(key_kk, key_bits=update_ops.key_bits_for(64 * M))
    ij_g = update_ops.group_by(key_ij, key_bits=12)
    return ctx, jslot, kk_g, ij_g


def assert_same(got, want):
    assert same(got[0], want[0]) and same(got[1], want[1])
    for g, w in ((got[2], want[2]), (got[3], want[3])):
        G = int(w[3].item())
        assert same(g[3], w[3])
        assert same(g[0], w[0]) and same(g[2], w[2])
        assert same(g[1][:G + 1], w[1][:G + 1])   # offs past the group count is scratch


@pytest.mark.parametrize("preset,buffer,n", [("fast", 96, 70), ("dpvo_2k", 2048, 2040)])
def test_tracker_edges(preset, buffer, n):
    import update_ops
    from dpvo.synthetic import steady_state_tracker
    with torch.no_grad():
        s = steady_state_tracker(preset, buffer=buffer, n=n, seed=4)
    args = (s.pg.ii, s.pg.jj, s.pg.kk, s.M, s.n - 64, s.M * s.pmem, s.pmem)
    fa = torch.zeros(1, dtype=torch.int32, device="cuda")
    fb = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert_same(update_ops.window_group_by(*args, flag=fa), separate(*args, flag=fb))
    assert int(fa.item()) == 0 == int(fb.item())


@pytest.mark.parametrize("E,M,seed", [(1, 4, 0), (63, 8, 1), (5000, 96, 2), (70001, 384, 3)])
def test_random_window_edges(E, M, seed):
    """ragged sizes, unsorted edges, repeated keys in runs (the histogram's
    run aggregation) and scattered ones"""
    import update_ops
    g = torch.Generator().manual_seed(seed)
    n = 200
    ii = torch.randint(n - 64, n, (E,), generator=g)
    jj = torch.randint(n - 64, n, (E,), generator=g)
    kk = ii * M + torch.randint(0, M, (E,), generator=g)
    runs = torch.randint(0, 2, (E,), generator=g).bool()
    ii[1:][runs[1:]] = ii[:-1][runs[1:]]                 # some runs of equal keys
    kk = torch.where(runs, ii * M + kk % M, kk)
    ii, jj, kk = ii.cuda(), jj.cuda(), kk.cuda()
    args = (ii, jj, kk, M, n - 64, M * 40, 40)
    assert_same(update_ops.window_group_by(*args), separate(*args))
    # the optional target-frame order: the same CSRs, and a permutation of the
    # edges with jj ascending (altcorr's visiting order)
    got = update_ops.window_group_by(*args, jj_order=True)
    assert_same(got[:4], separate(*args))
    order = got[4].long()
    assert same(torch.sort(order).values, torch.arange(E, device="cuda"))
    assert bool((jj[order][1:] >= jj[order][:-1]).all())


def test_groups_above_the_lds_cap():
    """one (ii, jj) pair holding 5000 edges and one patch holding 3000: the
    fix-up's global-scan branch (groups > 2048 members) keeps edge order"""
    import update_ops
    n, M, E = 100, 16, 9000
    g = torch.Generator().manual_seed(5)
    ii = torch.randint(n - 64, n, (E,), generator=g)
    jj = torch.randint(n - 64, n, (E,), generator=g)
    sel = torch.randperm(E, generator=g)[:5000]
    ii[sel], jj[sel] = n - 3, n - 1
    kk = ii * M + torch.randint(0, M, (E,), generator=g)
    kk[sel[:3000]] = (n - 3) * M + 7
    args = (ii.cuda(), jj.cuda(), kk.cuda(), M, n - 64, M * 40, 40)
    got = update_ops.window_group_by(*args)
    assert_same(got, separate(*args))
    offs = got[3][1]
    sizes = (offs[1:int(got[3][3].item()) + 1] - offs[:int(got[3][3].item())]).max()
    assert int(sizes.item()) == 5000


def test_out_of_window_edges_flag_and_mask_alike():
    import update_ops
    n, M = 100, 8
    ii = torch.tensor([n - 1, n - 5, n - 40, n - 2], device="cuda")
    jj = torch.tensor([n - 2, n - 1, n - 70, n - 1], device="cuda")
    kk = ii * M + 3
    args = (ii, jj, kk, M, n - 64, M * 36, 36)
    fa = torch.zeros(1, dtype=torch.int32, device="cuda")
    fb = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert_same(update_ops.window_group_by(*args, flag=fa), separate(*args, flag=fb))
    assert int(fa.item()) == -2 == int(fb.item())
    fa.fill_(7)
    update_ops.window_group_by(*args, flag=fa)
    assert int(fa.item()) == 7


def test_empty():
    import update_ops
    e = torch.empty(0, dtype=torch.int64, device="cuda")
    ctx, jslot, kk_g, ij_g = update_ops.window_group_by(e, e, e, 8, 0, 64, 8)
    assert ctx.numel() == 0 and int(kk_g[3].item()) == 0 and int(ij_g[3].item()) == 0
    assert int(kk_g[1][0].item()) == 0 and int(ij_g[1][0].item()) == 0


def test_errors():
    import update_ops
    x = torch.zeros(3, dtype=torch.int64, device="cuda")
    with pytest.raises(RuntimeError, match="same length"):
        update_ops.window_group_by(x, x[:2], x, 8, 0, 64, 8)
    with pytest.raises(RuntimeError, match="counting-sort range"):
        update_ops.window_group_by(x, x, x, 1 << 20, 0, 64, 8)
    with pytest.raises(RuntimeError):
        update_ops.window_group_by(x.cpu(), x.cpu(), x.cpu(), 8, 0, 64, 8)
