"""A/B of the CSR SoftAgg reduce at C3: softagg_csr(long_groups=True) (groups
of >= 64 edges cut over four waves) against the default kernel -- HIP-event
time for the update operator's two groupings, and the largest difference."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]


def run(tag):
    import torch
    import update_ops as U
    from dpvo.synthetic import steady_state_tracker
    s = steady_state_tracker("dpvo_2k", buffer=2048, seed=0)
    E = s.pg.kk.numel()
    torch.manual_seed(0)
    fg = torch.randn(E, 768, device="cuda").half()
    f, g = fg[:, :384], fg[:, 384:]
    res = {}
    for name, key in (("kk", s.pg.kk), ("ij", s.pg.ii * 12345 + s.pg.jj)):
        gid, offs, perm, G = U.group_by(key)
        lg = tag == "split"
        y = U.softagg_csr(f, g, offs, perm, G, E, long_groups=lg)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            U.softagg_csr(f, g, offs, perm, G, E, long_groups=lg)
        b.record()
        torch.cuda.synchronize()
        res[name + "_us"] = round(a.elapsed_time(b) / 20 * 1e3, 1)
        torch.save(y[:int(G.item())].float().cpu(), f"/tmp/sa_{name}_{tag}.pt")
    print(tag, res, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        env = dict(os.environ)
        subprocess.check_call([sys.executable, __file__, "split"], env=env)
        subprocess.check_call([sys.executable, __file__, "nosplit"], env=env)
        import torch
        for n in ("kk", "ij"):
            a, b = torch.load(f"/tmp/sa_{n}_split.pt"), torch.load(f"/tmp/sa_{n}_nosplit.pt")
            print(n, "bit-equal:", torch.equal(a, b), "max abs diff:", (a - b).abs().max().item())
