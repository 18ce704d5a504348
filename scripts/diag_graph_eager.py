"""Eager vs eager and eager vs graph-replayed update() on the small steady
state of tests/test_gpu_update_async.py: which tensors differ after each
update (determinism / capture check)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import torch  # noqa: E402


def make(seed=5, buffer=72):
    from dpvo.synthetic import steady_state_tracker
    return steady_state_tracker("dpvo_2k", buffer=buffer, seed=seed)


def cmp(tag, a, b):
    n, m = a.n, a.pg.m
    out = []
    for name, x, y in (("poses", a.pg.poses_[:n], b.pg.poses_[:n]), ("patches", a.pg.patches_[:m], b.pg.patches_[:m]),
                       ("net", a.pg.net, b.pg.net), ("target", a.pg.target, b.pg.target),
                       ("weight", a.pg.weight, b.pg.weight)):
        d = (x.float() - y.float()).abs()
        out.append(f"{name}: {'equal' if torch.equal(x, y) else f'max {d.max().item():.3g} n {(d > 0).sum().item()}'}")
    print(tag, "; ".join(out), flush=True)


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
with torch.no_grad():
    for mode in ("eager", "graph") * reps:
        a, b = make(), make()
        for i in range(4):
            a.update()
            b.update() if mode == "eager" else b.update_graphed()
            torch.cuda.synchronize()
            cmp(f"{mode} update {i}", a, b)
