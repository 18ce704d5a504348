"""The SoftAgg h Linear on G group rows (G = 497 frame pairs / 4,224 patches at
C3, read on the device) with the v3 row GEMM (default) or v2 (64-row tiles,
DPVO_ROWGEMM=2): HIP-event time per launch."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]


def run(tag):
    import torch
    import update_ops as U
    torch.manual_seed(0)
    W, b = U.pack_linear(torch.randn(384, 384, device="cuda") / 20, torch.randn(384, device="cuda") * 0.1)
    res = {}
    for G in (497, 4224):
        A = torch.randn(95424, 384, device="cuda").half()
        Md = torch.tensor([G], device="cuda")
        for _ in range(3):
            U.rowgemm(A, W, b, M_dev=Md)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            U.rowgemm(A, W, b, M_dev=Md)
        e.record()
        torch.cuda.synchronize()
        res[f"G{G}_us"] = round(s.elapsed_time(e) / 50 * 1e3, 1)
    print(tag, res, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        for v in ("3", "2"):
            subprocess.check_call([sys.executable, __file__, "v" + v], env=dict(os.environ, DPVO_ROWGEMM=v))
