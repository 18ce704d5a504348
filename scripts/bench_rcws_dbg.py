"""Timing experiment for rowchain_ws_kernel<RES> (the c1 / c2 chain at C3 size,
E = 95,424 rows): DPVO_RCWS_DBG variants (csrc/rowgemm.hip) under rocprofv3
--kernel-trace; RCWS_VARIANTS picks them (results wrong except 0 and 1)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
os.environ.setdefault("DPVO_RCWS", "1")
import torch  # noqa: E402

import update_ops as U  # noqa: E402


def main():
    E, D = 95424, 384
    torch.manual_seed(0)
    A = torch.randn(E, D, device="cuda").half()
    idx = torch.randint(-1, E, (E,), device="cuda")
    res32 = torch.randn(E, D, device="cuda")
    W1, b1 = U.pack_linear(torch.randn(D, D, device="cuda") / 20, torch.randn(D, device="cuda") * 0.1)
    W2, b2 = U.pack_linear(torch.randn(D, D, device="cuda") / 20, torch.randn(D, device="cuda") * 0.1)
    for d in os.environ.get("RCWS_VARIANTS", "0,2,4,6,8,14").split(","):
        os.environ["DPVO_RCWS_DBG"] = d
        for _ in range(10):
            U.rowchain(A, W1, b1, W2, b2, flags1=U.RELU, a_idx=idx, flags=U.RES, res32=res32, want32=True)
        torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
