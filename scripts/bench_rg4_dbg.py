"""Timing experiment for rowgemm4_kernel (plain K = 384 GEMM over E = 95,424
rows, DPVO_ROWGEMM=4): each DPVO_RG4_DBG variant drops one part of the kernel
(1 epilogue, 2 MFMA, 4 A loads, 8 W loads) so the time left shows what bounds
it.  Run under rocprofv3 --kernel-trace: the variants are told apart by their
template argument in the kernel name."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
os.environ["DPVO_ROWGEMM"] = "4"
import torch  # noqa: E402

import update_ops as U  # noqa: E402


def main():
    E, D, K = 95424, 384, int(os.environ.get("RG_K", "384"))
    torch.manual_seed(0)
    A = torch.randn(E, K, device="cuda").half()
    W16, b16 = U.pack_linear(torch.randn(D, K, device="cuda") / K ** 0.5, torch.randn(D, device="cuda") * 0.1)
    for d in ["0", "1", "16", "14", "30", "6", "22", "15"]:
        os.environ["DPVO_RG4_DBG"] = d
        for _ in range(10):
            U.rowgemm(A, W16, b16)
        torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
