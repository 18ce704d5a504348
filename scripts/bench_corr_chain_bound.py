"""Row f2 bound: what fusing altcorr into the corr -> Linear(882 -> 384)
chain could save at most.  Times the update operator's corr chain
(rowchain<LN|LN_RELU>, net.py:53-56; E = 95,424 rows of 896 fp16) reading
(a) the corr tensor as the tracker does (171 MB from HBM), and
(b) the same rows gathered from a 2,048-row block (3.7 MB, L2-resident): the
    chain with its A operand already on chip, as a fused kernel would see it.
Run under rocprofv3 --kernel-trace --stats (both variants are the same kernel:
read the per-call trace; the first 10 calls are (a), the last 10 (b))."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import torch  # noqa: E402

import update_ops as U  # noqa: E402


def main():
    E, K, D = 95424, 896, 384
    torch.manual_seed(0)
    corr = (torch.randn(E, K, device="cuda") * 0.5).half()
    W1, b1 = U.pack_linear(torch.randn(D, 882, device="cuda") / 30, torch.randn(D, device="cuda") * 0.1)
    W2, b2 = U.pack_linear(torch.randn(D, D, device="cuda") / 20, torch.randn(D, device="cuda") * 0.1)
    ln = (torch.ones(D, device="cuda"), torch.zeros(D, device="cuda"), 1e-3)
    onchip = torch.arange(E, device="cuda") % 2048
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    res = {}
    for name, idx in (("hbm", None), ("l2_resident", onchip)):
        for _ in range(3):
            U.rowchain(corr, W1, b1, W2, b2, flags1=U.RELU, a_idx=idx, flags=U.LN | U.LN_RELU, ln=ln)
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(10):
            U.rowchain(corr, W1, b1, W2, b2, flags1=U.RELU, a_idx=idx, flags=U.LN | U.LN_RELU, ln=ln)
        ev[1].record()
        torch.cuda.synchronize()
        res[name + "_us"] = round(ev[0].elapsed_time(ev[1]) / 10 * 1e3, 1)
    print(res, flush=True)


if __name__ == "__main__":
    main()
