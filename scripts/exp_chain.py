"""Microbench of the update operator's GEMM launches at C3 shapes (E = 95,424
rows): the c1 residual chain, the gated LN chain and the SoftAgg pair, timed
with HIP events on torch's stream.  Used to compare kernel variants."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "wild-video-3d-reconstruction_amd"))
import update_ops as U  # noqa: E402


def timeit(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    torch.manual_seed(0)
    E, dev = 95424, "cuda"
    lin = lambda: U.pack_linear(torch.randn(384, 384, device=dev) / 20.0, torch.randn(384, device=dev) * 0.1)
    n16 = (torch.randn(E, 384, device=dev) * 0.5).half()
    n32 = torch.randn(E, 384, device=dev)
    idx = torch.randperm(E, device=dev)
    idx[::7] = -1
    (W1, b1), (W2, b2), (Wg, bg) = lin(), lin(), lin()
    ln = (torch.rand(384, device=dev) + 0.5, torch.randn(384, device=dev) * 0.1, 1e-3)
    out = {}
    out["c1_res"] = timeit(lambda: U.rowchain(n16, W1, b1, W2, b2, flags1=U.RELU, a_idx=idx, flags=U.RES, res32=n32,
                                              want32=True))
    out["c1_no16"] = timeit(lambda: U.rowchain(n16, W1, b1, W2, b2, flags1=U.RELU, a_idx=idx, flags=U.RES, res32=n32,
                                               want32=True, want16=False))
    out["c1_plain"] = timeit(lambda: U.rowchain(n16, W1, b1, W2, b2, flags1=U.RELU, a_idx=idx, flags=U.LN | U.LN_RELU,
                                                ln=ln))
    out["gru_ln"] = timeit(lambda: U.rowchain(n16, W1, b1, W2, b2, flags1=U.RELU, flags=U.GATE | U.LN, res32=n32,
                                              gate=(Wg, bg), ln=ln, want32=True))
    Wa, Wb = U.kblock(W1), U.kblock(W2)
    out["pair"] = timeit(lambda: U.rowgemm_pair(n16, Wa, b1, Wb, b2))
    print(os.environ.get("DPVO_EXP_RC", "0"), " ".join(f"{k} {v:.1f}" for k, v in out.items()), flush=True)


if __name__ == "__main__":
    main()
