"""Bit-identity check for rowchain_kernel<RES> timing variants that keep the
arithmetic (DPVO_RC_DBG values in RC_EQUAL, default 2048): each variant's
out32 / out16 against DPVO_RC_DBG=0 on the c1-chain shape."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
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
    outs = {}
    for d in ["0"] + os.environ.get("RC_EQUAL", "2048").split(","):
        os.environ["DPVO_RC_DBG"] = d
        outs[d] = U.rowchain(A, W1, b1, W2, b2, flags1=U.RELU, a_idx=idx, flags=U.RES, res32=res32, want32=True)[:2]
    torch.cuda.synchronize()
    ok = True
    for d, (o32, o16) in outs.items():
        same = torch.equal(o32, outs["0"][0]) and torch.equal(o16, outs["0"][1])
        print(f"DPVO_RC_DBG={d}: bit-identical to 0: {same}", flush=True)
        ok &= same
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
