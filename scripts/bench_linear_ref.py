"""Reference point for the row GEMMs: one Linear(384 -> 384) over E = 95,424
fp16 rows (146 MB in + out) through hipBLASLt (torch.nn.functional.linear),
through the repo's rowgemm3 (update_ops.rowgemm), and a plain device copy of
the same bytes -- HIP-event time per call."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import torch  # noqa: E402

import update_ops as U  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / n * 1e3, 1)


def main():
    torch.manual_seed(0)
    E = 95424
    A = torch.randn(E, 384, device="cuda").half()
    Wf, bf = torch.randn(384, 384, device="cuda") / 20, torch.randn(384, device="cuda") * 0.1
    W16, b16 = Wf.half(), bf.half()
    Wp, bp = U.pack_linear(Wf, bf)
    out = torch.empty_like(A)
    res = {
        "hipblaslt_linear_us": timed(lambda: torch.nn.functional.linear(A, W16, b16)),
        "rowgemm3_us": timed(lambda: U.rowgemm(A, Wp, bp)),
        "copy_146MB_us": timed(lambda: out.copy_(A)),
    }
    print(res, flush=True)


if __name__ == "__main__":
    main()
