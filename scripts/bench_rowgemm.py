"""Micro-benchmark: the fused full-row GEMM vs torch/hipBLASLt at the C3 update
operator shape (E = 95,424 rows, 384 -> 384, fp16).  Prints JSON lines."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import torch  # noqa: E402

import update_ops as U  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    E, D = 95424, 384
    torch.manual_seed(0)
    for K in (384, 896):
        A = torch.randn(E, K, device="cuda").half()
        w = torch.randn(D, K, device="cuda") / K ** 0.5
        b = torch.randn(D, device="cuda") * 0.1
        W16, b16 = U.pack_linear(w, b)
        w16 = w.half()
        flops = 2.0 * E * K * D
        t_ours = timeit(lambda: U.rowgemm(A, W16, b16))
        t_blas = timeit(lambda: torch.nn.functional.linear(A, w16, b16))
        x = torch.randn(E, D, device="cuda")
        g = torch.ones(D, device="cuda")
        be = torch.zeros(D, device="cuda")
        t_fused = timeit(lambda: U.rowgemm(A, W16, b16, flags=U.RES | U.LN, res32=x, ln=(g, be, 1e-3), want32=True))

        def unfused():
            y = torch.nn.functional.linear(A, w16, b16)
            return torch.nn.functional.layer_norm(x + y, (D,), g, be, 1e-3)
        t_unf = timeit(unfused)
        print(json.dumps({"K": K, "rows": E, "rowgemm_ms": round(t_ours, 4), "hipblaslt_ms": round(t_blas, 4),
                          "rowgemm_tflops": round(flops / t_ours / 1e9, 1),
                          "hipblaslt_tflops": round(flops / t_blas / 1e9, 1),
                          "fused_res_ln_ms": round(t_fused, 4), "torch_linear_add_ln_ms": round(t_unf, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
