"""Frame-ingest timing (row f1): Patchifier on one 512x384 frame under fp16
autocast -- eager, graph-replayed, and the encoders in channels-last memory
format -- with HIP events.  Run under rocprofv3 --kernel-trace for the
per-kernel split."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import torch  # noqa: E402


def timed(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    from dpvo.net import VONet
    torch.manual_seed(0)
    net = VONet().cuda().eval()
    pf = net.patchify
    img = torch.randint(0, 255, (3, 384, 512), device="cuda", dtype=torch.uint8).float()
    res = {}
    img8 = img.to(torch.uint8)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        for native in (True, False):
            pf.NATIVE_ENCODERS = native
            tag = "native" if native else "torch"
            pf.graphed = False
            res[f"{tag}_eager_ms"] = timed(lambda: pf(img8, 96))
            pf.graphed = True
            res[f"{tag}_graph_ms"] = timed(lambda: pf(img8, 96))
        import encoder_ops
        enc = encoder_ops.NativeEncoders(pf.fnet, pf.inet)
        xs = torch.randint(1, 127, (96,), device="cuda")
        res["native_encoders_only_ms"] = timed(lambda: enc.run(img8, xs, xs % 95 + 1))
        pf.NATIVE_ENCODERS = False
        pf.graphed = False
        res["eager_ms"] = timed(lambda: pf(img, 96))
        x = 2 * (img[None, None] / 255.0) - 0.5
        res["fnet_eager_ms"] = timed(lambda: pf.fnet(x))
        res["inet_eager_ms"] = timed(lambda: pf.inet(x))
        pf.fnet.to(memory_format=torch.channels_last)
        pf.inet.to(memory_format=torch.channels_last)
        res["fnet_cl_ms"] = timed(lambda: pf.fnet(x))
        res["inet_cl_ms"] = timed(lambda: pf.inet(x))
        torch.backends.cudnn.benchmark = True
        res["fnet_cl_bench_ms"] = timed(lambda: pf.fnet(x))
        res["inet_cl_bench_ms"] = timed(lambda: pf.inet(x))
    print({k: round(v, 3) for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
