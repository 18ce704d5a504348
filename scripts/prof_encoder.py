"""Frame ingest x 20 for rocprofv3 --kernel-trace --stats: MODE=native (the
native encoders only), native_graph / torch_graph (the whole graph-replayed
ingest with the native or the torch encoders; one capture first)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import torch  # noqa: E402


def main():
    import encoder_ops
    from dpvo.net import Patchifier
    torch.manual_seed(0)
    pf = Patchifier(3).cuda().eval()
    img = torch.randint(0, 255, (3, 384, 512), device="cuda", dtype=torch.uint8)
    mode = os.environ.get("MODE", "native")
    if mode == "native":   # the two encoders only
        enc = encoder_ops.NativeEncoders(pf.fnet, pf.inet)
        xs = torch.randint(1, 127, (192,), device="cuda")
        with torch.no_grad():
            for _ in range(20):
                enc.run(img, xs, xs % 95 + 1)
    else:                  # the whole ingest replayed from its graph: torch modules or native encoders
        pf.NATIVE_ENCODERS = mode == "native_graph"
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            pf(img, 192)   # capture
            torch.cuda.synchronize()
            import time
            time.sleep(0.5)   # a gap in the kernel trace: what follows is the 20 replays
            for _ in range(20):
                pf(img, 192)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
