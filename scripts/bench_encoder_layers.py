"""Per-layer time of the Patchifier encoders (BasicEncoder4, fp16 autocast) at
512x384: finds the convolutions MIOpen runs slowly.  Prints one JSON line per
conv layer."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "wild-video-3d-reconstruction_amd")]
import torch  # noqa: E402


def main():
    from dpvo.net import Patchifier
    torch.manual_seed(0)
    pf = Patchifier(3).cuda().eval()
    img = torch.randint(0, 255, (3, 384, 512), device="cuda", dtype=torch.uint8)
    shapes = {}

    def hook(name):
        def f(mod, inp, out):
            shapes[name] = (mod, inp[0].detach())
        return f
    for enc_name, enc in (("fnet", pf.fnet), ("inet", pf.inet)):
        for name, m in enc.named_modules():
            if isinstance(m, torch.nn.Conv2d):
                m.register_forward_hook(hook(f"{enc_name}.{name}"))
    with torch.no_grad(), torch.autocast("cuda", enabled=True):
        pf(img, patches_per_image=192, return_color=True)
        for name, (mod, x) in shapes.items():
            for _ in range(3):
                mod(x)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                mod(x)
            e.record()
            torch.cuda.synchronize()
            print(json.dumps({"layer": name, "in": list(x.shape), "dtype": str(x.dtype), "k": mod.kernel_size[0],
                              "stride": mod.stride[0], "us": round(s.elapsed_time(e) / 10 * 1e3, 1)}), flush=True)
        for _ in range(3):
            pf(img, patches_per_image=192, return_color=True)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            pf(img, patches_per_image=192, return_color=True)
        e.record()
        torch.cuda.synchronize()
        print(json.dumps({"layer": "patchify (both encoders + 4 altcorr.patchify)",
                          "us": round(s.elapsed_time(e) / 10 * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
