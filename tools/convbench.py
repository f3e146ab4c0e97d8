#!/usr/bin/env python3
"""Single-conv micro-benchmark over the C ABI (upr_conv2d_nhwc).

Times the conv kernels on the UP-Retinex layer shapes in isolation (HIP events
on the current stream), for tuning and for per-kernel rocprofv3 --pmc passes:

  python tools/convbench.py --dtype fp16 --shapes dec1,bneck --iters 20
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "retinex-image-enhancement_amd"))

import torch  # noqa: E402

from upr import runtime  # noqa: E402

# name: (B, H, W, Cin, Cout, k, stride, pad, dil, residual)
SHAPES = {
    "dec1": (32, 512, 512, 32, 32, 3, 1, 1, 1, True),     # dec1.conv.3-like, 512^2 32ch
    "dec1p": (32, 512, 512, 32, 32, 3, 1, 1, 1, False),   # dec1.conv.0-like (ReLU, no residual)
    "fam64": (32, 512, 512, 64, 32, 3, 1, 1, 1, False),   # FAM fusion-like 32-wide GEMM, K = 576
    "fam_h": (32, 512, 512, 32, 64, 3, 1, 1, 1, False),   # FAM branch3/4 conv1 fused, N=64
    "dec2": (32, 256, 256, 64, 64, 3, 1, 1, 1, True),
    "dec2p": (32, 256, 256, 64, 64, 3, 1, 1, 1, False),  # dec2.conv.0-like (ReLU, no residual)
    "dec3": (32, 128, 128, 128, 128, 3, 1, 1, 1, True),
    "dec3p": (32, 128, 128, 128, 128, 3, 1, 1, 1, False),  # dec3.conv.0-like (ReLU, no residual)
    "bneck": (32, 64, 64, 256, 256, 3, 1, 1, 1, False),
    "bneckr": (32, 64, 64, 256, 256, 3, 1, 1, 1, True),   # bottleneck conv2 (+ residual)
    "enc1s2": (32, 512, 512, 32, 64, 3, 2, 1, 1, False),
    "d2": (32, 512, 512, 32, 32, 3, 1, 2, 2, False),
    "aspp6": (32, 64, 64, 256, 256, 3, 1, 6, 6, False),
    "aspp12": (32, 64, 64, 256, 256, 3, 1, 12, 12, False),
    "aspp18": (32, 64, 64, 256, 256, 3, 1, 18, 18, False),
    "fuse": (32, 64, 64, 1280, 256, 1, 1, 0, 1, False),
    "fuse1k": (32, 64, 64, 1024, 256, 1, 1, 0, 1, False),  # ASPP fusion as executed (global branch = bias)
    "a1x1": (32, 64, 64, 256, 256, 1, 1, 0, 1, False),     # ASPP conv1x1
    "enc3s2": (32, 128, 128, 128, 256, 3, 2, 1, 1, False),
    "enc2s2": (32, 256, 256, 64, 128, 3, 2, 1, 1, False),
    "enc1c2": (32, 256, 256, 64, 64, 3, 1, 1, 1, True),   # enc1.conv2 (without the shortcut segment)
    "enc2c2": (32, 128, 128, 128, 128, 3, 1, 1, 1, True),
    "vgg3": (16, 128, 128, 256, 256, 3, 1, 1, 1, False),  # perceptual-loss VGG conv3_2/3_3 at 512^2
    "vgg31": (16, 128, 128, 128, 256, 3, 1, 1, 1, False),  # VGG conv3_1
    "vgg2": (16, 256, 256, 128, 128, 3, 1, 1, 1, False),   # VGG conv2_2
    "vgg21": (16, 256, 256, 64, 128, 3, 1, 1, 1, False),   # VGG conv2_1
    "vgg1": (16, 512, 512, 64, 64, 3, 1, 1, 1, False),     # VGG conv1_2
    "up1": (32, 256, 256, 64, 128, 1, 1, 0, 1, False),    # dec1.up GEMM shape (plain store)
    "up2": (32, 128, 128, 128, 256, 1, 1, 0, 1, False),   # dec2.up
    "up3": (32, 64, 64, 256, 512, 1, 1, 0, 1, False),     # dec3.up
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", choices=["fp32", "fp16"], default="fp16")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--bufs", type=int, default=1,
                    help="cycle over this many input copies (> 1: inputs larger than the 256 MB MALL "
                         "come from HBM, as inside the model)")
    args = ap.parse_args()
    dt = torch.float16 if args.dtype == "fp16" else torch.float32
    dev = torch.device("cuda", 0)
    for name in args.shapes.split(","):
        B, H, W, Ci, Co, k, s, p, d, res = SHAPES[name]
        g = torch.Generator(device=dev).manual_seed(0)
        xs = [torch.randn(B, H, W, Ci, device=dev, generator=g).to(dt) for _ in range(args.bufs)]
        x = xs[0]
        w = (torch.randn(Co, k * k * Ci, device=dev, generator=g) / (k * k * Ci) ** 0.5).to(dt)
        b = torch.randn(Co, device=dev, generator=g)
        Ho = (H + 2 * p - d * (k - 1) - 1) // s + 1
        Wo = (W + 2 * p - d * (k - 1) - 1) // s + 1
        r = torch.randn(B, Ho, Wo, Co, device=dev, generator=g).to(dt) if res else None
        relu = r is None  # residual shapes: plain conv + skip add (the UpBlock epilogue)
        for _ in range(3):
            runtime.conv2d_nhwc(x, w, b, k, k, s, p, d, residual=r, relu=relu)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(args.iters):
            runtime.conv2d_nhwc(xs[i % args.bufs], w, b, k, k, s, p, d, residual=r, relu=relu)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        flops = 2.0 * B * Ho * Wo * Co * Ci * k * k
        elt = 2 if dt == torch.float16 else 4
        nbytes = elt * (B * H * W * Ci + B * Ho * Wo * Co * (2 if res else 1) + Co * Ci * k * k)
        print(f"{name:8s} {args.dtype} {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s  {nbytes / ms / 1e6:8.1f} GB/s")


if __name__ == "__main__":
    main()
