"""Times the AMP weight gradient (upr_t_conv_wgrad16) on the training step's
shapes (bs 8, 512^2 decoder / FAM convs).  UPR_LIB selects the library build."""
import argparse
import sys
import os

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "retinex-image-enhancement_amd"))
from upr import _lib as L  # noqa: E402

SHAPES = {
    "w32": (8, 512, 512, 32, 32, 1),
    "w32d2": (8, 512, 512, 32, 32, 2),
    "w64_32": (8, 512, 512, 64, 32, 1),
    "w32_64": (8, 512, 512, 32, 64, 1),
    "w64": (8, 256, 256, 64, 64, 1),
    "p96": (8, 512, 512, 96, 32, 0),
    "p128": (8, 512, 512, 128, 32, 0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dy16", action="store_true")
    args = ap.parse_args()
    lib = L.lib()
    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    for name in args.shapes.split(","):
        B, H, W, cin, cout, d = SHAPES[name]
        x16 = torch.randn(B, H, W, cin, device=dev).half()
        dy = torch.randn(B, H, W, cout, device=dev)
        dy16 = dy.half() if args.dy16 else None
        k = 1 if d == 0 else 3
        dw = torch.zeros(cout, cin, k, k, device=dev)

        def run():
            rc = lib.upr_t_conv_wgrad_into(None, x16.data_ptr(), B, H, W, cin, cin, 0, dy.data_ptr(),
                                           dy16.data_ptr() if dy16 is not None else None, H, W, cout, cout, 0,
                                           k, k, 1, d, max(d, 1), dw.data_ptr(), st)
            assert rc == 0, rc
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        fl = 2.0 * B * H * W * cout * k * k * cin
        by = B * H * W * (cin * 2 + cout * (2 if dy16 is not None else 4))
        print(f"{name:8s} {ms:7.3f} ms {fl / ms / 1e9:8.1f} TF/s {by / ms / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
