#!/usr/bin/env python3
"""End-to-end `main.py --mode enhance` directory throughput (decode -> device
letterbox -> model + CLAHE-in-Lab enhancer -> device u8 -> PNG encode):
enhance_batch_images over N synthetic low-light PNGs, images/s including IO.

  python tools/harness_bench.py --n 32 --size 512 [--precision fp16]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "retinex-image-enhancement_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--precision", choices=["fp32", "fp16"], default="fp32")
    args = ap.parse_args()
    from enhancers.simple_enhance import enhance_batch_images
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        src, out = os.path.join(d, "in"), os.path.join(d, "out")
        os.makedirs(src)
        rng = np.random.default_rng(0)
        for k in range(args.n):
            a = (rng.integers(0, 256, (args.size, args.size, 3)) * 0.35).astype(np.uint8)
            Image.fromarray(a).save(os.path.join(src, f"img{k:03d}.png"))
        with contextlib.redirect_stdout(io.StringIO()):
            enhance_batch_images(src, out + "_warm", "cuda", seed=0, precision=args.precision)  # warm-up (packing)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            enhance_batch_images(src, out, "cuda", seed=0, precision=args.precision)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        n_out = len(os.listdir(out))
    print(json.dumps({"metric": "enhance harness images/s (decode + letterbox + UP_Retinex preact+ASPP + "
                                "CLAHE-in-Lab + 3 PNG writes per image)", "value": args.n / el, "unit": "images/s",
                      "n": args.n, "size": args.size, "precision": args.precision, "seconds": el,
                      "files_written": n_out}))


if __name__ == "__main__":
    main()
