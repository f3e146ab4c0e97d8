#!/usr/bin/env python3
"""Root enhance CLI (drop-in for the reference simple_enhance.py:17-94):
--input/--output/--max_size/--device/--multi_scale/--content_aware, plus --seed."""
import argparse
import os
import sys
from pathlib import Path

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

from enhancers.simple_enhance import enhance_single_image, enhance_batch_images  # noqa: E402
from models.model import UP_Retinex  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description='简化版UP-Retinex图像增强工具 (MI355X)')
    ap.add_argument('--input', type=str, required=True)
    ap.add_argument('--output', type=str, default='./results')
    ap.add_argument('--max_size', type=int, default=None)
    ap.add_argument('--device', type=str, default=None)
    ap.add_argument('--multi_scale', action='store_true')
    ap.add_argument('--content_aware', action='store_true')
    ap.add_argument('--seed', type=int, default=None)
    args = ap.parse_args(argv)
    if args.device is None:
        args.device = 'cuda' if torch.cuda.is_available() else 'cpu'
    print(f"使用设备: {args.device}")
    if not os.path.exists(args.input):
        print(f"错误: 找不到输入路径 '{args.input}'")
        return
    p = Path(args.input)
    if p.is_file():
        if args.seed is not None:
            torch.manual_seed(args.seed)
        model = UP_Retinex().to(args.device).eval()
        # the reference passes only enable_multi_scale here (--content_aware is ignored, :66-77)
        enhance_single_image(model=model, image_path=str(p), output_dir=args.output, device=args.device,
                             max_size=args.max_size, enable_multi_scale=args.multi_scale)
    elif p.is_dir():
        enhance_batch_images(input_dir=str(p), output_dir=args.output, device=args.device, max_size=args.max_size,
                             seed=args.seed)
    else:
        print(f"错误: 输入路径 '{args.input}' 不是有效的文件或目录")
        return
    print(f"结果已保存到: {args.output}")


if __name__ == "__main__":
    main()
