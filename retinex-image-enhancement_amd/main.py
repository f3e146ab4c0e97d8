#!/usr/bin/env python3
"""UP-Retinex CLI (drop-in for the reference main.py; same flags, same modes).

`--mode enhance` is the hot path: every image runs the fused gfx950 graph
(libupr.so) and the device-side enhancers.  Additions: --seed (the reference
never seeds its random init, main.py:229) and --precision {fp32,fp16}.
Intentional divergences (reference bugs): a single-file --mode enhance works
(reference main.py:240-249 raises TypeError); --mode predict unpacks the
model's 3-tuple (reference predict.py:163 raises ValueError).
--mode train: the training STEP runs on the HIP path through the drop-in
trainers/train.py (train_step / train_one_epoch, losses/loss.py TotalLoss);
the reference's epoch driver around it (datasets, augmentation, schedulers,
TensorBoard, checkpoint files; reference trainers/train.py:134-330) is outside
this build's scope, so the CLI mode exits with that message.
"""
import argparse
import os
import sys
from pathlib import Path

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

from models.model import UP_Retinex  # noqa: E402
from enhancers.simple_enhance import (enhance_single_image, enhance_batch_images, list_images,  # noqa: E402
                                      load_image, save_image, create_comparison)
from enhancers.adaptive_params import AdaptiveParameterAdjuster  # noqa: E402


def build_parser():
    p = argparse.ArgumentParser(description='UP-Retinex: 基于Retinex理论的低光照图像增强 (MI355X)')
    p.add_argument('--mode', type=str, choices=['train', 'predict', 'enhance'], default='predict')
    p.add_argument('--train_dir', type=str, default='./data/train')
    p.add_argument('--test_dir', type=str, default='./data/test')
    p.add_argument('--input_path', type=str, default='./data/test')
    p.add_argument('--output_dir', type=str, default='./results')
    p.add_argument('--checkpoint', type=str, default='./checkpoints/best_model.pth')
    p.add_argument('--save_dir', type=str, default='./checkpoints')
    p.add_argument('--num_epochs', type=int, default=100)
    p.add_argument('--batch_size', type=int, default=8)
    p.add_argument('--image_size', type=int, default=640)
    p.add_argument('--lr', type=float, default=1e-4)
    p.add_argument('--weight_decay', type=float, default=1e-5)
    p.add_argument('--resume', type=str, default=None)
    p.add_argument('--weight_exp', type=float, default=10.0)
    p.add_argument('--weight_smooth', type=float, default=1.0)
    p.add_argument('--weight_col', type=float, default=0.5)
    p.add_argument('--weight_spa', type=float, default=1.0)
    p.add_argument('--weight_decouple', type=float, default=0.1)
    p.add_argument('--weight_perceptual', type=float, default=1.0)
    p.add_argument('--weight_freq', type=float, default=0.5)
    p.add_argument('--max_size', type=int, default=None)
    p.add_argument('--no_comparison', action='store_true')
    p.add_argument('--device', type=str, default=None)
    p.add_argument('--multi_scale', action='store_true')
    p.add_argument('--content_aware', action='store_true')
    p.add_argument('--num_workers', type=int, default=4)
    p.add_argument('--lr_decay_step', type=int, default=30)
    p.add_argument('--lr_decay_gamma', type=float, default=0.5)
    p.add_argument('--save_freq', type=int, default=10)
    p.add_argument('--use_amp', action='store_true')
    p.add_argument('--patience', type=int, default=20)
    p.add_argument('--use_cosine_scheduler', action='store_true')
    p.add_argument('--use_freq_loss', action='store_true')
    p.add_argument('--adaptive_weights', action='store_true')
    p.add_argument('--use_preact', action='store_true')
    p.add_argument('--use_aspp', action='store_true')
    p.add_argument('--advanced_augment', action='store_true')
    # additions
    p.add_argument('--seed', type=int, default=None, help='seed the random init (reproducible outputs)')
    p.add_argument('--precision', choices=['fp32', 'fp16'], default='fp32')
    return p


def _model(args):
    if args.seed is not None:
        torch.manual_seed(args.seed)
    m = UP_Retinex(use_preact=args.use_preact, use_aspp=args.use_aspp)
    return m


def _place(model, args):
    # compute precision follows the input tensor's dtype (fp16 inputs run the fp16 graph)
    return model.to(args.device).eval()


def _predict_one(model, path, args):
    """predictors/predict.py:144-191 predict_single_image: enhanced, illumination
    and the 3-panel [input | enhanced | illumination] comparison (:102-140; the
    1-channel map's channel mean is the map itself, replicated to RGB)."""
    x, _ = load_image(path, args.max_size)
    x = x.to(args.device)
    if args.precision == 'fp16':
        x = x.half()
    with torch.no_grad():
        enh, _, illu = model(x)
    os.makedirs(args.output_dir, exist_ok=True)
    name = os.path.splitext(os.path.basename(path))[0]
    save_image(enh, os.path.join(args.output_dir, f"{name}_enhanced.png"))
    save_image(illu, os.path.join(args.output_dir, f"{name}_illumination.png"))
    if not args.no_comparison:
        create_comparison(x, enh, os.path.join(args.output_dir, f"{name}_comparison.png"), illu_map=illu)


def main(argv=None):
    args = build_parser().parse_args(argv)
    if args.device is None:
        args.device = 'cuda' if torch.cuda.is_available() else 'cpu'
    print(f"使用设备: {args.device}")
    print(f"运行模式: {args.mode}")
    if args.mode == 'train':
        raise SystemExit("--mode train: the reference's epoch driver (datasets, augmentation, schedulers, "
                         "checkpoint files) is outside this build; the HIP training step itself is the drop-in "
                         "trainers.train.train_step / train_one_epoch with losses.loss.TotalLoss")
    if args.mode == 'predict':
        if not os.path.exists(args.checkpoint):
            print(f"错误: 找不到模型检查点文件 '{args.checkpoint}'")
            return
        model = _model(args)
        ckpt = torch.load(args.checkpoint, map_location='cpu', weights_only=True)
        model.load_state_dict(ckpt['model_state_dict'])
        model = _place(model, args)
        p = Path(args.input_path)
        files = [str(p)] if p.is_file() else (list_images(str(p)) if p.is_dir() else None)
        if files is None:
            print(f"错误: 输入路径 '{args.input_path}' 不存在")
            return
        for f in files:
            _predict_one(model, f, args)
        print("推理完成，结果已保存到:", args.output_dir)
        return
    # enhance
    os.makedirs(args.output_dir, exist_ok=True)
    p = Path(args.input_path)
    if p.is_file():
        model = _place(_model(args), args)
        enhance_single_image(model=model, image_path=str(p), output_dir=args.output_dir, device=args.device,
                             max_size=args.max_size, adjuster=AdaptiveParameterAdjuster(),
                             enable_multi_scale=args.multi_scale, enable_content_aware=args.content_aware,
                             precision=args.precision)
    elif p.is_dir():
        # reference: enhance_batch_images builds UP_Retinex() with its defaults (preact + ASPP)
        enhance_batch_images(input_dir=str(p), output_dir=args.output_dir, device=args.device,
                             max_size=args.max_size, seed=args.seed, precision=args.precision)
    else:
        print(f"错误: 输入路径 '{args.input_path}' 不存在")
        return
    print("图像增强完成，结果已保存到:", args.output_dir)


if __name__ == '__main__':
    main()
