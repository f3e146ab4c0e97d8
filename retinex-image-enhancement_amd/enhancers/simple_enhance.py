"""Enhance harness (drop-in for reference enhancers/simple_enhance.py).

Image decode/encode stays on the host (PIL), everything between load and save
runs on the device.  Intentional divergences, each a reference bug:
  * enhance_single_image accepts and ignores `adjuster=` so main.py's
    single-file branch works (reference main.py:240-249 vs simple_enhance.py:135
    raises TypeError);
  * enhance_batch_images takes optional use_preact/use_aspp/seed (defaults keep
    the reference behaviour: UP_Retinex() defaults, unseeded init).
"""
import os
from concurrent.futures import ThreadPoolExecutor
import time

import numpy as np
import torch
from PIL import Image

from models.model import UP_Retinex
from enhancers.adaptive_params import AdaptiveParameterAdjuster
from enhancers.multi_scale import MultiScaleEnhancer
from enhancers.content_aware import ContentAwareEnhancer
from utils.letterbox import letterbox_u8_image

# PNG encoders running beside the GPU (PIL's encoder releases the GIL); 3 files per
# image, ~90 / ~160 ms of host CPU each for a 512^2 / comparison PNG of a noisy image,
# so the batch harness is encode-bound: one writer per usable core but two, at most 14
# (os.cpu_count() is the whole machine on a shared box; UPR_PNG_WRITERS overrides)
def _writer_count():
    try:
        n = int(os.environ.get("UPR_PNG_WRITERS", "0"))
    except ValueError:
        n = 0
    return n if n > 0 else min(14, max(2, (os.cpu_count() or 8) - 2))


_WRITERS = _writer_count()
VALID_EXTENSIONS = {'.jpg', '.jpeg', '.png', '.bmp', '.tif', '.tiff'}


def _decode(image_path):
    """PIL decode -> (uint8 HWC RGB array, (W, H)).  Runs on the harness's
    prefetch thread for the next file of a batch."""
    img = Image.open(image_path).convert('RGB')
    return np.array(img, dtype=np.uint8), img.size


def load_image(image_path, max_size=None, device=None, decoded=None):
    """Decode + letterbox (reference :23-62) -> ([1,3,H,W] float32, (W, H)).

    The decoded uint8 pixels go to the ROCm device as bytes and ToTensor +
    letterbox_tensor run there as one launch (utils/letterbox.py); the tensor is
    returned on that device (the reference returns it on the CPU and the caller
    moves it -- the callers' .to(device) is then a no-op).  `decoded` takes an
    already decoded (array, size) pair (the batch harness's prefetch)."""
    a, original_size = decoded if decoded is not None else _decode(image_path)
    new_shape = max_size if max_size is not None else a.shape[:2]
    t, _, _ = letterbox_u8_image(a, new_shape=new_shape, auto=True, scaleup=False, device=device)
    return t.unsqueeze(0), original_size


def _to_u8_hwc(t):
    """(np.clip(x, 0, 1) * 255).astype(np.uint8) of one [C,H,W] image, 1-channel
    maps replicated to RGB (reference :65-99): one device launch, then the
    3 B/pixel copy to the host for the PNG encoder."""
    from upr import runtime
    return runtime.to_u8_hwc(t.detach()).cpu().numpy()


def _write_png(arr, save_path, msg):
    Image.fromarray(arr).save(save_path)
    print(f"{msg}: {save_path}")


def _emit(arr, save_path, msg, writer):
    if writer is None:
        _write_png(arr, save_path, msg)
    else:  # PNG encode + file write on the batch harness's writer thread
        writer.submit(_write_png, arr, save_path, msg)


def save_image(tensor, save_path, writer=None):
    """[1,C,H,W] or [C,H,W] -> PNG; 1-channel maps are replicated to RGB (reference :65-99)."""
    if tensor.dim() == 4:
        tensor = tensor.squeeze(0)
    _emit(_to_u8_hwc(tensor), save_path, "已保存", writer)


def create_comparison(img_low, img_enhanced, save_path, writer=None, illu_map=None):
    """[input | enhanced] side by side (reference :102-132); with `illu_map`
    the predictor's 3-panel form [input | enhanced | illumination]
    (reference predictors/predict.py:102-140)."""
    panels = [_to_u8_hwc(img_low.squeeze(0)), _to_u8_hwc(img_enhanced.squeeze(0))]
    if illu_map is not None:
        panels.append(_to_u8_hwc(illu_map.squeeze(0)))
    _emit(np.concatenate(panels, axis=1), save_path, "已保存对比图像", writer)


def enhance_single_image(model, image_path, output_dir, device, max_size=None, enable_multi_scale=False,
                         enable_content_aware=False, adjuster=None, precision="fp32", _decoded=None, _writer=None):
    """Enhance one file and write {name}_enhanced/_illumination/_comparison.png (reference :135-199).
    precision="fp16" runs the fp16 storage / fp16-MFMA graph (input cast to half)."""
    print(f"正在处理: {os.path.basename(image_path)}")
    img_low, _ = load_image(image_path, max_size, decoded=_decoded)
    if precision == "fp16":
        img_low = img_low.half()
    adjuster = AdaptiveParameterAdjuster()
    multi_scale_enhancer = MultiScaleEnhancer()
    content_aware_enhancer = ContentAwareEnhancer()
    start = time.time()
    if enable_content_aware:
        img_enhanced, illu_map = content_aware_enhancer.apply_content_aware_enhancement(model, img_low, device)
    elif enable_multi_scale:
        img_enhanced, illu_map = multi_scale_enhancer.enhance_with_pyramid(model, img_low, device)
    else:
        img_enhanced, illu_map = adjuster.apply_adaptive_enhancement(model, img_low, device)
    if torch.cuda.is_available() and img_enhanced.is_cuda:
        torch.cuda.synchronize(img_enhanced.device)
    print(f"增强耗时: {time.time() - start:.4f}s")
    os.makedirs(output_dir, exist_ok=True)
    name = os.path.splitext(os.path.basename(image_path))[0]
    save_image(img_enhanced, os.path.join(output_dir, f"{name}_enhanced.png"), _writer)
    save_image(illu_map, os.path.join(output_dir, f"{name}_illumination.png"), _writer)
    create_comparison(img_low, img_enhanced, os.path.join(output_dir, f"{name}_comparison.png"), _writer)
    print("图像增强完成！")
    return img_enhanced, illu_map


def list_images(input_dir):
    files = [os.path.join(input_dir, f) for f in os.listdir(input_dir)
             if os.path.splitext(f)[1].lower() in VALID_EXTENSIONS]
    return sorted(files)


def enhance_batch_images(input_dir, output_dir, device, max_size=None, use_preact=True, use_aspp=True, seed=None,
                         precision="fp32"):
    """Enhance every image of a directory (reference :202-250)."""
    print("正在加载模型...")
    if seed is not None:
        torch.manual_seed(seed)
    model = UP_Retinex(use_preact=use_preact, use_aspp=use_aspp).to(device).eval()
    image_files = list_images(input_dir)
    if not image_files:
        print(f"在目录 '{input_dir}' 中未找到有效图像文件")
        return
    print(f"找到 {len(image_files)} 个图像文件")
    print("=" * 50)
    total = 0.0
    # host pipeline around the device work: the next file is decoded on a
    # prefetch thread and the PNG encodes run on writer threads while the GPU
    # enhances the current image (the reference does all three serially)
    with ThreadPoolExecutor(max_workers=1) as reader, ThreadPoolExecutor(max_workers=_WRITERS) as writer:
        nxt = reader.submit(_decode, image_files[0])
        for i, path in enumerate(image_files, 1):
            print(f"[{i}/{len(image_files)}]")
            t0 = time.time()
            decoded = nxt.result()
            if i < len(image_files):
                nxt = reader.submit(_decode, image_files[i])
            enhance_single_image(model, path, output_dir, device, max_size, precision=precision, _decoded=decoded,
                                 _writer=writer)
            total += time.time() - t0
            print("-" * 50)
    print("=" * 50)
    print(f"总共处理了 {len(image_files)} 张图像")
    print(f"总耗时: {total:.2f}s")
    print(f"平均每张图像耗时: {total / len(image_files):.4f}s")
    print("=" * 50)
