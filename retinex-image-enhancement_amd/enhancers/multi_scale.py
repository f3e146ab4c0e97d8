"""MultiScaleEnhancer (drop-in for reference enhancers/multi_scale.py).

The scalar adjustment factor 1 + 0.1 * sum_i w_i * mean(features_i) is
computed on the device per image in one pass over the image for all three
scales (ms_sums3_kernel: fp64 per-tile partials, added in tile order by
ms_fin_kernel, which writes the factor); the reference syncs three times
through .item() (:313-314) and means over the whole batch — it only ever runs
B = 1.
"""
import torch

from upr import runtime


class MultiScaleEnhancer:
    def __init__(self):
        pass

    def extract_multi_scale_features(self, image_tensor):
        """[1,3,H,W] -> 3 tensors [1,7,h,w] at scales 1, 0.5, 0.25 (reference :17-60)."""
        if image_tensor.dim() == 3:
            image_tensor = image_tensor.unsqueeze(0)
        return [runtime.multiscale_features(image_tensor, i) for i in range(3)]

    def apply_multi_scale_enhancement(self, model, image_tensor, device):
        """model forward, then clamp(enh * factor, 0, 1) (reference :62-100)."""
        image_tensor = image_tensor.to(device)
        if image_tensor.dim() == 3:
            image_tensor = image_tensor.unsqueeze(0)
        with torch.no_grad():
            enhanced_img, reflectance, illu_map = model(image_tensor)
        out, _, _ = runtime.multiscale(image_tensor, enhanced_img)
        return out, illu_map

    def enhance_with_pyramid(self, model, image_tensor, device):
        """Alias used by simple_enhance (reference :102-115)."""
        return self.apply_multi_scale_enhancement(model, image_tensor, device)
