"""ContentAwareEnhancer (drop-in for reference enhancers/content_aware.py).

Saliency (8-bit gray -> |Laplacian| -> 15x15 Gaussian, fp64 like the
reference's OpenCV CV_64F path), attention and the final modulation all run
on the device.  Intentional divergence: the reference keeps the saliency map
on the CPU and then multiplies it with a device tensor (:56-57 vs :85), which
raises on a GPU; here every map lives on the input's device.
"""
import torch

from upr import runtime


def _batch(t):
    return t.unsqueeze(0) if t.dim() == 3 else t


class ContentAwareEnhancer:
    def __init__(self):
        pass

    def compute_saliency_map(self, image_tensor):
        """[1,3,H,W] -> [1,1,H,W] float32 in [0,1] (reference :19-59)."""
        x = _batch(image_tensor)
        _, sal, _ = runtime.content_aware(x, saliency=True)
        return sal.unsqueeze(1)

    def compute_attention_map(self, image_tensor):
        """saliency / (luminance + 0.1), min-max normalised (reference :61-91)."""
        x = _batch(image_tensor)
        _, _, att = runtime.content_aware(x, attention=True)
        return att.unsqueeze(1)

    def apply_content_aware_enhancement(self, model, image_tensor, device):
        """model forward, then clamp(enh * (1 + 0.2 * attention), 0, 1) (reference :93-122)."""
        image_tensor = _batch(image_tensor.to(device))
        with torch.no_grad():
            enhanced_img, reflectance, illu_map = model(image_tensor)
        out, _, _ = runtime.content_aware(image_tensor, enhanced_img)
        return out, illu_map
