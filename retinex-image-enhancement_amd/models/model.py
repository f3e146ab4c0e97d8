"""UP-Retinex model surface (drop-in for the reference's models/model.py).

Module tree, attribute names, constructor arguments and construction order are
those of the reference (models/model.py:11-464), so
`torch.manual_seed(s); UP_Retinex(...)` yields the same state_dict (keys and
values) and checkpoints load unchanged.  Execution is not PyTorch's: on a ROCm
device `MultiScaleUP_Retinex.forward` / `ResidualIENet.forward` run the fused
gfx950 kernel graph of libupr.so (BatchNorm folded, implicit-GEMM MFMA convs,
fused FAM attention and Retinex tail).  In training mode the forward runs the
HIP training engine (upr/train.py: batch-statistics BatchNorm, Dropout, an
explicit backward reached through `loss.backward()`).  The submodules
(EnhancedFAM, ResBlock, PreActResBlock, ASPPModule, UpBlock) called on their own
run on the per-module HIP layer objects (upr/modules.py), in eval or training
mode.  There is no eager fallback: CPU tensors raise.
"""
import torch
import torch.nn as nn

from upr.runtime import ModelHandle

class _FusedModule(nn.Module):
    """Submodules: fused into the model's HIP graph inside MultiScaleUP_Retinex;
    a direct call runs the module alone on the HIP layer kernels
    (upr/modules.py: NCHW float32 / float16 in / out, eval or training mode)."""

    def forward(self, x):
        from upr.modules import submodule_forward
        return submodule_forward(self, x)


class EnhancedFAM(_FusedModule):
    """Feature Aggregation Module: 4 branches -> concat -> 1x1 fusion -> ReLU ->
    channel attention -> spatial attention (reference models/model.py:11-97).
    HIP: one 64-channel 3x3 GEMM for both cascaded first convs, one GEMM over the
    virtual concat with the fusion 1x1 composed into every branch, then the
    attention kernels (csrc/model.hip Builder::fam)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        ci, co = in_channels, out_channels
        self.branch1 = nn.Conv2d(ci, co, kernel_size=1, padding=0)
        self.branch2_pool = nn.MaxPool2d(kernel_size=3, stride=1, padding=1)
        self.branch2_conv = nn.Conv2d(ci, co, kernel_size=1, padding=0)
        self.branch3_conv1 = nn.Conv2d(ci, co, kernel_size=3, padding=1)
        self.branch3_conv2 = nn.Conv2d(co, co, kernel_size=3, padding=1)
        self.branch4_conv1 = nn.Conv2d(ci, co, kernel_size=3, padding=1)
        self.branch4_conv2 = nn.Conv2d(co, co, kernel_size=3, padding=2, dilation=2)
        self.fusion = nn.Conv2d(4 * co, co, kernel_size=1, padding=0)
        squeeze = co // 16
        self.channel_attention = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(co, squeeze, 1),
                                               nn.ReLU(inplace=True), nn.Conv2d(squeeze, co, 1), nn.Sigmoid())
        self.spatial_attention = nn.Sequential(nn.Conv2d(2, 1, 7, padding=3), nn.Sigmoid())
        self.relu = nn.ReLU(inplace=True)


def _shortcut(ci, co, stride):
    if stride != 1 or ci != co:
        return nn.Sequential(nn.Conv2d(ci, co, kernel_size=1, stride=stride, bias=False), nn.BatchNorm2d(co))
    return nn.Sequential()


class ResBlock(_FusedModule):
    """conv3x3(s)-BN-ReLU-conv3x3-BN + shortcut, ReLU (reference :100-135).
    HIP: two GEMMs; BN folded; the projecting shortcut is a second K-segment of
    conv2's GEMM."""

    def __init__(self, in_channels, out_channels, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, out_channels, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(out_channels)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(out_channels, out_channels, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(out_channels)
        self.shortcut = _shortcut(in_channels, out_channels, stride)


class PreActResBlock(_FusedModule):
    """BN-ReLU-conv, BN-ReLU-conv + shortcut, no trailing ReLU (reference :138-178).
    HIP: relu(bn1(x)) is a per-channel prologue of the GEMMs reading x."""

    def __init__(self, in_channels, out_channels, stride=1):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(in_channels)
        self.relu = nn.ReLU(inplace=True)
        self.conv1 = nn.Conv2d(in_channels, out_channels, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(out_channels)
        self.conv2 = nn.Conv2d(out_channels, out_channels, kernel_size=3, stride=1, padding=1, bias=False)
        self.shortcut = _shortcut(in_channels, out_channels, stride)


class ASPPModule(_FusedModule):
    """1x1 + dilated 3x3 (6/12/18) + global-pool branches, concat, 1x1 fusion
    (reference :181-251).  HIP: branches write channel slices of one 1024-ch
    buffer; the global branch becomes a per-image bias of the fusion GEMM."""

    def __init__(self, in_channels, out_channels, dilations=(1, 6, 12, 18)):
        super().__init__()
        dilations = list(dilations)
        self.dilations = dilations
        ci, co = in_channels, out_channels
        self.conv1x1 = nn.Sequential(nn.Conv2d(ci, co, kernel_size=1, bias=False), nn.BatchNorm2d(co),
                                     nn.ReLU(inplace=True))
        self.aspp_branches = nn.ModuleList(
            nn.Sequential(nn.Conv2d(ci, co, kernel_size=3, padding=d, dilation=d, bias=False), nn.BatchNorm2d(co),
                          nn.ReLU(inplace=True))
            for d in dilations[1:])
        self.global_pool = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(ci, co, kernel_size=1, bias=False),
                                         nn.BatchNorm2d(co), nn.ReLU(inplace=True))
        self.fusion = nn.Sequential(nn.Conv2d(co * (len(dilations) + 1), co, kernel_size=1, bias=False),
                                    nn.BatchNorm2d(co), nn.ReLU(inplace=True), nn.Dropout(0.1))


class UpBlock(_FusedModule):
    """ConvTranspose2d(k2,s2) then 2 x [conv3x3 -> BN -> ReLU] (reference :254-274).
    HIP: the transposed conv is a GEMM with a pixel-shuffle store."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.up = nn.ConvTranspose2d(in_channels, out_channels, kernel_size=2, stride=2)
        c = out_channels
        self.conv = nn.Sequential(nn.Conv2d(c, c, kernel_size=3, padding=1), nn.BatchNorm2d(c), nn.ReLU(inplace=True),
                                  nn.Conv2d(c, c, kernel_size=3, padding=1), nn.BatchNorm2d(c), nn.ReLU(inplace=True))


class _HipGraphMixin:
    """Caches one packed-weight handle per (device, dtype) and rebuilds it when
    any parameter/buffer changes (load_state_dict, in-place updates, .to())."""

    _ienet_only = False
    _key_prefix = ""

    def _signature(self):
        from upr.autograd import weights_epoch
        return (weights_epoch(),) + tuple((t.data_ptr(), t._version) for t in self.state_dict().values())

    def _run_hip(self, x):
        if not isinstance(x, torch.Tensor) or x.device.type != "cuda":
            dev = x.device if isinstance(x, torch.Tensor) else type(x)
            raise RuntimeError(
                f"{type(self).__name__}.forward: input on '{dev}'. This framework executes UP-Retinex only on "
                f"ROCm devices (gfx950 HIP kernels, no CPU path): use model.to('cuda') and a 'cuda' tensor.")
        if self.training:
            if self._ienet_only:
                from upr.autograd import ienet_train_forward
                return None, None, ienet_train_forward(self, x)
            from upr.autograd import model_train_forward
            return model_train_forward(self, x)
        key = (x.device, x.dtype)
        sig = self._signature()
        cache = self.__dict__.setdefault("_upr_cache", {})
        ent = cache.get(key)
        if ent is None or ent[0] != sig:
            handle = ModelHandle(self.state_dict(), self._use_preact, self._use_aspp, x.dtype, x.device,
                                 ienet_only=self._ienet_only, prefix=self._key_prefix)
            ent = (sig, handle)
            cache[key] = ent
        return ent[1].forward(x)


class ResidualIENet(_HipGraphMixin, nn.Module):
    """Residual illumination estimator (reference :277-360):
    input 3->32, encoder 32->64->128->256 (stride 2), bottleneck (2 blocks, or
    block-ASPP-block), decoder with skip adds, residual head, sigmoid(mean + r)."""

    _ienet_only = True
    _key_prefix = "ie_net."

    def __init__(self, use_preact=False, use_aspp=False):
        super().__init__()
        self._use_preact = bool(use_preact)
        self._use_aspp = bool(use_aspp)
        self.use_aspp = use_aspp
        Block = PreActResBlock if use_preact else ResBlock
        self.input_layer = nn.Conv2d(3, 32, kernel_size=3, padding=1)
        self.enc1 = Block(32, 64, stride=2)
        self.enc2 = Block(64, 128, stride=2)
        self.enc3 = Block(128, 256, stride=2)
        mid = [Block(256, 256)]
        if use_aspp:
            mid.append(ASPPModule(256, 256, dilations=[1, 6, 12, 18]))
        mid.append(Block(256, 256))
        self.bottleneck = nn.Sequential(*mid)
        self.dec3 = UpBlock(256, 128)
        self.dec2 = UpBlock(128, 64)
        self.dec1 = UpBlock(64, 32)
        self.residual_head = nn.Sequential(nn.Conv2d(32, 32, kernel_size=3, padding=1), nn.ReLU(inplace=True),
                                           nn.Conv2d(32, 1, kernel_size=1))
        self.sigmoid = nn.Sigmoid()

    def forward(self, x):
        """x [B,3,H,W] -> illumination [B,1,H,W] (H, W multiples of 8)."""
        return self._run_hip(x)[2]


def _scale_branch(pool):
    layers = [] if pool == 1 else [nn.MaxPool2d(pool)]
    layers += [nn.Conv2d(3, 32, kernel_size=3, padding=1), nn.ReLU(inplace=True), EnhancedFAM(32, 32)]
    return nn.Sequential(*layers)


class MultiScaleUP_Retinex(_HipGraphMixin, nn.Module):
    """UP-Retinex (reference :363-455): illumination I = IENet(X), reflectance
    R = X / (I + 1e-6), 3-scale FAM enhancement map E, Y = R*E + (1-R)*E^2."""

    def __init__(self, use_preact=True, use_aspp=True):
        super().__init__()
        self._use_preact = bool(use_preact)
        self._use_aspp = bool(use_aspp)
        self.ie_net = ResidualIENet(use_preact=use_preact, use_aspp=use_aspp)
        self.scale1 = _scale_branch(1)
        self.scale2 = _scale_branch(2)
        self.scale3 = _scale_branch(4)
        self.fusion = nn.Conv2d(96, 32, kernel_size=1)
        self.output_layer = nn.Conv2d(32, 3, kernel_size=1)

    def retinex_decompose(self, x, illu):
        """Reflectance x / (illu + 1e-6) (reference :405-413); inside forward()
        this is fused into the tail kernel, called on its own it is one device
        kernel (upr_retinex_decompose), differentiable in x and illu."""
        from upr.runtime import retinex_decompose
        return retinex_decompose(x, illu)

    def multi_scale_enhance(self, x, reflectance, illu):
        """Enhanced image from the 3-scale FAM head of x and the given
        reflectance: R*E + (1-R)*E^2 with E = sigmoid(output_layer(fusion(...)))
        (reference :415-443; `illu` is not read there either).  The head has
        no BatchNorm or Dropout, so train and eval mode compute the same values.
        With grad enabled and a reflectance that requires grad (or the model in
        training mode with parameters that require grad) the call is
        differentiable as the reference's is: the head's training graph
        (upr.autograd._HeadStep; float32, H and W multiples of 16) returns
        dL/d reflectance and accumulates the head parameters' gradients.  A
        reflectance that requires grad outside those shapes is refused; in
        training mode alone such a call warns and returns the inference value.  Otherwise
        it runs on the inference kernels (UPR_MODEL_HEAD_ONLY handle) and the
        result records no history.  x gets no gradient (as in forward()): an
        x that requires grad is refused rather than silently detached."""
        from upr.runtime import _require_device
        _require_device(x)
        _require_device(reflectance, "reflectance")
        if torch.is_grad_enabled() and x.requires_grad:
            raise NotImplementedError("multi_scale_enhance: no gradient w.r.t. x (the HIP head differentiates "
                                      "w.r.t. the reflectance and the parameters); pass x.detach()")
        if torch.is_grad_enabled() and (reflectance.requires_grad or
                                        (self.training and any(p.requires_grad for p in self.parameters()))):
            B, C, H, W = x.shape
            ok = (x.dtype == torch.float32 and reflectance.dtype == torch.float32 and H % 16 == 0 and W % 16 == 0
                  and tuple(reflectance.shape) == (B, 3, H, W))
            if ok:
                from upr.autograd import head_train_forward
                return head_train_forward(self, x, reflectance)
            if reflectance.requires_grad:
                raise ValueError(f"multi_scale_enhance: the differentiable head takes float32 x / reflectance "
                                 f"[B,3,H,W] with H, W multiples of 16 (got {tuple(x.shape)} {x.dtype}, "
                                 f"{tuple(reflectance.shape)} {reflectance.dtype}); detach the reflectance for "
                                 f"a value without gradients")
            # training mode, only the parameters would take gradients, and the
            # training graph does not run this shape / dtype: the value from the
            # inference kernels, without history (as before the head was
            # differentiable), and a warning that no gradient is recorded
            import warnings
            warnings.warn(f"multi_scale_enhance: {tuple(x.shape)} {x.dtype} is outside the differentiable head "
                          f"(float32, H, W multiples of 16); returning a value without parameter gradients",
                          RuntimeWarning, stacklevel=2)
        key = ("head", x.device, x.dtype)
        sig = self._signature()
        cache = self.__dict__.setdefault("_upr_cache", {})
        ent = cache.get(key)
        if ent is None or ent[0] != sig:
            ent = (sig, ModelHandle(self.state_dict(), self._use_preact, self._use_aspp, x.dtype, x.device,
                                    head_only=True))
            cache[key] = ent
        return ent[1].enhance(x, reflectance)

    def forward(self, x):
        """x [B,3,H,W] float32/float16 in [0,1] on a ROCm device, H, W multiples
        of 8 -> (enhanced [B,3,H,W], reflectance [B,3,H,W], illumination [B,1,H,W])."""
        return self._run_hip(x)


UP_Retinex = MultiScaleUP_Retinex


def count_parameters(model):
    """Trainable parameter count (reference :462-464)."""
    return sum(p.numel() for p in model.parameters() if p.requires_grad)
