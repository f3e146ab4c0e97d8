"""HIP path vs CPU oracle on the MI355X (run with `-m gpu`).

Tolerances: fp32 model outputs |d| <= 1e-3 per pixel (BASELINE.json north_star);
integer/byte enhancer stages bit-exact given the same input; fp16 storage +
fp16 MFMA (fp32 accumulate) reported against the fp32 oracle with its own bound.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import has_gpu
from oracle import cv_u8
from oracle import enhancers as oenh
from oracle import net as onet

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs a ROCm device")]

DEV = "cuda:0"
VARIANTS = [(False, False), (True, False), (False, True), (True, True)]
FP32_TOL = 1e-3
FP16_TOL = 1e-3  # observed 2.5-3.1e-4 (fp16-rounded input to both sides); refl is relative to max(1, max|refl|)


def vname(pre, aspp):
    return f"pre{int(pre)}_aspp{int(aspp)}"


def make_model(pre, aspp, seed=0):
    from models.model import UP_Retinex
    torch.manual_seed(seed)
    return UP_Retinex(use_preact=pre, use_aspp=aspp).eval()


def maxdiff(a, b):
    return (a.detach().float().cpu() - b.detach().float().cpu()).abs().max().item()


# ---------------------------------------------------------------------------
# op level: implicit-GEMM conv vs torch CPU fp32 conv
# ---------------------------------------------------------------------------
CONV_CASES = [
    # B, H, W, Cin, Cout, k, stride, pad, dil, relu, residual
    (2, 16, 16, 32, 32, 3, 1, 1, 1, True, False),
    (2, 16, 24, 32, 64, 3, 2, 1, 1, False, True),
    (1, 20, 12, 64, 128, 3, 1, 2, 2, True, True),
    (2, 8, 8, 256, 256, 3, 1, 6, 6, True, False),
    (1, 16, 16, 128, 256, 1, 2, 0, 1, False, False),
    (3, 7, 9, 32, 96, 1, 1, 0, 1, True, False),
    (1, 9, 11, 96, 32, 3, 1, 1, 1, False, True),
    # shapes routed to the halo-tiled kernel (stride 1, Wo >= 24, Ho >= 8), incl. partial tiles
    (2, 24, 40, 32, 32, 3, 1, 1, 1, True, True),
    (1, 17, 70, 32, 64, 3, 1, 2, 2, False, True),
    (2, 12, 33, 64, 64, 3, 1, 1, 1, True, False),
    (1, 9, 48, 32, 128, 1, 1, 0, 1, False, False),
    (1, 16, 64, 128, 64, 3, 1, 1, 1, True, True),
    (1, 8, 32, 256, 256, 3, 1, 1, 1, False, False),
    # shapes routed to the wide-tile LDS-DMA kernel in fp16 (Cin % 64, Cout % 128), partial tiles
    (3, 20, 28, 64, 128, 3, 2, 1, 1, True, True),
    (2, 30, 34, 256, 256, 3, 1, 12, 12, False, True),
    (1, 17, 23, 128, 512, 1, 1, 0, 1, True, False),
    # shapes routed to the streaming LDS-DMA halo kernel in fp16 (3x3 s1, C 32/64, no pre-ReLU residual)
    (2, 20, 45, 32, 32, 3, 1, 1, 1, True, False),
    (1, 9, 70, 32, 64, 3, 1, 1, 1, False, False),
    (3, 13, 29, 64, 64, 3, 1, 1, 1, True, False),
    # row-ring streaming kernel (fp16): several strips / row bands, partial strips, residual
    (2, 20, 45, 32, 32, 3, 1, 1, 1, False, True),
    (1, 37, 70, 64, 64, 3, 1, 1, 1, False, True),
    (2, 66, 96, 32, 64, 3, 1, 1, 1, True, False),
    (4, 130, 40, 32, 32, 3, 1, 1, 1, True, False),
    (2, 24, 50, 32, 64, 3, 1, 1, 1, False, True),
    # 64-pixel strips (32 -> 32, W >= 48): partial last strip, residual / ReLU
    (2, 20, 100, 32, 32, 3, 1, 1, 1, False, True),
    (1, 33, 150, 32, 32, 3, 1, 1, 1, True, False),
    (2, 20, 100, 64, 64, 3, 1, 1, 1, True, False),   # 64 -> 64, several 32-pixel strips
    # row-ring stride-2 (enc1.conv1 shape class): de-interleaved ring rows, partial strips
    (2, 36, 70, 32, 64, 3, 2, 1, 1, True, False),
    (1, 64, 128, 32, 64, 3, 2, 1, 1, False, False),
    # halo-tiled A operand of the wide kernel (fp16; 3x3 s1 d1, W 64 / 128, tiles of whole rows):
    # BN 256 x W 64 over 4 chunks (region double buffer), BN 128 x W 64, BN 128 x W 128, one chunk
    (2, 64, 64, 256, 256, 3, 1, 1, 1, True, True),
    # statically unrolled halo kernel (hwide4: bottleneck 64x64x256 -> 256): several images, ReLU only
    (3, 64, 64, 256, 256, 3, 1, 1, 1, True, False),
    (1, 64, 64, 256, 512, 3, 1, 1, 1, False, True),
    (1, 32, 64, 128, 128, 3, 1, 1, 1, False, True),
    (2, 16, 128, 128, 128, 3, 1, 1, 1, True, False),
    # runtime-cursor hwide3 (the fallback for W 64 / 128 shapes hwide4 has no program for:
    # 1 or 3 chunks at W 64 x N 256, 3 chunks at W 128)
    (1, 8, 64, 64, 256, 3, 1, 1, 1, False, False),
    (1, 8, 128, 192, 128, 3, 1, 1, 1, True, False),
    (2, 4, 64, 192, 256, 3, 1, 1, 1, False, True),
    # dilated region form of hwide4 (ASPP branches: 3x3, dilation = padding, 256 -> 256 at W 64)
    (2, 64, 64, 256, 256, 3, 1, 6, 6, True, False),
    (1, 64, 64, 256, 256, 3, 1, 18, 18, False, True),
    (1, 32, 64, 256, 512, 3, 1, 12, 12, True, False),
    # pointwise hwide4 (1x1 over whole 64-pixel rows: ASPP conv1x1 K 256, fusion K 1024 / 1280)
    (2, 64, 64, 1024, 256, 1, 1, 0, 1, True, False),
    (1, 16, 64, 256, 512, 1, 1, 0, 1, False, True),
    (3, 12, 64, 1280, 256, 1, 1, 0, 1, False, False),
    # stride-2 hwide4 (de-interleaved region planes, BN 128): W 64 x 4-row tiles over 1 / 2 / 4
    # chunks (enc3.conv1 class), W 128 x 2-row tiles over one chunk (enc2.conv1 class)
    (2, 128, 128, 128, 256, 3, 2, 1, 1, True, False),
    (1, 16, 128, 256, 128, 3, 2, 1, 1, True, False),
    (2, 8, 128, 64, 256, 3, 2, 1, 1, False, False),
    (1, 64, 256, 64, 128, 3, 2, 1, 1, False, True),
    # 64 -> 64 at W 256 (dec2 shape class: the row ring)
    (1, 8, 256, 64, 64, 3, 1, 1, 1, True, False),
    (2, 6, 256, 64, 64, 3, 1, 1, 1, False, True),
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_conv2d_nhwc(case, dtype):
    from upr import runtime
    B, H, W, Cin, Cout, k, s, p, d, relu, res = case
    g = torch.Generator().manual_seed(hash(case) & 0xffff)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=g)
    ref = F.conv2d(x, w, b, s, p, d)
    r = torch.randn_like(ref) if res else None
    if res:
        ref = ref + r
    if relu:
        ref = F.relu(ref)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)
    wd = runtime.pack_conv_weight(w).to(DEV, dtype)
    rd = r.permute(0, 2, 3, 1).contiguous().to(DEV, dtype) if res else None
    y = runtime.conv2d_nhwc(xd, wd, b.to(DEV), k, k, s, p, d, residual=rd, relu=relu)
    torch.cuda.synchronize()
    err = maxdiff(y.permute(0, 3, 1, 2), ref)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert err <= tol, f"conv {case} {dtype}: max|d| {err}"


# ---------------------------------------------------------------------------
# model level: 4 variants at the golden 64x64 B=2 inputs, rect, real crop
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("pre,aspp", VARIANTS)
def test_model_forward_fp32(golden, pre, aspp):
    gd = golden(f"g2_forward_{vname(pre, aspp)}.npz")
    m = make_model(pre, aspp)
    x = torch.from_numpy(gd["x"])
    m = m.to(DEV)
    with torch.no_grad():
        e, r, i = m(x.to(DEV))
    torch.cuda.synchronize()
    assert e.shape == (2, 3, 64, 64) and r.shape == (2, 3, 64, 64) and i.shape == (2, 1, 64, 64)
    assert e.dtype == torch.float32
    for name, a in (("enh", e), ("refl", r), ("illu", i)):
        err = maxdiff(a, torch.from_numpy(gd[name]))
        assert err <= FP32_TOL, f"{vname(pre, aspp)} {name}: {err}"
    if "x_low" in gd:
        with torch.no_grad():
            e, r, i = m(torch.from_numpy(gd["x_low"]).to(DEV))
        assert maxdiff(e, torch.from_numpy(gd["enh_low"])) <= FP32_TOL
        assert maxdiff(i, torch.from_numpy(gd["illu_low"])) <= FP32_TOL


def test_model_forward_rect(golden):
    gd = golden("g2_forward_rect_pre1_aspp1.npz")
    m = make_model(True, True).to(DEV)
    with torch.no_grad():
        e, r, i = m(torch.from_numpy(gd["x"]).to(DEV))
    assert maxdiff(e, torch.from_numpy(gd["enh"])) <= FP32_TOL
    assert maxdiff(r, torch.from_numpy(gd["refl"])) <= FP32_TOL
    assert maxdiff(i, torch.from_numpy(gd["illu"])) <= FP32_TOL


def test_model_real_crop(golden):
    gd = golden("g4_real_crop.npz")
    x = torch.from_numpy(gd["img_u8"].astype(np.float32) / 255.0).permute(2, 0, 1)[None].contiguous()
    m = make_model(False, False).to(DEV)
    with torch.no_grad():
        e, r, i = m(x.to(DEV))
    assert maxdiff(e, torch.from_numpy(gd["enh"])) <= FP32_TOL
    assert maxdiff(i, torch.from_numpy(gd["illu"])) <= FP32_TOL


@pytest.mark.parametrize("pre,aspp", [(False, False), (True, True)])
def test_model_forward_fp16(pre, aspp):
    m = make_model(pre, aspp)
    x = torch.rand(2, 3, 96, 128, generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        ref = onet.forward(m.state_dict(), x.half().float(), pre, aspp)  # same (fp16-rounded) input
        m = m.to(DEV)
        out = m(x.to(DEV).half())
    torch.cuda.synchronize()
    for name, a, b in zip(("enh", "refl", "illu"), out, ref):
        assert a.dtype == torch.float16
        err = maxdiff(a, b) / (1.0 if name != "refl" else max(1.0, b.abs().max().item()))
        print(f"fp16 {vname(pre, aspp)} {name} max|d| = {err:.3e}")
        assert err <= FP16_TOL, f"fp16 {name}: {err}"


def test_ienet_standalone_matches_full():
    m = make_model(True, True).to(DEV)
    x = torch.rand(1, 3, 64, 96, generator=torch.Generator().manual_seed(5)).to(DEV)
    with torch.no_grad():
        _, _, illu = m(x)
        illu2 = m.ie_net(x)
    assert maxdiff(illu, illu2) <= 1e-6


def test_batch_independence():
    """Eval forward is per-image independent (the property batch sharding relies on)."""
    m = make_model(True, True).to(DEV)
    x = torch.rand(4, 3, 64, 64, generator=torch.Generator().manual_seed(6)).to(DEV)
    with torch.no_grad():
        full = m(x)
        parts = [m(x[i:i + 1]) for i in range(4)]
    for k in range(3):
        cat = torch.cat([p[k] for p in parts])
        assert maxdiff(full[k], cat) <= 1e-6


def test_state_change_repacks():
    m = make_model(False, False).to(DEV)
    x = torch.rand(1, 3, 32, 32, generator=torch.Generator().manual_seed(7)).to(DEV)
    with torch.no_grad():
        a = m(x)[0].clone()
        m.output_layer.bias.add_(0.5)
        b = m(x)[0]
        ref = onet.forward({k: v.cpu() for k, v in m.state_dict().items()}, x.cpu(), False, False)[0]
    assert maxdiff(a, b) > 1e-3
    assert maxdiff(b, ref) <= FP32_TOL


def test_bad_shapes_raise():
    m = make_model(False, False).to(DEV)
    with pytest.raises(RuntimeError):
        m(torch.rand(1, 3, 36, 32, device=DEV))  # H % 8 != 0 (reference fails on the skip add too)
    with pytest.raises(RuntimeError):
        m(torch.rand(1, 4, 32, 32, device=DEV))


# ---------------------------------------------------------------------------
# enhancer kernels: bit-exact vs the numpy restatement
# ---------------------------------------------------------------------------
def test_quantize_u8(golden):
    from upr import runtime
    gd = golden("g8_cast_u8.npz")
    q = runtime.quantize_u8(torch.from_numpy(gd["x"]).to(DEV)).cpu().numpy()
    np.testing.assert_array_equal(q, gd["u8"])
    x = torch.randn(100003, generator=torch.Generator().manual_seed(8)) * 3
    q = runtime.quantize_u8(x.to(DEV)).cpu().numpy()
    np.testing.assert_array_equal(q, cv_u8.quantize_u8(x.numpy()))


def test_lab_roundtrip_kernels():
    from upr import runtime
    rng = np.random.default_rng(9)
    rgb = rng.integers(0, 256, (1 << 20, 3)).astype(np.uint8)
    rgb[:8] = [[0, 0, 0], [255, 255, 255], [255, 0, 0], [0, 255, 0], [0, 0, 255], [1, 2, 3], [254, 1, 128],
               [128, 128, 128]]
    lab = runtime.rgb2lab_u8(torch.from_numpy(rgb).to(DEV)).cpu().numpy()
    np.testing.assert_array_equal(lab, cv_u8.rgb2lab_u8(rgb))
    labs = rng.integers(0, 256, (1 << 20, 3)).astype(np.uint8)
    back = runtime.lab2rgb_u8(torch.from_numpy(labs).to(DEV)).cpu().numpy()
    np.testing.assert_array_equal(back, cv_u8.lab2rgb_u8(labs))


@pytest.mark.parametrize("hw", [(64, 64), (256, 256), (100, 75), (31, 45), (512, 384)])
def test_clahe_u8(hw):
    from upr import runtime
    rng = np.random.default_rng(hw[0] * 1000 + hw[1])
    H, W = hw
    imgs = [rng.integers(0, 256, (H, W)).astype(np.uint8),
            np.clip(rng.normal(60, 20, (H, W)), 0, 255).astype(np.uint8),  # low-light, clipping active
            np.full((H, W), 100, np.uint8)]
    src = np.stack(imgs)
    out = runtime.clahe_u8(torch.from_numpy(src).to(DEV)).cpu().numpy()
    for b in range(len(imgs)):
        np.testing.assert_array_equal(out[b], cv_u8.clahe_apply(src[b]), err_msg=f"image {b} {hw}")


def test_clahe_enhance_pipeline():
    from upr import runtime
    g = torch.Generator().manual_seed(10)
    x = torch.rand(2, 3, 64, 80, generator=g) * 0.6
    x[0, :, :4, :4] = 1.2  # wrap-around values
    out = runtime.clahe_enhance(x.to(DEV)).cpu()
    ref = oenh.clahe_enhancement(x)
    assert torch.equal(out, ref), f"max|d| {maxdiff(out, ref)}"


@pytest.mark.parametrize("B,H,W,dt", [
    (1, 512, 512, torch.float32),   # one image: each tile split into 2 row bands (partial histograms + LUT pass)
    (1, 1024, 768, torch.float16),  # 8 bands per tile, fp16 in / out
    (3, 100, 75, torch.float32),    # reflect-padded rows and columns: the 1-pixel item path
    (2, 256, 252, torch.float32),   # W % 8 != 0 (column padding), W % 4 == 0: 4-pixel apply, 1-pixel histogram
    (1, 31, 45, torch.float16),
])
def test_clahe_enhance_shapes(B, H, W, dt):
    """upr_clahe_enhance bit-exact to the OpenCV restatement (oracle/cv_u8.py)
    on every launch form: row-band split histograms (few images), the
    reflect-padded 1-pixel path, fp16 input and output."""
    from upr import runtime
    g = torch.Generator().manual_seed(H * 7 + W)
    x = (torch.rand(B, 3, H, W, generator=g) * 0.7).to(dt)
    out = runtime.clahe_enhance(x.to(DEV)).cpu()
    ref = oenh.clahe_enhancement(x.float())
    assert out.dtype == dt
    assert torch.equal(out, ref.to(dt)), f"max|d| {maxdiff(out.float(), ref)}"


def test_clahe_enhance_full_batch_bs32_512():
    """The bench's enhance workload (bs 32, 512^2, fp32, one histogram block
    per tile with the LUT in the same block): images 0 and 31 bit-exact to
    the restatement, and the batch is per-image independent (image 31 alone
    gives the same bytes)."""
    from upr import runtime
    x = torch.rand(32, 3, 512, 512, generator=torch.Generator().manual_seed(12)) * 0.8
    xd = x.to(DEV)
    out = runtime.clahe_enhance(xd)
    for b in (0, 31):
        ref = oenh.clahe_enhancement(x[b:b + 1])
        assert torch.equal(out[b:b + 1].cpu(), ref), (b, maxdiff(out[b:b + 1].cpu(), ref))
    alone = runtime.clahe_enhance(xd[31:32].contiguous())
    assert torch.equal(alone, out[31:32])


def test_gray_hist():
    from upr import runtime
    x = torch.rand(3, 3, 50, 70, generator=torch.Generator().manual_seed(11))
    h = runtime.gray_hist(x.to(DEV)).cpu().numpy()
    for b in range(3):
        gray = cv_u8.rgb_to_gray_u8(cv_u8.quantize_u8(x[b].permute(1, 2, 0).numpy()))
        np.testing.assert_array_equal(h[b], np.bincount(gray.reshape(-1), minlength=256))


def test_multiscale_kernel(golden):
    from upr import runtime
    gd = golden("g5_multiscale.npz")
    for tag in ("a", "b"):
        x = torch.from_numpy(gd[f"{tag}_x"]).to(DEV)
        _, factor, _ = runtime.multiscale(x)
        assert abs(factor.item() - float(gd[f"{tag}_factor"])) < 1e-6
    x = torch.rand(3, 3, 64, 48, generator=torch.Generator().manual_seed(12))
    enh = torch.rand_like(x)
    out, factor, _ = runtime.multiscale(x.to(DEV), enh.to(DEV))
    fac = oenh.multiscale_factor(x)
    for b in range(3):
        assert abs(factor[b].item() - fac[b]) < 1e-6
        ref = torch.clamp(enh[b] * fac[b], 0, 1)
        assert maxdiff(out[b], ref) <= 1e-6


@pytest.mark.parametrize("B,H,W,dtype", [
    (2, 100, 136, torch.float32),   # single pass (H, W % 4 == 0), partial 32 x 64 tiles
    (1, 8, 8, torch.float32),       # smallest: 2 x 2 quarter scale inside one tile
    (3, 66, 50, torch.float32),     # H % 4 != 0: the three-launch path
    (2, 96, 128, torch.float16),    # fp16 input, single pass
    (32, 512, 512, torch.float32),  # the bench's enhance leg (images 0 and 31 checked)
])
def test_multiscale_single_pass(B, H, W, dtype):
    """upr_multiscale's one-pass kernel (ms_rows1_kernel: all three scales from
    one read of each colour plane, per-wave partials added in order by
    ms_fin1_kernel) vs the
    oracle's per-image factor (multi_scale.py:62-100), called three times in a
    row (the three results must be bit-identical)."""
    from upr import runtime
    x = torch.rand(B, 3, H, W, generator=torch.Generator().manual_seed(21)).to(dtype)
    enh = torch.rand(B, 3, H, W, generator=torch.Generator().manual_seed(22)).to(dtype)
    xd, ed = x.to(DEV), enh.to(DEV)
    runs = [runtime.multiscale(xd, ed) for _ in range(3)]
    torch.cuda.synchronize()
    idx = [0, B - 1] if B > 1 else [0]
    fac = oenh.multiscale_factor(x[idx].float())
    out0, f0, s0 = runs[0]
    for out, f, sm in runs[1:]:
        assert torch.equal(f, f0) and torch.equal(sm, s0) and torch.equal(out, out0)
    for j, b in enumerate(idx):
        assert abs(f0[b].item() - fac[j]) < 1e-6, (b, f0[b].item(), fac[j])
        ref = torch.clamp(enh[b].float() * fac[j], 0, 1)
        assert maxdiff(out0[b].float(), ref) <= (1e-6 if dtype == torch.float32 else 1e-3)


@pytest.mark.parametrize("B,H,W,dtype", [
    (1, 64, 520, torch.float32),    # three 256-column strips, the last one 8 pixels wide
    (2, 36, 300, torch.float32),    # partial 16-row band, partial strip
    (2, 100, 136, torch.float32),
    (1, 48, 256, torch.float16),
    (1, 16, 1024, torch.float32),   # one band, four strips: every strip edge interior
])
def test_multiscale_sums_vs_feature_maps(B, H, W, dtype):
    """The per-scale feature sums of upr_multiscale's one-pass kernel
    (ms_rows1_kernel: one colour plane's 256-column strip walked row by row
    in registers per wave, the strip-edge neighbours from the edge lanes'
    extra quads; the luminance sum formed from the planes' sums) against the fp64
    sums of the oracle's seven feature maps per scale (multi_scale.py:17-60):
    per pixel the features agree to the gradient magnitude's square root
    (hardware, <= 1 ulp), so the sums to 1e-6 relative -- a wrong neighbour
    column at one strip edge moves them by ~1e-5."""
    from upr import runtime
    x = torch.rand(B, 3, H, W, generator=torch.Generator().manual_seed(H + W)).to(dtype)
    _, _, sums = runtime.multiscale(x.to(DEV))
    torch.cuda.synchronize()
    for b in range(B):
        feats = oenh.multiscale_features(x[b:b + 1].float())
        for i, f in enumerate(feats):
            ref = f.double().sum().item()
            got = sums[b, i].item()
            assert abs(got - ref) <= 1e-6 * abs(ref), (b, i, got, ref)


# ---------------------------------------------------------------------------
# full-size configs (BASELINE.json configs[1..3]): the whole batch runs on the
# GPU, the oracle checks the first and the last image of the batch (direct
# per-pixel parity at full size; the last image exercises the largest offsets)
# ---------------------------------------------------------------------------
FULL_CASES = [
    # B, size, pre, aspp, dtype
    (32, 512, False, False, torch.float32),   # configs[1]
    (32, 512, True, True, torch.float16),     # configs[2]
    (4, 512, False, False, torch.float16),    # plain fp16 (ResBlock enc2.conv2 + shortcut on hwide4)
    (32, 1024, True, True, torch.float32),    # configs[3] per-GPU shard
    (32, 1024, True, True, torch.float16),
]


@pytest.mark.parametrize("case", FULL_CASES, ids=lambda c: f"B{c[0]}_{c[1]}_pre{int(c[2])}aspp{int(c[3])}_{str(c[4])[6:]}")
def test_full_size_config(case):
    B, S, pre, aspp, dt = case
    m = make_model(pre, aspp)
    sd = m.state_dict()
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.rand(B, 3, S, S, generator=g, device=DEV)
    m = m.to(DEV)
    with torch.no_grad():
        out = m(x.to(dt))
    torch.cuda.synchronize()
    for k, o in enumerate(out):
        assert torch.isfinite(o).all(), f"non-finite output {k}"
    tol = FP32_TOL if dt == torch.float32 else FP16_TOL
    for b in (0, B - 1):
        with torch.no_grad():
            ref = onet.forward(sd, x[b:b + 1].to(dt).float().cpu(), pre, aspp)
        for name, a, r in zip(("enh", "refl", "illu"), out, ref):
            err = maxdiff(a[b:b + 1], r)
            if name == "refl" and dt == torch.float16:
                err /= max(1.0, r.abs().max().item())
            print(f"B{B} {S}^2 {dt} image {b} {name} max|d| = {err:.3e}")
            assert err <= tol, f"image {b} {name}: {err}"
    del out, x
    torch.cuda.empty_cache()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_forward_deterministic(dtype):
    """Two forwards of the same batch are bit-for-bit equal (the pool sums are
    fixed-point integer atomics), for both precisions and at a size where each
    image's FAM / ASPP pool sums gather many tiles."""
    m = make_model(True, True).to(DEV)
    if dtype == torch.float16:
        m = m.half()
    g = torch.Generator(device=DEV).manual_seed(21)
    x = torch.rand(4, 3, 256, 256, generator=g, device=DEV).to(dtype)
    with torch.no_grad():
        a = [t.clone() for t in m(x)]
        b = m(x)
    torch.cuda.synchronize()
    for u, v in zip(a, b):
        assert torch.equal(u, v)


def test_two_streams_distinct_handles():
    """Two models (distinct handles) forwarding concurrently on two HIP streams:
    each stream gets its own workspace (upr/runtime.py _Workspace), so the
    results equal the serial ones bit for bit (include/upr.h threading rule;
    the per-image pool sums of the EnhancedFAM channel attention and the ASPP
    global branch are 64-bit fixed-point integer atomics, independent of the
    order tiles finish in), where a shared workspace would corrupt whole
    activations."""
    m1 = make_model(False, False).to(DEV)
    m2 = make_model(True, True).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(13)
    x1 = torch.rand(4, 3, 128, 128, generator=g, device=DEV)
    x2 = torch.rand(2, 3, 256, 192, generator=g, device=DEV)
    with torch.no_grad():
        r1 = [t.clone() for t in m1(x1)]
        r2 = [t.clone() for t in m2(x2)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    s2.wait_stream(torch.cuda.current_stream())
    with torch.no_grad():
        for _ in range(3):
            with torch.cuda.stream(s1):
                o1 = m1(x1)
            with torch.cuda.stream(s2):
                o2 = m2(x2)
    torch.cuda.synchronize()
    for name, o, r in (("plain", o1, r1), ("preact+aspp", o2, r2)):
        for a, b in zip(o, r):
            print(f"two streams: {name} max|d| vs serial {maxdiff(a, b):.2e}")
            assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_multiscale_side_stream_matches_serial(dtype):
    """The executor runs the multi-scale ops (scale pyramid, scale2/3 first
    convs, the three EnhancedFAM blocks) on a side stream forked before the
    bottleneck and joined before the Retinex tail (csrc/model.hip side_of); a
    profiled forward (upr_model_profile) keeps every op on the caller's stream.
    Both orders give bit-identical outputs, on the default stream and on a
    non-default caller stream, for repeated forwards of different batches
    (a missing fork / join edge would read a half-written buffer).  Every
    model forks by default (fp32 too since round 5); under UPR_MS_STREAMS=0
    this is the serial order twice."""
    m = make_model(True, True).to(DEV)
    if dtype == torch.float16:
        m = m.half()
    g = torch.Generator(device=DEV).manual_seed(5)
    xs = [torch.rand(4, 3, 256, 256, generator=g, device=DEV).to(dtype) for _ in range(2)]
    with torch.no_grad():
        m(xs[0])
        handle = next(iter(m.__dict__["_upr_cache"].values()))[1]
        handle.profile(True)
        serial = [[t.clone() for t in m(x)] for x in xs]
        handle.profile(False)
        n0 = handle.forks()
        forked = [[t.clone() for t in m(x)] for x in xs]
        # models fork on torch's default (null) stream too (unless
        # UPR_MS_STREAMS=0), not only on an explicit caller stream
        import os
        env = os.environ.get("UPR_MS_STREAMS")
        want = True if env is None else (int(env) != 0)
        assert handle.forks() - n0 == (len(xs) if want else 0)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            on_s = [[t.clone() for t in m(x)] for x in xs for _ in range(2)][::2]
    torch.cuda.synchronize()
    for i in range(len(xs)):
        for a, b, c in zip(serial[i], forked[i], on_s[i]):
            assert torch.equal(a, b)
            assert torch.equal(a, c)
