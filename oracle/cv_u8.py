"""numpy restatement of the OpenCV 8-bit arithmetic the reference enhancers call.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Third-party dependency: OpenCV (`cv2`, package opencv-python) — imported by
enhancers/adaptive_params.py:8, enhancers/content_aware.py:8, utils/letterbox.py:5;
NOT installed in the build container, not vendored, and its version is pinned
nowhere (requirements.txt omits it).  What is restated here is OpenCV 4.x's
published algorithm:
  * cvtColor BGR2GRAY 8U  (imgproc/src/color_rgb / color.hpp: yuv_shift 14)
  * cvtColor BGR2Lab / Lab2BGR 8U, sRGB (imgproc/src/color_lab.cpp: RGB2Lab_b,
    Lab2RGBinteger, initLabTabs) — bit-exact integer path
  * CLAHE 8U (imgproc/src/clahe.cpp: CLAHE_Impl::apply, CLAHE_CalcLut_Body,
    CLAHE_Interpolation_Body)
  * Laplacian ksize=1 CV_64F, GaussianBlur 15x15 sigma=0 on CV_64F, both with
    BORDER_REFLECT_101 (imgproc/src/deriv.cpp, smooth.dispatch.cpp)
Parity with cv2 itself is UNPINNED (no cv2 to generate vectors from); the
restatement is pinned by hand-derived known-answer tests in
tests/test_cpu_cv_oracle.py.
"""

import numpy as np

F32 = np.float32


def _round_half_even(v):
    return int(np.rint(v))


# ---------------------------------------------------------------------------
# float -> u8 cast of the reference: (x * 255).astype(np.uint8) on float32
# (enhancers/adaptive_params.py:142, content_aware.py:40, letterbox.py:93)
# ---------------------------------------------------------------------------
def quantize_u8(x):
    x = np.asarray(x, dtype=np.float32)
    t = (x * np.float32(255)).astype(np.float32)
    out = np.zeros(t.shape, np.uint8)
    ok = np.isfinite(t) & (np.abs(t) < 2.0 ** 31)
    out[ok] = (np.trunc(t[ok]).astype(np.int64) & 255).astype(np.uint8)
    return out


# ---------------------------------------------------------------------------
# gray (COLOR_BGR2GRAY / RGB2GRAY, 8U): (B*1868 + G*9617 + R*4899 + 2^13) >> 14
# ---------------------------------------------------------------------------
def rgb_to_gray_u8(rgb):
    rgb = np.asarray(rgb).astype(np.int64)
    r, g, b = rgb[..., 0], rgb[..., 1], rgb[..., 2]
    return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)


# ---------------------------------------------------------------------------
# Lab tables (initLabTabs).  softfloat -> float32, softdouble -> float64.
# ---------------------------------------------------------------------------
def _gamma(x):
    return x / (323.0 / 25.0) if x <= 809.0 / 20000.0 else ((x + 11.0 / 200.0) / (1.0 + 11.0 / 200.0)) ** (12.0 / 5.0)


def _inv_gamma(x):
    return x * (323.0 / 25.0) if x <= 7827.0 / 2500000.0 else \
        x ** (1.0 / (12.0 / 5.0)) * (1.0 + 11.0 / 200.0) - 11.0 / 200.0


def _fma32(a, b, c):
    return F32(float(np.float64(a) * np.float64(b) + np.float64(c)))  # exact product, one rounding


_TABLES = None


def lab_tables():
    global _TABLES
    if _TABLES is not None:
        return _TABLES
    f255 = F32(255)
    gamma_b = np.zeros(256, np.uint16)
    for i in range(256):
        x = F32(F32(i) / f255)
        g = F32(_gamma(float(x)))
        gamma_b[i] = _round_half_even(float(F32(F32(2040) * g)))
    lthresh, lscale, lbias = F32(F32(216) / F32(24389)), F32(F32(841) / F32(108)), F32(F32(16) / F32(116))
    cbscale = F32(F32(1) / F32(f255 * F32(8)))
    cbrt_b = np.zeros(3072, np.uint16)
    for i in range(3072):
        x = F32(cbscale * F32(i))
        f = _fma32(x, lscale, lbias) if x < lthresh else F32(np.cbrt(np.float64(x)))
        cbrt_b[i] = _round_half_even(float(F32(F32(32768) * f)))
    invgamma_b = np.zeros(4096, np.uint16)
    for i in range(4096):
        x = F32(F32(1.0 / 4096) * F32(i))
        g = F32(_inv_gamma(float(x)))
        invgamma_b[i] = _round_half_even(float(F32(f255 * g)))
    BASE = 1 << 14
    yf_b = np.zeros(512, np.uint16)
    for i in range(256):
        if i <= 20:
            y = _round_half_even(float(F32(F32(i * BASE * 20 * 9) / F32(17 * 29 * 29 * 29))))
            ify = _round_half_even(float(F32(F32(BASE) * F32(F32(F32(16) / F32(116)) +
                                                             F32(F32(i * 5) / F32(3 * 17 * 29))))))
        else:
            fy = F32(F32(F32(i * 100 * BASE) / F32(255 * 116)) + F32(F32(16 * BASE) / F32(116)))
            ify = _round_half_even(float(fy))
            y = _round_half_even(float(F32(F32(F32(fy * fy) * fy) / F32(BASE * BASE))))
        yf_b[2 * i], yf_b[2 * i + 1] = y, ify
    rgb2xyz = np.array([0.412453, 0.357580, 0.180423, 0.212671, 0.715160, 0.072169, 0.019334, 0.119193, 0.950227])
    xyz2rgb = np.array([3.240479, -1.53715, -0.498535, -0.969256, 1.875991, 0.041556, 0.055648, -0.204043, 1.057311])
    wp = [0.950456, 1.0, 1.088754]
    m1 = np.array([_round_half_even(4096.0 * rgb2xyz[r * 3 + c] / wp[r]) for r in range(3) for c in range(3)],
                  np.int32)
    m2 = np.array([_round_half_even(4096.0 * xyz2rgb[r * 3 + c] * wp[c]) for r in range(3) for c in range(3)],
                  np.int32)
    _TABLES = {"gamma": gamma_b, "cbrt": cbrt_b, "yf": yf_b, "invgamma": invgamma_b, "rgb2xyz": m1, "xyz2rgb": m2}
    return _TABLES


def _descale(x, n):
    return (x + (1 << (n - 1))) >> n


def rgb2lab_u8(rgb):
    """RGB2Lab_b::operator() on uint8 [..., 3] (R, G, B order)."""
    T = lab_tables()
    a = np.asarray(rgb).astype(np.int64)
    R, G, B = (T["gamma"][a[..., i]].astype(np.int64) for i in range(3))
    c = T["rgb2xyz"].astype(np.int64)
    fX = T["cbrt"][_descale(R * c[0] + G * c[1] + B * c[2], 12)].astype(np.int64)
    fY = T["cbrt"][_descale(R * c[3] + G * c[4] + B * c[5], 12)].astype(np.int64)
    fZ = T["cbrt"][_descale(R * c[6] + G * c[7] + B * c[8], 12)].astype(np.int64)
    Lscale = (116 * 255 + 50) // 100
    Lshift = -((16 * 255 * (1 << 15) + 50) // 100)
    L = _descale(Lscale * fY + Lshift, 15)
    A = _descale(500 * (fX - fY) + 128 * (1 << 15), 15)
    Bb = _descale(200 * (fY - fZ) + 128 * (1 << 15), 15)
    return np.clip(np.stack([L, A, Bb], -1), 0, 255).astype(np.uint8)


def _c_div(a, b):
    """C integer division (truncation toward zero) on int64 arrays."""
    q = np.abs(a) // abs(b)
    return np.where((a < 0) ^ (b < 0), -q, q)


def _ab_to_xz(v):
    BASE = 1 << 14
    lo = _c_div(v * 108, 841) - (BASE * 16 // 116 * 108 // 841)
    hi = _c_div(_c_div(v * v, BASE) * v, BASE)
    return np.where(v <= 3390, lo, hi)


def lab2rgb_u8(lab):
    """Lab2RGBinteger::process on uint8 [..., 3] (L, a, b) -> RGB uint8."""
    T = lab_tables()
    a = np.asarray(lab).astype(np.int64)
    L, A, Bb = a[..., 0], a[..., 1], a[..., 2]
    BASE = 1 << 14
    y = T["yf"][2 * L].astype(np.int64)
    ify = T["yf"][2 * L + 1].astype(np.int64)
    adiv = ((5 * A * 53687 + (1 << 7)) >> 13) - 128 * BASE // 500
    bdiv = ((Bb * 41943 + (1 << 4)) >> 9) - 128 * BASE // 200 + 1
    x = _ab_to_xz(ify + adiv)
    z = _ab_to_xz(ify - bdiv)
    c = T["xyz2rgb"].astype(np.int64)
    out = []
    for r in range(3):
        v = _descale(c[3 * r] * x + c[3 * r + 1] * y + c[3 * r + 2] * z, 14)
        v = np.clip(v, 0, 4095)
        out.append(T["invgamma"][v])
    return np.stack(out, -1).astype(np.uint8)


# ---------------------------------------------------------------------------
# CLAHE (clahe.cpp), 8-bit, one image [H, W]
# ---------------------------------------------------------------------------
def _reflect101(i, n):
    if n == 1:
        return np.zeros_like(i)
    i = np.abs(i)
    period = 2 * (n - 1)
    i = i % period
    return np.where(i >= n, period - i, i)


def clahe_luts(src, clip=2.0, tiles=(8, 8)):
    src = np.asarray(src, np.uint8)
    H, W = src.shape
    tx_n, ty_n = tiles
    Hp = H + (ty_n - H % ty_n) if H % ty_n else H
    Wp = W + (tx_n - W % tx_n) if W % tx_n else W
    tw, th = Wp // tx_n, Hp // ty_n
    if Hp != H or Wp != W:
        ry = _reflect101(np.arange(Hp), H)
        rx = _reflect101(np.arange(Wp), W)
        ext = src[ry][:, rx]
    else:
        ext = src
    area = tw * th
    lut_scale = F32(F32(255) / F32(area))
    clip_limit = 0
    if clip > 0:
        clip_limit = max(int(clip * area / 256), 1)
    luts = np.zeros((ty_n * tx_n, 256), np.uint8)
    for ty in range(ty_n):
        for tx in range(tx_n):
            tile = ext[ty * th:(ty + 1) * th, tx * tw:(tx + 1) * tw]
            hist = np.bincount(tile.reshape(-1), minlength=256).astype(np.int64)
            if clip_limit > 0:
                over = np.maximum(hist - clip_limit, 0)
                clipped = int(over.sum())
                hist = np.minimum(hist, clip_limit)
                batch = clipped // 256
                residual = clipped - batch * 256
                hist += batch
                if residual:
                    step = max(256 // residual, 1)
                    i = 0
                    while i < 256 and residual > 0:
                        hist[i] += 1
                        i += step
                        residual -= 1
            cdf = np.cumsum(hist)
            v = (cdf.astype(np.float32) * lut_scale).astype(np.float32)
            luts[ty * tx_n + tx] = np.clip(np.rint(v), 0, 255).astype(np.uint8)
    return luts, tw, th


def clahe_apply(src, clip=2.0, tiles=(8, 8)):
    src = np.asarray(src, np.uint8)
    H, W = src.shape
    tx_n, ty_n = tiles
    luts, tw, th = clahe_luts(src, clip, tiles)
    inv_tw = F32(F32(1) / F32(tw))
    inv_th = F32(F32(1) / F32(th))
    x = np.arange(W, dtype=np.float32)
    txf = (x * inv_tw).astype(np.float32) - F32(0.5)
    tx1 = np.floor(txf).astype(np.int64)
    xa = (txf - tx1.astype(np.float32)).astype(np.float32)
    xa1 = (F32(1) - xa).astype(np.float32)
    tx2 = np.minimum(tx1 + 1, tx_n - 1)
    tx1 = np.maximum(tx1, 0)
    out = np.zeros_like(src)
    for y in range(H):
        tyf = F32(F32(F32(y) * inv_th) - F32(0.5))
        ty1 = int(np.floor(tyf))
        ya = F32(tyf - F32(ty1))
        ya1 = F32(F32(1) - ya)
        ty2 = min(ty1 + 1, ty_n - 1)
        ty1 = max(ty1, 0)
        v = src[y].astype(np.int64)
        l11 = luts[ty1 * tx_n + tx1, v].astype(np.float32)
        l12 = luts[ty1 * tx_n + tx2, v].astype(np.float32)
        l21 = luts[ty2 * tx_n + tx1, v].astype(np.float32)
        l22 = luts[ty2 * tx_n + tx2, v].astype(np.float32)
        top = (l11 * xa1).astype(np.float32) + (l12 * xa).astype(np.float32)
        bot = (l21 * xa1).astype(np.float32) + (l22 * xa).astype(np.float32)
        res = (top.astype(np.float32) * ya1).astype(np.float32) + (bot.astype(np.float32) * ya).astype(np.float32)
        out[y] = np.clip(np.rint(res.astype(np.float32)), 0, 255).astype(np.uint8)
    return out


# ---------------------------------------------------------------------------
# Laplacian(ksize=1, CV_64F) and GaussianBlur((15,15), 0) on CV_64F,
# BORDER_REFLECT_101 (content_aware.py:46, :50)
# ---------------------------------------------------------------------------
def _pad101(a, p):
    H, W = a.shape
    ry = _reflect101(np.arange(-p, H + p), H)
    rx = _reflect101(np.arange(-p, W + p), W)
    return a[ry][:, rx]


def laplacian_k1_f64(gray):
    g = _pad101(np.asarray(gray, np.float64), 1)
    return g[:-2, 1:-1] + g[2:, 1:-1] + g[1:-1, :-2] + g[1:-1, 2:] - 4.0 * g[1:-1, 1:-1]


def gaussian_kernel_f64(ksize, sigma):
    if sigma <= 0:
        sigma = ((ksize - 1) * 0.5 - 1) * 0.3 + 0.8
    scale2x = -0.5 / (sigma * sigma)
    k = np.zeros(ksize, np.float64)
    s = 0.0
    for i in range(ksize):  # getGaussianKernel: t = exp(scale2X*x*x); sum; cd *= 1/sum
        x = i - (ksize - 1) * 0.5
        k[i] = np.exp(scale2x * x * x)
        s += k[i]
    return k * (1.0 / s)


def gaussian_blur_f64(img, ksize=15, sigma=0.0):
    """sepFilter2D order: RowFilter (taps left to right), then SymmColumnFilter
    (centre tap first, then k[c+j] * (S[y+j] + S[y-j]))."""
    k = gaussian_kernel_f64(ksize, sigma)
    p = ksize // 2
    a = _pad101(np.asarray(img, np.float64), p)
    H, W = np.asarray(img).shape
    tmp = k[0] * a[:, 0:W]
    for j in range(1, ksize):
        tmp = tmp + k[j] * a[:, j:j + W]
    out = k[p] * tmp[p:p + H, :] + 0.0
    for j in range(1, p + 1):
        out = out + k[p + j] * (tmp[p + j:p + j + H, :] + tmp[p - j:p - j + H, :])
    return out
