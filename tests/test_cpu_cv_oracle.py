"""Hand-derived known-answer tests pinning the numpy OpenCV restatement
(oracle/cv_u8.py).  cv2 is absent, so these plus OpenCV's documented values
are the only anchors ("parity unpinned" against cv2 itself)."""
import numpy as np

from oracle import cv_u8


def test_gray_known_values():
    px = np.array([[0, 0, 0], [255, 255, 255], [255, 0, 0], [0, 255, 0], [0, 0, 255], [10, 20, 30]], np.uint8)
    # (B*1868 + G*9617 + R*4899 + 8192) >> 14
    assert cv_u8.rgb_to_gray_u8(px).tolist() == [0, 255, 76, 150, 29, 18]


def test_lab_known_values():
    # OpenCV 8-bit Lab of the sRGB primaries / greys (documented cvtColor results)
    px = np.array([[255, 255, 255], [0, 0, 0], [255, 0, 0], [0, 255, 0], [0, 0, 255], [128, 128, 128]], np.uint8)
    lab = cv_u8.rgb2lab_u8(px)
    assert lab.tolist() == [[255, 128, 128], [0, 128, 128], [136, 208, 195], [224, 42, 211], [82, 207, 20],
                            [137, 128, 128]]
    back = cv_u8.lab2rgb_u8(lab)
    assert back[0].tolist() == [255, 255, 255] and back[1].tolist() == [0, 0, 0]
    assert back[5].tolist() == [128, 128, 128]


def test_lab_roundtrip_greys_and_error_bound():
    g = np.repeat(np.arange(256, dtype=np.uint8)[:, None], 3, 1)
    rt = cv_u8.lab2rgb_u8(cv_u8.rgb2lab_u8(g)).astype(int)
    assert np.abs(rt - g).max() <= 1          # neutral axis survives the 8-bit round trip
    lab = cv_u8.rgb2lab_u8(g)
    assert (lab[:, 1] == 128).all() and (lab[:, 2] == 128).all()
    assert (np.diff(lab[:, 0].astype(int)) >= 0).all()


def test_clahe_constant_image():
    # 512x512, 8x8 tiles -> 64x64 tiles, area 4096, clip = int(2*4096/256) = 32.
    # constant 100: excess 4064 -> 15 per bin + 1 for bins 0..223; cdf[100] = 16*100 + 48 = 1648
    # LUT[100] = round(1648 * 255/4096) = 103, identical in every tile -> constant output 103.
    img = np.full((512, 512), 100, np.uint8)
    out = cv_u8.clahe_apply(img)
    assert (out == 103).all()


def test_clahe_single_tile_is_lut_lookup():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (40, 40)).astype(np.uint8)
    luts, tw, th = cv_u8.clahe_luts(img, 2.0, (1, 1))
    assert (tw, th) == (40, 40)
    np.testing.assert_array_equal(cv_u8.clahe_apply(img, 2.0, (1, 1)), luts[0][img])


def test_clahe_no_clip_is_equalisation():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (32, 32)).astype(np.uint8)
    luts, _, _ = cv_u8.clahe_luts(img, 0.0, (1, 1))
    hist = np.bincount(img.ravel(), minlength=256)
    expect = np.clip(np.rint(np.cumsum(hist).astype(np.float32) * np.float32(255.0 / 1024)), 0, 255)
    np.testing.assert_array_equal(luts[0], expect.astype(np.uint8))


def test_clahe_odd_sizes_use_reflect101_extension():
    # 37 x 45: rows/cols are extended by BORDER_REFLECT_101 to 40 x 48 for the tile histograms
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (37, 45)).astype(np.uint8)
    luts, tw, th = cv_u8.clahe_luts(img)
    assert (tw, th) == (6, 5)
    ry = [r if r < 37 else 2 * 36 - r for r in range(40)]
    rx = [c if c < 45 else 2 * 44 - c for c in range(48)]
    ext = img[ry][:, rx]
    luts_ext, _, _ = cv_u8.clahe_luts(ext)
    np.testing.assert_array_equal(luts, luts_ext)
    # a horizontal ramp stays monotone inside each tile row where only one LUT column applies
    ramp = np.tile(np.arange(0, 256, 2, dtype=np.uint8), (16, 1))  # 16 x 128, 16-px tiles
    out = cv_u8.clahe_apply(ramp, 2.0, (1, 1))
    assert (np.diff(out.astype(int), axis=1) >= 0).all()


def test_clahe_redistribution_residual():
    # one tile, all pixels in bin 0: clipped = area - clip; residual spread with step max(256//r, 1)
    img = np.zeros((16, 16), np.uint8)
    luts, _, _ = cv_u8.clahe_luts(img, 2.0, (1, 1))
    area, clip = 256, 2
    excess = area - clip
    batch, resid = excess // 256, excess % 256
    hist = np.full(256, batch)
    hist[0] += clip
    step = max(256 // resid, 1)
    for i in range(0, 256, step)[:resid]:
        hist[i] += 1
    expect = np.clip(np.rint(np.cumsum(hist).astype(np.float32) * np.float32(255.0 / 256)), 0, 255)
    np.testing.assert_array_equal(luts[0], expect.astype(np.uint8))


def test_laplacian_and_gaussian():
    img = np.zeros((9, 9), np.uint8)
    img[4, 4] = 10
    lap = cv_u8.laplacian_k1_f64(img)
    assert lap[4, 4] == -40 and lap[3, 4] == 10 and lap[4, 3] == 10 and lap[0, 0] == 0
    k = cv_u8.gaussian_kernel_f64(15, 0)
    assert abs(k.sum() - 1) < 1e-15 and np.allclose(k, k[::-1])
    sigma = ((15 - 1) * 0.5 - 1) * 0.3 + 0.8
    assert abs(sigma - 2.6) < 1e-12
    flat = cv_u8.gaussian_blur_f64(np.full((20, 20), 3.0))
    assert np.allclose(flat, 3.0, atol=1e-12)
