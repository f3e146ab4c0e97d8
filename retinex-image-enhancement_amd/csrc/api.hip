// C ABI of the enhancer kernels (see include/upr.h for the contract of each).
#include <cstring>

#include "upr_common.h"
#include "lab_tables.h"
#include "../../include/upr.h"

namespace upr {
int launch_clahe_pipeline(const void* enh, void* out, uint8_t* ws, int B, int H, int W, float clip, int tilesX,
                          int tilesY, int dtype, hipStream_t st);
size_t clahe_pipeline_ws(int B, int H, int W, int tilesX, int tilesY);
int launch_clahe_u8(const uint8_t* src, uint8_t* dst, uint8_t* lut, int B, int H, int W, float clip, int tilesX,
                    int tilesY, hipStream_t st);
int launch_rgb2lab(const uint8_t* rgb, uint8_t* lab, size_t npix, hipStream_t st);
int launch_lab2rgb(const uint8_t* lab, uint8_t* rgb, size_t npix, hipStream_t st);
int launch_quantize(const void* x, uint8_t* out, size_t n, int dtype, hipStream_t st);
int launch_to_u8_hwc(const void* x, int C, int H, int W, int dtype, uint8_t* out, hipStream_t st);
int launch_letterbox(const void* src, int src_kind, int H, int W, int top, int left, int nh, int nw, int Ho, int Wo,
                     const int* xtab, const int* ytab, int color, void* out, int out_kind, hipStream_t st);
int launch_gray_hist(const void* img, int* hist, int B, int H, int W, int dtype, hipStream_t st);
int launch_multiscale(const void* x, const void* enh, void* out, double* sums, double* factor, int B, int H, int W,
                      int dtype, hipStream_t st);
int launch_ms_features(const void* x, void* out, int B, int H, int W, int scale_idx, int dtype, hipStream_t st);
size_t content_aware_ws(int B, int H, int W);
int launch_content_aware(const void* x, const void* enh, void* out, float* sal_out, float* att_out, uint8_t* ws,
                         int B, int H, int W, int dtype, hipStream_t st);
int launch_decompose(const void* x, const void* illu, void* refl, int B, int C, int HW, int illu_c, int dtype,
                     hipStream_t st);
int launch_decompose_bwd(const void* x, const void* illu, const void* g, void* gx, void* gillu, int B, int C, int HW,
                         int illu_c, int dtype, hipStream_t st);
}  // namespace upr

using namespace upr;

static bool dtype_ok(int dt) { return dt == UPR_F32 || dt == UPR_F16; }

extern "C" {

int upr_quantize_u8(const void* x, uint8_t* out, size_t n, int dtype, void* stream) {
  if (!x || !out || !dtype_ok(dtype)) return UPR_ERR_ARG;
  if (n == 0) return UPR_OK;
  return launch_quantize(x, out, n, dtype, (hipStream_t)stream);
}

int upr_letterbox(const void* src, int src_kind, int H, int W, int top, int left, int nh, int nw, int Ho, int Wo,
                  const int32_t* xtab, const int32_t* ytab, int color, void* out, int out_kind, void* stream) {
  if (!src || !out || (src_kind != 0 && src_kind != 1) || (out_kind != 0 && out_kind != 1)) return UPR_ERR_ARG;
  if (H <= 0 || W <= 0 || nh <= 0 || nw <= 0 || top < 0 || left < 0 || top + nh > Ho || left + nw > Wo)
    return UPR_ERR_SHAPE;
  if ((xtab == nullptr) != (ytab == nullptr)) return UPR_ERR_ARG;
  if (!xtab && (nh != H || nw != W)) return UPR_ERR_SHAPE;
  return launch_letterbox(src, src_kind, H, W, top, left, nh, nw, Ho, Wo, xtab, ytab, color, out, out_kind,
                          (hipStream_t)stream);
}

int upr_to_u8_hwc(const void* x, int C, int H, int W, int dtype, uint8_t* out, void* stream) {
  if (!x || !out || !dtype_ok(dtype) || (C != 1 && C != 3)) return UPR_ERR_ARG;
  if (H <= 0 || W <= 0) return UPR_ERR_SHAPE;
  return launch_to_u8_hwc(x, C, H, W, dtype, out, (hipStream_t)stream);
}

int upr_rgb2lab_u8(const uint8_t* rgb, uint8_t* lab, size_t npix, void* stream) {
  if (!rgb || !lab) return UPR_ERR_ARG;
  if (npix == 0) return UPR_OK;
  return launch_rgb2lab(rgb, lab, npix, (hipStream_t)stream);
}

int upr_lab2rgb_u8(const uint8_t* lab, uint8_t* rgb, size_t npix, void* stream) {
  if (!rgb || !lab) return UPR_ERR_ARG;
  if (npix == 0) return UPR_OK;
  return launch_lab2rgb(lab, rgb, npix, (hipStream_t)stream);
}

int upr_clahe_u8(const uint8_t* src, uint8_t* dst, uint8_t* lut_ws, int B, int H, int W, float clip, int tiles_x,
                 int tiles_y, void* stream) {
  if (!src || !dst || !lut_ws || B <= 0 || H <= 0 || W <= 0 || tiles_x <= 0 || tiles_y <= 0) return UPR_ERR_ARG;
  if (tiles_x > W || tiles_y > H) return UPR_ERR_SHAPE;
  return launch_clahe_u8(src, dst, lut_ws, B, H, W, clip, tiles_x, tiles_y, (hipStream_t)stream);
}

size_t upr_clahe_enhance_workspace(int B, int H, int W, int tiles_x, int tiles_y) {
  if (B <= 0 || H <= 0 || W <= 0 || tiles_x <= 0 || tiles_y <= 0) return 0;
  return clahe_pipeline_ws(B, H, W, tiles_x, tiles_y);
}

int upr_clahe_enhance(const void* enh, void* out, void* workspace, int B, int H, int W, float clip, int tiles_x,
                      int tiles_y, int dtype, void* stream) {
  if (!enh || !out || !workspace || B <= 0 || H <= 0 || W <= 0 || !dtype_ok(dtype)) return UPR_ERR_ARG;
  if (tiles_x <= 0 || tiles_y <= 0 || tiles_x > W || tiles_y > H) return UPR_ERR_SHAPE;
  return launch_clahe_pipeline(enh, out, (uint8_t*)workspace, B, H, W, clip, tiles_x, tiles_y, dtype,
                               (hipStream_t)stream);
}

int upr_gray_hist(const void* x, int32_t* hist, int B, int H, int W, int dtype, void* stream) {
  if (!x || !hist || B <= 0 || H <= 0 || W <= 0 || !dtype_ok(dtype)) return UPR_ERR_ARG;
  return launch_gray_hist(x, hist, B, H, W, dtype, (hipStream_t)stream);
}

int upr_multiscale(const void* x, const void* enh, void* out, double* sums, double* factor, int B, int H, int W,
                   int dtype, void* stream) {
  if (!x || !sums || B <= 0 || H <= 0 || W <= 0 || !dtype_ok(dtype)) return UPR_ERR_ARG;
  if (H < 8 || W < 8) return UPR_ERR_SHAPE;  // torch.gradient needs >= 2 samples at the 1/4 scale
  return launch_multiscale(x, enh, out, sums, factor, B, H, W, dtype, (hipStream_t)stream);
}

int upr_multiscale_features(const void* x, void* out, int B, int H, int W, int scale_idx, int dtype, void* stream) {
  if (!x || !out || B <= 0 || H <= 0 || W <= 0 || scale_idx < 0 || scale_idx > 2 || !dtype_ok(dtype))
    return UPR_ERR_ARG;
  return launch_ms_features(x, out, B, H, W, scale_idx, dtype, (hipStream_t)stream);
}

size_t upr_content_aware_workspace(int B, int H, int W) {
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  return content_aware_ws(B, H, W);
}

int upr_content_aware(const void* x, const void* enh, void* out, float* saliency, float* attention, void* workspace,
                      size_t workspace_bytes, int B, int H, int W, int dtype, void* stream) {
  if (!x || !workspace || B <= 0 || H <= 0 || W <= 0 || !dtype_ok(dtype)) return UPR_ERR_ARG;
  if ((enh == nullptr) != (out == nullptr)) return UPR_ERR_ARG;
  if (workspace_bytes < content_aware_ws(B, H, W)) return UPR_ERR_WORKSPACE;
  return launch_content_aware(x, enh, out, saliency, attention, (uint8_t*)workspace, B, H, W, dtype,
                              (hipStream_t)stream);
}

int upr_retinex_decompose(const void* x, const void* illu, void* refl, int B, int C, int H, int W, int illu_c,
                          int dtype, void* stream) {
  if (!x || !illu || !refl || !dtype_ok(dtype) || B <= 0 || C <= 0 || (illu_c != 1 && illu_c != C)) return UPR_ERR_ARG;
  if (H <= 0 || W <= 0 || (long long)B * H * W * C >= (1LL << 40)) return UPR_ERR_SHAPE;
  return launch_decompose(x, illu, refl, B, C, H * W, illu_c, dtype, (hipStream_t)stream);
}

int upr_retinex_decompose_bwd(const void* x, const void* illu, const void* g, void* gx, void* gillu, int B, int C,
                              int H, int W, int illu_c, int dtype, void* stream) {
  if (!x || !illu || !g || !dtype_ok(dtype) || B <= 0 || C <= 0 || (illu_c != 1 && illu_c != C)) return UPR_ERR_ARG;
  if (H <= 0 || W <= 0) return UPR_ERR_SHAPE;
  if (!gx && !gillu) return UPR_OK;
  return launch_decompose_bwd(x, illu, g, gx, gillu, B, C, H * W, illu_c, dtype, (hipStream_t)stream);
}

void upr_lab_tables(uint16_t* gamma, uint16_t* cbrt, uint16_t* yf, uint16_t* invgamma, int32_t* rgb2xyz,
                    int32_t* xyz2rgb) {
  const LabTables& t = lab_tables();
  if (gamma) memcpy(gamma, t.gamma_b, sizeof(t.gamma_b));
  if (cbrt) memcpy(cbrt, t.cbrt_b, sizeof(t.cbrt_b));
  if (yf) memcpy(yf, t.yf_b, sizeof(t.yf_b));
  if (invgamma) memcpy(invgamma, t.invgamma_b, sizeof(t.invgamma_b));
  if (rgb2xyz) memcpy(rgb2xyz, t.rgb2xyz, sizeof(t.rgb2xyz));
  if (xyz2rgb) memcpy(xyz2rgb, t.xyz2rgb, sizeof(t.xyz2rgb));
}

}  // extern "C"
