/*
 * upr.h — C ABI of libupr.so, the MI355X (gfx950) UP-Retinex kernel library.
 *
 * The reference (xh92117/Retinex-image-Enhancement) has no native code and no
 * FFI: its hot path is the Python/PyTorch surface below.  Each entry point
 * names the reference interface it replaces (file:line, relative to the
 * reference root).  Conventions:
 *   - every buffer is caller-allocated device memory unless stated otherwise
 *     (params of upr_model_create are HOST fp32 arrays); the library never
 *     frees caller memory;
 *   - `stream` is a hipStream_t passed as void*; launches are stream-ordered
 *     and never synchronise internally;
 *   - images are NCHW with C = 3 (the reference's tensor layout), dtype
 *     UPR_F32 (float) or UPR_F16 (IEEE half);
 *   - return 0 on success, a hipError_t value (> 0) passed through, or a
 *     negative UPR_ERR_* code; upr_status_string() describes either.
 * Thread safety: distinct models / streams may be used concurrently; one model
 * handle must not be used on two streams at once.  A forward (fp32 or fp16;
 * UPR_MS_STREAMS=0 turns it off) forks its multi-scale head onto a side stream
 * of the library's own, keyed by (device, caller stream), with fork / join
 * events of that side.  NULL is treated as the one legacy stream: it forks
 * too, and two threads forwarding on NULL share one side stream and its
 * events, so a handle -- or two handles -- must not be used from two threads
 * on NULL at once.  hipStreamPerThread (a different real stream per thread)
 * never forks: such forwards run on the one stream.
 */
#ifndef UPR_H_
#define UPR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { UPR_F32 = 0, UPR_F16 = 1 };

enum {
  UPR_OK = 0,
  UPR_ERR_ARG = -1,
  UPR_ERR_SHAPE = -2,
  UPR_ERR_MISSING_PARAM = -3,
  UPR_ERR_WORKSPACE = -4,
  UPR_ERR_UNSUPPORTED = -5
};

/* model flags: UPR_MODEL_IENET_ONLY = ResidualIENet alone; UPR_MODEL_HEAD_ONLY =
 * MultiScaleUP_Retinex.multi_scale_enhance alone (the 3-scale FAM head, the
 * enhancement map and R*E + (1-R)*E^2 with a caller-given reflectance). */
enum { UPR_MODEL_IENET_ONLY = 1, UPR_MODEL_HEAD_ONLY = 2 };

typedef struct UprModel UprModel;

/* One state_dict entry: reference key name (e.g. "ie_net.enc1.conv1.weight"),
 * host fp32 data, shape. */
typedef struct {
  const char* name;
  const float* data;
  int ndim;
  int64_t shape[4];
} UprTensorDesc;

/* Replaces constructing + .to(device) + .eval() of MultiScaleUP_Retinex
 * (models/model.py:375-403) / ResidualIENet (:289-331, flag
 * UPR_MODEL_IENET_ONLY): packs an eval-mode state_dict (BatchNorm folded,
 * linear 1x1 chains composed, weights laid out [N][K] in `dtype`) into device
 * memory owned by the handle.  Keys follow the reference state_dict
 * (ResidualIENet keys carry the "ie_net." prefix).  `flags`: 0 or ONE of
 * UPR_MODEL_IENET_ONLY / UPR_MODEL_HEAD_ONLY; unknown bits or both flags
 * return UPR_ERR_ARG before any device call. */
int upr_model_create(const UprTensorDesc* params, int n_params, int use_preact, int use_aspp, int dtype,
                     int flags, UprModel** out);

/* Device bytes of workspace upr_model_forward needs for a B x 3 x H x W batch. */
size_t upr_model_workspace(const UprModel* model, int B, int H, int W);

/* Replaces MultiScaleUP_Retinex.forward (models/model.py:445-455):
 * x [B,3,H,W] in [0,1], H and W multiples of 8 (>= 16)  ->
 * enh [B,3,H,W], refl [B,3,H,W], illu [B,1,H,W] (all `dtype` of the model).
 * With UPR_MODEL_IENET_ONLY (ResidualIENet.forward, :333-360) only `illu` is
 * written and enh/refl may be NULL.  With UPR_MODEL_HEAD_ONLY
 * (multi_scale_enhance(x, reflectance, illu), :415-443) `refl` is an INPUT
 * [B,3,H,W], only `enh` is written and `illu` may be NULL (the reference
 * method does not read it).
 * An fp16 full model forks its multi-scale ops onto an internal side stream
 * after the first conv and joins it before the Retinex tail: completion of
 * `stream` implies completion of the whole forward (env UPR_MS_STREAMS=0: one
 * stream for every model, =1: fp32 models fork too). */
int upr_model_forward(UprModel* model, const void* x, int B, int H, int W, void* enh, void* refl, void* illu,
                      void* workspace, size_t workspace_bytes, void* stream);

void upr_model_destroy(UprModel* model);

/* Number of forwards of this handle so far that ran the two-stream schedule
 * above (0 when every forward stayed on one stream; -1 for NULL).  No
 * reference counterpart: lets a caller report which executor actually ran. */
long long upr_model_forks(const UprModel* model);

/* Per-op profiling of upr_model_forward (no reference counterpart: the
 * reference only brackets whole calls with time.time(), simple_enhance.py:165-179).
 * enable != 0 records a hipEvent pair around every op of every later forward
 * (stream-ordered, no synchronisation); enable == 0 stops and clears.
 * upr_model_profile_read waits for the recorded events and returns, per op in
 * launch order, the calls, summed device milliseconds, summed GEMM flops
 * (2*M*N*K of the launch) and summed algorithmic bytes. */
enum { UPR_OP_CONV_IGEMM = 0, UPR_OP_OTHER = 1 };
typedef struct {
  char name[64];
  int kind;
  int calls;
  double ms;
  double flops;
  double bytes;
} UprOpStat;
int upr_model_profile(UprModel* model, int enable);
int upr_model_profile_read(UprModel* model, UprOpStat* out, int max_ops, int* n_ops);

const char* upr_status_string(int status);

/* MultiScaleUP_Retinex.retinex_decompose (models/model.py:405-413) on its own:
 * refl = x / (illu + 1e-6) for x [B,C,H,W] and illu [B,illu_c,H,W], illu_c 1
 * (broadcast over C) or C; fp32 arithmetic rounded once to `dtype`.  The
 * backward (autograd of the reference expression) writes dx = g / (illu + 1e-6)
 * and dillu = -sum_c g * x / (illu + 1e-6)^2 (over c when broadcast) into the
 * non-NULL of gx [B,C,H,W] / gillu [B,illu_c,H,W] (overwritten). */
int upr_retinex_decompose(const void* x, const void* illu, void* refl, int B, int C, int H, int W, int illu_c,
                          int dtype, void* stream);
int upr_retinex_decompose_bwd(const void* x, const void* illu, const void* g, void* gx, void* gillu, int B, int C,
                              int H, int W, int illu_c, int dtype, void* stream);

/* Generic NHWC convolution (op-level hook used by the parity tests and by
 * callers composing their own graphs): y = act(conv(x, w) + bias [+ residual]).
 * x [B,H,W,Cin] (Cin % 32 == 0), w packed [Cout][kh*kw*Cin] (tap-major, then
 * channel), bias fp32 [Cout] or NULL, residual [B,Ho,Wo,Cout] or NULL (added
 * before the ReLU), y [B,Ho,Wo,Cout] with Cout % 32 == 0. */
int upr_conv2d_nhwc(const void* x, int B, int H, int W, int Cin, const void* w, const float* bias, int Cout, int kh,
                    int kw, int stride, int pad, int dil, const void* residual, int relu, void* y, int dtype,
                    void* stream);

/* float -> uint8 exactly as `(x * 255).astype(np.uint8)` on float32
 * (enhancers/adaptive_params.py:142, letterbox.py:93): truncation, wrap mod
 * 256, NaN / |x*255| >= 2^31 -> 0.  n elements, any layout. */
int upr_quantize_u8(const void* x, uint8_t* out, size_t n, int dtype, void* stream);

/* letterbox / letterbox_tensor (utils/letterbox.py:9-102) of ONE image in one
 * launch: src is u8 HWC RGB (src_kind 0) or float32 CHW in [0,1] (src_kind 1,
 * quantised as (x*255).astype(uint8), letterbox.py:93); the H x W source is
 * resized to nh x nw with cv2.resize INTER_LINEAR 8-bit fixed-point semantics
 * (xtab [4][nw], ytab [4][nh] int32: source index 0 / 1, 11-bit weights 0 / 1,
 * built on the host like OpenCV's tables; both NULL when nh == H, nw == W),
 * placed at (top, left) of an Ho x Wo canvas filled with `color`
 * (0xBBGGRR bytes: channel c = (color >> 8c) & 255); out is float32 CHW / 255
 * (out_kind 0, what letterbox_tensor returns) or u8 HWC (out_kind 1). */
int upr_letterbox(const void* src, int src_kind, int H, int W, int top, int left, int nh, int nw, int Ho, int Wo,
                  const int32_t* xtab, const int32_t* ytab, int color, void* out, int out_kind, void* stream);

/* save_image's pixels (enhancers/simple_enhance.py:65-99): one image x [C,H,W]
 * (C = 3, or 1 = replicated to RGB) -> u8 HWC RGB as
 * (np.clip(x, 0, 1) * 255).astype(np.uint8). */
int upr_to_u8_hwc(const void* x, int C, int H, int W, int dtype, uint8_t* out, void* stream);

/* cv2.cvtColor(..., COLOR_RGB2LAB) / (..., COLOR_LAB2RGB) on 8-bit interleaved
 * pixels (adaptive_params.py:142-145, :158-161 — the reference goes through
 * BGR, which is the same arithmetic). */
int upr_rgb2lab_u8(const uint8_t* rgb, uint8_t* lab, size_t npix, void* stream);
int upr_lab2rgb_u8(const uint8_t* lab, uint8_t* rgb, size_t npix, void* stream);

/* cv2.createCLAHE(clip, (tiles_x, tiles_y)).apply on B planar 8-bit images
 * [B,H,W] (adaptive_params.py:149-152).  lut_ws: B*tiles_x*tiles_y*256 bytes. */
int upr_clahe_u8(const uint8_t* src, uint8_t* dst, uint8_t* lut_ws, int B, int H, int W, float clip, int tiles_x,
                 int tiles_y, void* stream);

/* Fused AdaptiveParameterAdjuster.apply_clahe_enhancement
 * (adaptive_params.py:121-169) on a batch: enh [B,3,H,W] float -> quantise ->
 * Lab -> CLAHE(clip, tiles) on L -> RGB -> /255 -> out [B,3,H,W].
 * Workspace: upr_clahe_enhance_workspace() bytes. */
size_t upr_clahe_enhance_workspace(int B, int H, int W, int tiles_x, int tiles_y);
int upr_clahe_enhance(const void* enh, void* out, void* workspace, int B, int H, int W, float clip, int tiles_x,
                      int tiles_y, int dtype, void* stream);

/* 256-bin histogram of the 8-bit BGR2GRAY image of each x [B,3,H,W] float
 * (calculate_brightness_features, adaptive_params.py:24-68): hist int32 [B,256]. */
int upr_gray_hist(const void* x, int32_t* hist, int B, int H, int W, int dtype, void* stream);

/* MultiScaleEnhancer (enhancers/multi_scale.py:17-115) per image:
 * sums fp64 [B,3] = per-scale feature sums; factor fp64 [B] (nullable);
 * when enh/out are non-NULL, out = clamp(enh * factor, 0, 1). */
int upr_multiscale(const void* x, const void* enh, void* out, double* sums, double* factor, int B, int H, int W,
                   int dtype, void* stream);

/* MultiScaleEnhancer.extract_multi_scale_features (multi_scale.py:17-60), one
 * scale (0: x1, 1: x0.5, 2: x0.25, size int(h*s) x int(w*s)):
 * out [B,7,hs,ws] = [bilinear image (3), luminance, gradient magnitude (3)]. */
int upr_multiscale_features(const void* x, void* out, int B, int H, int W, int scale_idx, int dtype, void* stream);

/* ContentAwareEnhancer (enhancers/content_aware.py:19-122) per image of
 * x [B,3,H,W]: saliency fp32 [B,H,W] (compute_saliency_map, nullable),
 * attention fp32 [B,H,W] (compute_attention_map, nullable) and, when enh/out
 * are non-NULL, out = clamp(enh * (1 + 0.2 * attention), 0, 1)
 * (apply_content_aware_enhancement :93-122, all on the device — the
 * reference's saliency stays on the CPU, :56-57). */
size_t upr_content_aware_workspace(int B, int H, int W);
int upr_content_aware(const void* x, const void* enh, void* out, float* saliency, float* attention, void* workspace,
                      size_t workspace_bytes, int B, int H, int W, int dtype, void* stream);

/* Host copies of the 8-bit Lab integer tables (for CPU-side verification):
 * gamma[256], cbrt[3072], yf[512], invgamma[4096] (uint16), rgb2xyz[9], xyz2rgb[9]. */
void upr_lab_tables(uint16_t* gamma, uint16_t* cbrt, uint16_t* yf, uint16_t* invgamma, int32_t* rgb2xyz,
                    int32_t* xyz2rgb);

/* Measured ceilings for the bench's roofline report (bench.py --ceilings; not
 * on the model path).  Runs `reps` back-to-back launches of `blocks` 256-thread
 * workgroups on `stream` and returns the average milliseconds per launch:
 *   UPR_CALIB_MFMA_F16: `iters` x 8 v_mfma_f32_16x16x32_f16 per wave on random
 *     fp16 operands held in registers (FLOPs = blocks * 4 * iters * 8 * 16384);
 *     src >= 1 MiB of fp16 (bytes), dst = blocks * 256 * 4 floats;
 *   UPR_CALIB_HBM_COPY: dst[0:bytes] = src[0:bytes], 16 B per lane (HBM bytes =
 *     2 * bytes; 16-byte aligned); iters selects the access form: 0 grid-stride,
 *     1 grid-stride non-temporal, 2 one contiguous slice per workgroup.
 * Stands in for no reference interface: the reference has no roofline. */
enum { UPR_CALIB_MFMA_F16 = 0, UPR_CALIB_HBM_COPY = 1 };
int upr_calib_run(int which, int blocks, int iters, const void* src, void* dst, size_t bytes, int reps,
                  float* ms_per_launch, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* UPR_H_ */
