/*
 * upr_train.h — C ABI of the UP-Retinex TRAINING kernels in libupr.so (gfx950).
 *
 * The reference trains with PyTorch autograd (trainers/train.py:63-103:
 * forward -> losses/loss.py TotalLoss -> loss.backward() -> clip_grad_norm_ ->
 * Adam.step()).  It has no native code, so every entry below replaces a piece
 * of that Python/PyTorch path; each names the reference code it stands for.
 * The host side (retinex-image-enhancement_amd/upr/train.py) strings these
 * kernels into an explicit forward + backward of MultiScaleUP_Retinex and of
 * TotalLoss — there is no autograd tape inside.
 *
 * Conventions (as upr.h): caller-allocated device buffers, fp32 unless stated,
 * `stream` = hipStream_t as void*, stream-ordered, no internal synchronisation;
 * return 0, a hipError_t (> 0) or a negative UPR_ERR_* code.
 *
 * Activations are described by UprView: element strides of the four logical
 * axes (batch, row, column, channel), so one kernel reads NCHW network
 * inputs, NHWC activations and channel slices of concat buffers alike.
 * "Accumulate" arguments add into the destination instead of overwriting —
 * the gradient of a tensor consumed by several ops is summed in place.
 */
#ifndef UPR_TRAIN_H_
#define UPR_TRAIN_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  void* data;
  int64_t sb, sh, sw, sc;
} UprView;

/* hipMemsetAsync(p, 0, bytes) on the stream (zero a gradient / accumulator). */
int upr_t_zero(void* p, size_t bytes, void* stream);

/* ---- convolution ------------------------------------------------------- */

/* nn.Conv2d.forward for any channel count (model.py:29-62 small convs:
 * input/scale 3->32, output_layer 32->3, residual_head.2 32->1, channel /
 * spatial attention; VGG conv1_1 of loss.py:198-211): direct FMA kernel,
 * weights in PyTorch layout [Cout][Cin][kh][kw]. */
int upr_t_conv_direct(const UprView* x, int B, int H, int W, int Cin, const float* w, const float* bias, int Cout,
                      int kh, int kw, int stride, int pad, int dil, const UprView* y, int Ho, int Wo, int relu,
                      int accumulate, void* stream);
/* The same forward also writing y16 = (half)y compact [B*Ho*Wo][Cout] (the
 * next autocast conv's operand): the 3 -> 32 / 64 3x3 kernel only, else
 * UPR_ERR_UNSUPPORTED (nothing launched).  skip32: y is not written (an
 * activation whose readers all take y16; accumulate must be 0). */
int upr_t_conv_direct16(const UprView* x, int B, int H, int W, int Cin, const float* w, const float* bias, int Cout,
                        int kh, int kw, int stride, int pad, int dil, const UprView* y, int Ho, int Wo, int relu,
                        int accumulate, void* y16, int skip32, void* stream);
/* Input gradient of a 3 -> Cout (32 / 64) 3x3 / stride 1 / pad 1 conv under
 * autocast (VGG-19 conv1_1): dy16 = the fp16 output gradient, compact
 * [B][H][W][Cout]; weights [Cout][3][3][3] fp32, rounded to fp16; fp32
 * accumulation on MFMA.  dx [B][H][W][3] view (+= when accumulate). */
int upr_t_conv_dgrad_c3_16(const void* dy16, int B, int H, int W, const float* w, int Cout, const UprView* dx,
                           int accumulate, void* stream);
/* d(loss)/d(input) of the same conv (autograd of F.conv2d). */
int upr_t_conv_direct_dgrad(const UprView* dy, int Ho, int Wo, const float* w, int B, int H, int W, int Cin, int Cout,
                            int kh, int kw, int stride, int pad, int dil, const UprView* dx, int accumulate,
                            void* stream);
/* d(loss)/d(weight) [Cout][Cin][kh][kw] and d(loss)/d(bias) [Cout] (nullable),
 * both ACCUMULATED (fp32 atomics). */
int upr_t_conv_direct_wgrad(const UprView* x, const UprView* dy, int B, int H, int W, int Cin, int Ho, int Wo,
                            int Cout, int kh, int kw, int stride, int pad, int dil, float* dw, float* dbias,
                            void* stream);
/* The same with dy masked by y > 0 on the fly (y: the producing ReLU's output,
 * dy's shape) -- a ReLU backward whose masked gradient only this weight
 * gradient reads (the first conv of a stem, its input the image).  Cout <= 32
 * on the generic small-channel kernel, else UPR_ERR_UNSUPPORTED. */
int upr_t_conv_direct_wgrad_relu(const UprView* x, const UprView* dy, const UprView* y, int B, int H, int W, int Cin,
                                 int Ho, int Wo, int Cout, int kh, int kw, int stride, int pad, int dil, float* dw,
                                 float* dbias, void* stream);
/* The image stems' case of it (Cin 3 -> Cout 32, 3x3, stride 1, pad 1,
 * dilation 1, with bias): dy contiguous [B][H][W][32] fp32 (16-byte aligned),
 * the mask from the ReLU output's compact fp16 copy y16 ([B][H][W][32]), x any
 * view of the 3-channel input.  dw ([32][27], PyTorch's [co][ci][kh][kw]) and
 * dbias += the sums.  UPR_ERR_UNSUPPORTED off those layouts. */
int upr_t_conv_stem_wgrad_relu16(const UprView* x, const float* dy, const void* y16, int B, int H, int W, float* dw,
                                 float* dbias, void* stream);

/* MFMA implicit-GEMM conv (the inference kernels of conv.hip/conv_halo.hip) on
 * NHWC sources with channel stride/offset; Cin, Cout multiples of 32.
 * wp: packed [N][kh*kw*Cin] (upr_t_pack_weight).  res (nullable) is added
 * before the ReLU — with res == y it accumulates.  store 1 = ConvTranspose2d
 * k2 s2 pixel shuffle (N = 4*Cout rows, y is [B,2Ho,2Wo]). */
int upr_t_conv_mfma(const float* x, int B, int H, int W, int Cin, int x_cs, int x_coff, const float* wp,
                    const float* bias, int N, int kh, int kw, int stride, int pad, int dil, const float* res,
                    int res_cs, int relu, float* y, int y_cs, int y_coff, int store, void* stream);
/* Autocast (AMP) form of upr_t_conv_mfma (reference trainers/train.py:72 runs
 * the step under torch.cuda.amp.autocast(): convs in fp16).  x (fp32 view) is
 * cast into x16 (dense fp16 [B,H,W,Cin], caller-allocated) unless x16_ready;
 * wp16 = the packed weights in fp16 (upr_t_cast_f16); the fp16 MFMA conv
 * (fp32 accumulate, bias, ReLU) writes y16 (dense fp16 [B,Ho,Wo,N], or the
 * ConvTranspose layout for store 1), then y = float(y16) (+ res, in fp32,
 * indexed like upr_t_conv_mfma's: res == y accumulates).  res and relu are
 * exclusive.  store | 2: y16 must afterwards hold (half)y exactly (no res):
 * the next autocast conv reading y can take it as its x16 (x16_ready); without
 * that bit y16 is scratch.  y16_cs: y16's channel stride (0 = compact: N, or
 * N / 4 for store 1), e.g. a channel slice of a concat's fp16 copy.
 * store | 4 (with | 2): y need not be written (every reader takes y16); the
 * fp32 store is skipped where the kernel allows it.
 * store | 8: the input gradient of a 1x1 stride-2 conv (model.py:119-122
 * shortcut) without the zero-upsampled operand: x is dy at H x W, y (and res,
 * which must be given: y accumulates) is the 2H x 2W gradient, and pixel
 * (b, i, j) of the 1x1 stride-1 product is added at (b, 2i, 2j) only (the
 * other pixels of y are untouched); kh = kw = 1, pad 0, no relu, store 0.
 * store | 16: the input gradient of a 3x3 stride-2 pad-1 conv from dy itself
 * (x = dy at H x W, wp16 the flipped filter, y = 2H x 2W; the four output
 * phases as small convs over dy, no zero-upsampled operand): kh = kw = 3,
 * stride 1, no bias / relu; UPR_ERR_UNSUPPORTED when the kernel does not take
 * the shape (64 -> 32 channels, W % 16).
 * store | 32 (with x16_ready): x16 is in x's layout, element (pixel p, channel
 * c) at x16[p * x_cs + c] (the pointer already at the channel offset): a
 * channel slice of a concat's fp16 copy is read in place. */
int upr_t_conv_mfma16(const float* x, int B, int H, int W, int Cin, int x_cs, int x_coff, const void* wp16,
                      const float* bias, int N, int kh, int kw, int stride, int pad, int dil, const float* res,
                      int res_cs, int relu, float* y, int y_cs, int y_coff, int store, void* x16, int x16_ready,
                      void* y16, int y16_cs, void* stream);
/* y[i] = (fp16) x[i], n elements. */
int upr_t_cast_f16(const float* x, void* y, size_t n, void* stream);
/* Weight gradient of an NHWC conv as an MFMA GEMM over pixels:
 * dwp[co][(ky,kx,ci)] += sum_p dy[p][co] * x[window(p, ky, kx)][ci]
 * (packed layout of upr_t_pack_weight mode 0).  Cin, Cout multiples of 32. */
int upr_t_conv_wgrad(const float* x, int B, int H, int W, int Cin, int x_cs, int x_coff, const float* dy, int Ho,
                     int Wo, int Cout, int dy_cs, int dy_coff, int kh, int kw, int stride, int pad, int dil,
                     float* dwp, void* stream);
/* AMP weight gradient (trainers/train.py:72, convs under autocast): the same
 * contract as upr_t_conv_wgrad with both operands rounded to fp16 and fp32
 * accumulation (v_mfma_f32_16x16x32_f16).  x16: the compact fp16 copy
 * [B][H][W][Cin] of x made by the AMP forward (upr_t_conv_mfma16), or NULL
 * (x is cast into a stream-ordered temporary).  Shapes the fp16 kernel does
 * not take (Wo % 64 != 0, ...) run the fp32 upr_t_conv_wgrad. */
int upr_t_conv_wgrad16(const float* x, const void* x16, int B, int H, int W, int Cin, int x_cs, int x_coff,
                       const float* dy, int Ho, int Wo, int Cout, int dy_cs, int dy_coff, int kh, int kw, int stride,
                       int pad, int dil, float* dwp, void* stream);
/* Stride-1 input gradient on fp16 MFMA (x16 = the fp16 output gradient, wp16
 * = the flipped weights of upr_t_pack_weight mode 1 in fp16) with the ReLU
 * backward of the activation it flows into fused: y (fp32, skipped when
 * skip32) and y16 (compact fp16, y16_cs) are zero where mask16[pix *
 * mask16_cs + n] <= 0 (mask16 = that activation's fp16 copy).  No bias,
 * residual or accumulation.  UPR_ERR_UNSUPPORTED when no out32 kernel takes
 * the shape (nothing launched: run upr_t_conv_mfma16 + upr_t_relu_mask16). */
int upr_t_conv_mfma16_relu_bwd(const void* x16, int B, int H, int W, int Cin, const void* wp16, int N, int kh, int kw,
                               int pad, int dil, float* y, int y_cs, int y_coff, void* y16, int y16_cs,
                               const void* mask16, int mask16_cs, int skip32, void* stream);
/* The same with x16 a channel slice of a wider fp16 tensor: pixel p's Cin
 * values at x16[p * x16_cs] (x16 points at the slice's first channel; x16_cs
 * % 8 == 0) -- a slice of a shared concat gradient copy read in place. */
int upr_t_conv_mfma16_relu_bwd_cs(const void* x16, int x16_cs, int B, int H, int W, int Cin, const void* wp16, int N,
                                  int kh, int kw, int pad, int dil, float* y, int y_cs, int y_coff, void* y16,
                                  int y16_cs, const void* mask16, int mask16_cs, int skip32, void* stream);
/* The weight gradient added straight into PyTorch's layout: dw[co][ci][ky][kx]
 * += (no packed buffer, zero fill or unpack pass).  x16 non-NULL: the AMP
 * arithmetic of upr_t_conv_wgrad16 (x may then be NULL when the fp16 path
 * takes the shape); else the fp32 upr_t_conv_wgrad.  dy16 (nullable, AMP
 * only): dy's fp16 copy = (half)dy in dy's own layout (element (pixel p,
 * channel c) at dy16[p * dy_cs + dy_coff + c]: a channel slice of a concat's
 * gradient reads the concat's copy), read instead of dy (the same operand
 * values, half the bytes).  dw needs no alignment. */
int upr_t_conv_wgrad_into(const float* x, const void* x16, int B, int H, int W, int Cin, int x_cs, int x_coff,
                          const float* dy, const void* dy16, int Ho, int Wo, int Cout, int dy_cs, int dy_coff, int kh,
                          int kw, int stride, int pad, int dil, float* dw, void* stream);
/* Weight layout transforms.  mode 0: [Co][Ci][kh][kw] -> [Co][(ky,kx,ci)];
 * mode 1: -> [Ci][(ky,kx,co)] spatially flipped (stride-1 dgrad as a conv);
 * mode 2: ConvTranspose [Ci][Co][2][2] -> [(a,b,co)][ci] (forward GEMM);
 * mode 3: ConvTranspose [Ci][Co][2][2] -> [ci][(a,b,co)] (dgrad = k2 s2 conv). */
int upr_t_pack_weight(const float* w, float* out, int Co, int Ci, int kh, int kw, int mode, void* stream);
/* Every re-pack of a training step in one launch (the per-conv pack + fp16
 * cast launches were ~250 per step).  jobs: DEVICE array of njobs entries;
 * each packs w ([Co][Ci][kh][kw], n = Co*Ci*kh*kw elements) with its mode
 * (0-3 as upr_t_pack_weight; 4: replicate a bias of Co into out[q*Co + c],
 * q < 4, n = Co) into out32 (fp32) and / or out16 (fp16, the same value
 * rounded once), either may be NULL.  max_n: the largest n. */
typedef struct UprPackJob {
  const float* w;
  float* out32;
  void* out16;
  int Co, Ci, kh, kw, mode, n;
} UprPackJob;
int upr_t_pack_weights(const UprPackJob* jobs, int njobs, int max_n, void* stream);
/* Inverse of pack modes 0 and 3 for gradients; accumulate != 0 adds. */
int upr_t_unpack_grad(const float* gp, float* g, int Co, int Ci, int kh, int kw, int mode, int accumulate,
                      void* stream);
/* z[B,2Ho,2Wo,C] = dy scattered to even positions, zeros elsewhere (dgrad of
 * a stride-2 conv as a stride-1 conv over z). */
int upr_t_zero_upsample(const float* dy, int B, int Ho, int Wo, int C, int dy_cs, int dy_coff, float* z,
                        void* stream);

/* ---- BatchNorm2d, training mode (nn.BatchNorm2d, model.py:106-162,196-229) -- */
/* acc[2C] = (sum x, sum x^2) per channel of x[M][cs], overwritten (acc:
 * upr_t_reduce_acc_doubles(C) doubles; the atomic fallback for C % 4 / unaligned
 * rows clears acc itself first). */
int upr_t_bn_stats(const float* x, int M, int C, int cs, int coff, double* acc, void* stream);
/* batch mean / 1/sqrt(var_biased + eps); running stats updated with the
 * unbiased variance and momentum; *nbt += 1 (num_batches_tracked). */
int upr_t_bn_finalize(const double* acc, int M, int C, float momentum, float eps, float* running_mean,
                      float* running_var, int64_t* nbt, float* mean, float* invstd, void* stream);
/* Eval-mode BatchNorm (nn.BatchNorm2d.eval(), model.py's BN in a standalone
 * submodule forward): mean = running_mean, invstd = 1/sqrt(running_var + eps). */
int upr_t_bn_eval_stats(const float* running_mean, const float* running_var, int C, float eps, float* mean,
                        float* invstd, void* stream);
/* y = [relu](gamma*(x-mean)*invstd + beta + res_pre) + res_post  (res nullable). */
int upr_t_bn_apply(const float* x, int M, int C, int x_cs, int x_coff, const float* mean, const float* invstd,
                   const float* gamma, const float* beta, const float* res, int res_cs, int res_coff, int res_post,
                   int relu, float* y, int y_cs, int y_coff, void* stream);
/* upr_t_bn_apply that also writes y16[m][C] = (fp16) y (compact, nullable): the
 * autocast conv consuming y reads it instead of casting y again. */
int upr_t_bn_apply16(const float* x, int M, int C, int x_cs, int x_coff, const float* mean, const float* invstd,
                     const float* gamma, const float* beta, const float* res, int res_cs, int res_coff, int res_post,
                     int relu, float* y, int y_cs, int y_coff, void* y16, void* stream);
/* acc[2C] = (sum g, sum g*xhat) per channel (acc: upr_t_reduce_acc_doubles(C)
 * doubles; zeroed beforehand when C % 4 or the rows' alignment forces the
 * atomic single-stage form, which adds). */
int upr_t_bn_bwd_reduce(const float* g, int g_cs, int g_coff, const float* x, int x_cs, int x_coff, const float* mean,
                        const float* invstd, int M, int C, double* acc, void* stream);
/* batch_stats 1 (train-mode BN): dx = gamma*invstd*(g - sum_g/M - xhat*sum_gx/M); batch_stats 0 (an eval-mode
 * BN inside a training graph: running statistics are constants): dx = gamma*invstd*g.  dgamma/dbeta
 * (nullable) += sums either way. */
int upr_t_bn_bwd_apply(const float* g, int g_cs, int g_coff, const float* x, int x_cs, int x_coff, const float* mean,
                       const float* invstd, const float* gamma, const double* acc, int M, int C, float* dgamma,
                       float* dbeta, float* dx, int dx_cs, int dx_coff, int accumulate, int batch_stats,
                       void* stream);
/* upr_t_bn_bwd_reduce + upr_t_bn_bwd_apply in one call, with (relu != 0) the
 * consumer ReLU of a relu(bn(x)) folded in: g counts only where bn(x) > 0,
 * recomputed from x with the forward's expression (so no separate ReLU-mask
 * pass), and (dx16 non-NULL) a compact [M][C] fp16 copy of dx for the
 * autocast input-gradient conv that consumes it.  acc: 2C doubles of scratch
 * (zeroed here).  Needs C % 4 == 0, C <= 1024, 16-byte aligned rows;
 * UPR_ERR_UNSUPPORTED otherwise (the caller takes the separate kernels). */
int upr_t_bn_bwd_fused(const float* g, int g_cs, int g_coff, const float* x, int x_cs, const float* mean,
                       const float* invstd, const float* gamma, const float* beta, int relu, int M, int C,
                       double* acc, float* dgamma, float* dbeta, float* dx, int dx_cs, int dx_coff, int accumulate,
                       int batch_stats, void* dx16, void* stream);
/* BatchNorm training passes reading x from its compact fp16 copy x16 ([M][C])
 * instead of the fp32 tensor: under autocast the BN input is an fp16 conv's
 * output, so both hold the same values (bit-identical statistics, outputs and
 * gradients) at half the bytes.  C % 4 == 0 (and <= 1024 for the reductions),
 * else UPR_ERR_UNSUPPORTED. */
int upr_t_bn_stats16(const void* x16, int M, int C, double* acc, void* stream);
/* upr_t_bn_stats16 then upr_t_bn_finalize, the slot sums and the finalise in
 * one kernel (the same acc, mean / invstd and running statistics bits). */
int upr_t_bn_stats16_fin(const void* x16, int M, int C, double* acc, float momentum, float eps, float* running_mean,
                         float* running_var, int64_t* nbt, float* mean, float* invstd, void* stream);
int upr_t_bn_apply16h(const void* x16, int M, int C, const float* mean, const float* invstd, const float* gamma,
                      const float* beta, const float* res, int res_cs, int res_coff, int res_post, int relu, float* y,
                      int y_cs, int y_coff, void* y16, int skip32, void* stream);
/* upr_t_bn_apply16h with y16 a channel slice of a wider fp16 copy: y16 points
 * at the slice's first channel, y16_cs is the copy's channel stride (0: the
 * compact [M][C] form).  The ASPP concat under autocast (its fusion conv reads
 * the concat's fp16 copy). */
int upr_t_bn_apply16h_cs(const void* x16, int M, int C, const float* mean, const float* invstd, const float* gamma,
                         const float* beta, const float* res, int res_cs, int res_coff, int res_post, int relu,
                         float* y, int y_cs, int y_coff, void* y16, int y16_cs, int skip32, void* stream);
/* g16 (nullable): g read from the input-gradient conv's fp16 output instead
 * (compact [M][C]; g / g_cs / g_coff then unused). */
int upr_t_bn_bwd_fused16(const float* g, const void* g16, int g_cs, int g_coff, const void* x16, const float* mean,
                         const float* invstd, const float* gamma, const float* beta, int relu, int M, int C,
                         double* acc, float* dgamma, float* dbeta, float* dx, int dx_cs, int dx_coff, int accumulate,
                         int batch_stats, void* dx16, int skip32, void* stream);
/* skip32 (needs dx16 / y16; no accumulate): dx / y itself is not written -- the input
 * gradient's readers (the autocast conv's dgrad, weight gradient and bias sum)
 * all take dx16.  Bias gradient from an fp16 gradient copy ([M][C] compact):
 * out[c] (+)= sum over m (two-stage, ws = upr_t_reduce_acc_doubles(C)
 * doubles). */
int upr_t_chan_sum16(const void* g16, int M, int C, float* out, int accumulate, double* ws, void* stream);
/* upr_t_chan_sum16 over a channel slice of a wider fp16 copy: g16 points at the
 * slice's first channel, cs is the copy's channel stride. */
int upr_t_chan_sum16s(const void* g16, int M, int C, int cs, float* out, int accumulate, double* ws, void* stream);
/* upr_t_zero_upsample16 from the gradient's compact fp16 copy dy16. */
int upr_t_zero_upsample16h(const void* dy16, int B, int Ho, int Wo, int C, void* z16, void* stream);
/* upr_t_zero_upsample with an fp16 result z16 [B,2Ho,2Wo,C] (dy rounded to
 * fp16: the autocast stride-2 input-gradient conv's operand); C % 8 == 0. */
int upr_t_zero_upsample16(const float* dy, int B, int Ho, int Wo, int C, int dy_cs, int dy_coff, void* z16,
                          void* stream);
/* Doubles of `acc` that upr_t_bn_stats / upr_t_bn_bwd_reduce / upr_t_bn_bwd_fused
 * need (and of `ws` for upr_t_chan_sum_ws): acc[0, 2C) receives the per-channel
 * sums, the rest holds the per-block partial sums of the two-stage reduction
 * (deterministic: slots added in a fixed order). */
int upr_t_reduce_acc_doubles(int C);
/* upr_t_chan_sum through the two-stage reduction (ws: upr_t_reduce_acc_doubles(C)
 * doubles of scratch). */
int upr_t_chan_sum_ws(const float* g, int M, int C, int cs, int coff, float* out, int accumulate, double* ws,
                      void* stream);
/* out[C] (+)= per-channel sum of g[M][cs] (conv bias gradients). */
int upr_t_chan_sum(const float* g, int M, int C, int cs, int coff, float* out, int accumulate, void* stream);

/* ---- elementwise / layout ---------------------------------------------- */
/* g[m][c] *= (y[m][c] > 0)  (ReLU backward from the ReLU's output). */
int upr_t_relu_mask(float* g, int g_cs, int g_coff, const float* y, int y_cs, int y_coff, int M, int C,
                    void* stream);
/* The same mask also writing g16[m][c] = (half)(masked g), contiguous [M][C]
 * (the autocast dgrad operand); g is rewritten only when write32.  Needs C,
 * the strides and offsets multiples of 4 and 16-byte aligned g / y, else
 * UPR_ERR_UNSUPPORTED. */
int upr_t_relu_mask16(float* g, int g_cs, int g_coff, const float* y, int y_cs, int y_coff, int M, int C, void* g16,
                      int write32, void* stream);
/* The same with the mask taken from the activation's fp16 copy y16 (channel
 * stride y16_cs). */
int upr_t_relu_mask16h(float* g, int g_cs, int g_coff, const void* y16, int y16_cs, int M, int C, void* g16,
                       int write32, void* stream);
/* dst (+)= src, any layouts (NCHW <-> NHWC, concat slices). */
int upr_t_copy(const UprView* src, const UprView* dst, int B, int H, int W, int C, int accumulate, void* stream);
/* n contiguous elements.  op 0: out = sigmoid(a); op 1: out = a*b*(1-b)
 * (sigmoid backward, b = sigmoid output); op 2: out = a*mask/(1-p) with
 * mask_out[i] = hash(seed, i) >= p (nn.Dropout(p) train); op 3: out =
 * a*mask_in/(1-p) (its backward); op 4: out = a + b; op 5: out = a * b[0]
 * (scale by a device scalar, e.g. autograd's incoming loss gradient).
 * out may alias a. */
int upr_t_pointwise(const float* a, const float* b, float* out, size_t n, int op, const uint8_t* mask_in,
                    uint8_t* mask_out, float p, uint64_t seed, void* stream);

/* ---- pooling / resampling ---------------------------------------------- */
/* nn.MaxPool2d(k, s, p) forward / backward (backward recomputes the argmax
 * codes below, then gathers them deterministically; dx accumulated). */
int upr_t_maxpool(const UprView* x, int B, int H, int W, int C, int k, int s, int p, const UprView* y, int Ho, int Wo,
                  void* stream);
int upr_t_maxpool_bwd(const UprView* x, const UprView* dy, int B, int H, int W, int C, int k, int s, int p, int Ho,
                      int Wo, const UprView* dx, void* stream);
/* The same forward also writing code[b][oy][ox][c] = ky * k + kx of each
 * window's maximum (PyTorch's rule: the first in-bounds tap, then every tap
 * with v > max or v NaN; 255 for an empty window; code may be NULL), and the
 * backward from those codes: dx[b][iy][ix][c] (+)= dy of every window whose
 * code points at (iy, ix), in ascending (oy, ox) order (deterministic).
 * code holds B*Ho*Wo*C bytes, 4-byte aligned.  3x3/1/1 and 2x2/2/0 on
 * channel-contiguous views run 4 channels per thread.  y16 (nullable): also
 * the compact fp16 copy of y ([B][Ho][Wo][C], the autocast consumer's
 * operand) -- 4-channel path only, else UPR_ERR_UNSUPPORTED. */
int upr_t_maxpool_code(const UprView* x, int B, int H, int W, int C, int k, int s, int p, const UprView* y, int Ho,
                       int Wo, unsigned char* code, void* y16, void* stream);
int upr_t_maxpool_bwd_code(const unsigned char* code, const UprView* dy, int B, int H, int W, int C, int k, int s,
                           int p, int Ho, int Wo, const UprView* dx, int accumulate, void* stream);
/* upr_t_maxpool_bwd_code (3x3/1/1, 2x2/2/0) writing the gathered gradient
 * only as the compact fp16 g16 ([B][H][W][C]), masked by y16 > 0 when y16
 * (the pool input = a ReLU's compact fp16 output) is given: the pool backward
 * and the ReLU mask of a frozen fp16 dgrad's operand in one pass.
 * UPR_ERR_UNSUPPORTED off the 4-channel path. */
int upr_t_maxpool_bwd_code16(const unsigned char* code, const UprView* dy, int B, int H, int W, int C, int k, int s,
                             int p, int Ho, int Wo, const void* y16, void* g16, void* stream);
/* upr_t_maxpool_code reading the input's compact fp16 copy x16 ([B][H][W][C];
 * the autocast VGG activations exist in fp16 only): 3x3/1/1 and 2x2/2/0 with
 * C % 4 == 0, else UPR_ERR_UNSUPPORTED. */
/* upr_t_maxpool16_code: y->data NULL writes the fp16 copy y16 only (the pooled values are fp16 values). */
int upr_t_maxpool16_code(const void* x16, int B, int H, int W, int C, int k, int s, int p, const UprView* y, int Ho,
                         int Wo, unsigned char* code, void* y16, void* stream);
/* upr_t_copy / upr_t_bilinear also writing the fp16 copy of the result at
 * dst16[pixel * dst16_cs + c] (dst16 points at the slice's first channel of
 * a [B][H][W][dst16_cs] fp16 concat): 4-channel views only, else
 * UPR_ERR_UNSUPPORTED (nothing launched).  accumulate 2: the fp16 copy only
 * (dst's fp32 untouched) -- for a concat whose every reader takes its fp16
 * copy. */
int upr_t_copy16(const UprView* src, const UprView* dst, int B, int H, int W, int C, int accumulate, void* dst16,
                 int dst16_cs, void* stream);
int upr_t_bilinear16(const UprView* x, int B, int H, int W, int C, const UprView* y, int Ho, int Wo, int accumulate,
                     void* y16, int y16_cs, void* stream);
/* out = a + b (n floats) and out16 = (half)out; n % 4 == 0, 16-byte aligned
 * fp32 / 8-byte aligned fp16, else UPR_ERR_UNSUPPORTED. */
int upr_t_add16(const float* a, const float* b, float* out, size_t n, void* out16, void* stream);
/* F.interpolate(mode='bilinear', align_corners=False) H x W -> Ho x Wo
 * (scale = in/out per axis) and its backward (dx accumulated, atomics). */
int upr_t_bilinear(const UprView* x, int B, int H, int W, int C, const UprView* y, int Ho, int Wo, int accumulate,
                   void* stream);
int upr_t_bilinear_bwd(const UprView* dy, int B, int H, int W, int C, int Ho, int Wo, const UprView* dx,
                       void* stream);
/* out[B][C] (+)= scale * sum over pixels (AdaptiveAvgPool2d(1) with scale = 1/HW). */
int upr_t_pixel_sum(const float* x, int B, int HW, int C, int cs, int coff, float scale, float* out, int accumulate,
                    void* stream);
/* y[b][p][c] (+)= v[b][c] * scale  (broadcast of a per-image vector). */
int upr_t_broadcast(const float* v, int B, int HW, int C, float scale, float* y, int y_cs, int y_coff, int accumulate,
                    void* stream);
/* y16[b][p][y_coff + c] = (half)(v[b][c] * scale): the fp16 form (a channel
 * slice of an fp16 copy, channel stride y_cs). */
int upr_t_broadcast16(const float* v, int B, int HW, int C, float scale, void* y16, int y_cs, int y_coff,
                      void* stream);

/* ---- EnhancedFAM attention (model.py:47-59, 84-97) ---------------------- */
/* o2 = o*ca[b][c]; m[b][p] = (mean_c o2, max_c o2).  o [B,HW,C] contiguous. */
int upr_t_fam_ca_apply(const float* o, const float* ca, int B, int HW, int C, float* o2, float* m, void* stream);
/* sa = sigmoid(s_pre); out = o2*sa. */
int upr_t_fam_sa_apply(const float* o2, const float* s_pre, int B, int HW, int C, float* sa, float* out,
                       void* stream);
/* g_o2 = g*sa; g_spre = sum_c(g*o2) * sa*(1-sa). */
int upr_t_fam_sa_bwd(const float* g, const float* o2, const float* sa, int B, int HW, int C, float* g_o2,
                     float* g_spre, void* stream);
/* The same with g a channel slice: pixel p's C gradients at g[p * g_cs]
 * (the fusion concat's first slice read in place, no split copy). */
int upr_t_fam_sa_bwd_cs(const float* g, int g_cs, const float* o2, const float* sa, int B, int HW, int C,
                        float* g_o2, float* g_spre, void* stream);
/* g_o2 += g_m (mean/max routes); g_o = g_o2*ca; g_ca[b][c] += sum_p g_o2*o. */
int upr_t_fam_ca_bwd(const float* g_o2, const float* g_m, const float* o, const float* o2, const float* ca, int B,
                     int HW, int C, float* g_o, float* g_ca, void* stream);
/* g_o = (g_o + g_pool[b][c]/HW) * (o > 0). */
int upr_t_fam_pool_bwd(float* g_o, const float* g_pool, const float* o, int B, int HW, int C, void* stream);
/* The same also writing g16 = the result's compact fp16 copy ([B*HW][C]; the
 * fusion conv's autocast gradient operand).  C % 4 == 0 with C / 4 dividing
 * 256 and 16-byte aligned g_o / g_pool / o, else UPR_ERR_UNSUPPORTED. */
int upr_t_fam_pool_bwd16(float* g_o, const float* g_pool, const float* o, int B, int HW, int C, void* g16,
                         void* stream);

/* ---- network tail (model.py:351-358, 405-413, 439-455) ------------------ */
/* illu = sigmoid(mean_c x + r): x [B,3,H,W], r [B,H,W] (1 channel), illu [B,1,H,W]. */
int upr_t_head_fwd(const float* x, const float* r, float* illu, int B, int H, int W, void* stream);
/* e = sigmoid(o) (o NHWC [B,H,W,3]); refl = x/(illu+1e-6); enh = refl*e + (1-refl)*e^2 (NCHW). */
int upr_t_retinex_fwd(const float* x, const float* illu, const float* o, float* e, float* refl, float* enh, int B,
                      int H, int W, void* stream);
/* Backward of the two above from (g_enh, g_refl, g_illu) (NCHW; g_refl /
 * g_illu nullable): g_o NHWC [B,H,W,3], g_r [B,H,W]. */
int upr_t_retinex_bwd(const float* x, const float* illu, const float* e, const float* refl, const float* g_enh,
                      const float* g_refl, const float* g_illu, float* g_o, float* g_r, int B, int H, int W,
                      void* stream);

/* multi_scale_enhance's combine with a caller-given reflectance (model.py:439-443,
 * the head alone): e = sigmoid(o) (o NHWC [B,H,W,3]), enh = refl*e + (1-refl)*e^2
 * (refl / enh NCHW).  Backward from g_enh: g_o NHWC, g_refl NCHW (nullable). */
int upr_t_enhance_fwd(const float* refl, const float* o, float* e, float* enh, int B, int H, int W, void* stream);
int upr_t_enhance_bwd(const float* e, const float* refl, const float* g_enh, float* g_o, float* g_refl, int B, int H,
                      int W, void* stream);

/* ---- TotalLoss (losses/loss.py:586-753) -------------------------------- */
/* The loss modules' constructor arguments (reference defaults in brackets). */
typedef struct UprLossParams {
  int patch;              /* AdaptiveExposureLoss patch_size [16] (loss.py:24) */
  float base_exposure;    /* base_target_exposure [0.6] */
  float smooth_lambda;    /* EdgeAwareSmoothnessLoss lambda_val [10] (:76) */
  float smooth_alpha;     /* alpha [1] */
  float decouple_lambda;  /* IlluminationReflectanceDecouplingLoss lambda_val [0.1] (:271) */
  float freq_high;        /* FrequencyLoss weight_high [1] (:442) */
  float freq_low;         /* weight_low [0.5] */
  int dynamic_smooth;     /* TotalLoss use_dynamic_smooth_weight [1] (:617) */
  int illu_channels;      /* channels of illu / g_illu: 1 (the model's [B,1,H,W]) or 3 (the
                             reference self-test's [B,3,H,W], loss.py:806-844); 0 = 1.
                             Smoothness: mean over the C planes (:148, :171-172); decoupling:
                             C = 1 the expanded uncentred cross-covariance (:308-312) and
                             the mse of channel-mean means (:326-329), C = 3 the centred 3x3
                             covariance (:302-304) and the per-channel mean mse (:323-324) */
} UprLossParams;
/* Loss workspace bytes for a B x 3 x H x W batch (H, W multiples of 16). */
size_t upr_t_loss_workspace(int B, int H, int W);
/* ... for exposure patch size `patch` (H, W >= patch; floor(H/patch) x
 * floor(W/patch) patches, as F.avg_pool2d). */
size_t upr_t_loss_workspace_p(int B, int H, int W, int patch);
/* calculate_texture_complexity(img, method) (losses/loss.py:523-583) on its own:
 * img [B,C,H,W] fp32 (H, W >= 2) -> out[B] fp32; method 0 'tv' (mean |horizontal
 * difference| + mean |vertical difference|), 1 'edge_density' (share of pixels
 * whose reflect-padded Sobel magnitude of the channel-mean gray exceeds 1.5x
 * its per-image mean).  acc: 2B doubles of scratch. */
int upr_t_texture_complexity(const float* img, int B, int C, int H, int W, int method, double* acc, float* out,
                             void* stream);
/* Every non-perceptual, non-frequency term: exposure (:29-58), edge-aware
 * smoothness (:138-176), colour (:351-371), spatial (:408-427), decoupling
 * (:275-334), texture complexity of img_low (:523-583; texture 0 = 'tv',
 * 1 = 'edge_density') and the dynamic smooth weight
 * clamp(w_smooth * (1 - 0.8 * batch-mean complexity), 0.1, 5) (:704-720).
 * terms (device fp32, layout of upr_t_loss_total) receives [0..4] and [8];
 * with grads != 0, g_enh / g_illu / g_refl (NCHW) are OVERWRITTEN with the
 * weighted gradient of those terms. */
int upr_t_loss_pixel(const float* low, const float* enh, const float* illu, const float* refl, int B, int H, int W,
                     void* ws, float* terms, float* g_enh, float* g_illu, float* g_refl, int grads, float w_exp,
                     float w_col, float w_spa, float w_dec, float w_smooth, int texture, void* stream);
/* The same with the loss modules' arguments (upr_t_loss_pixel = the defaults);
 * dynamic_smooth = 0 makes terms[8] = w_smooth (no texture pass). */
int upr_t_loss_pixel_p(const float* low, const float* enh, const float* illu, const float* refl, int B, int H, int W,
                       void* ws, float* terms, float* g_enh, float* g_illu, float* g_refl, int grads, float w_exp,
                       float w_col, float w_spa, float w_dec, float w_smooth, int texture,
                       const UprLossParams* params, void* stream);
/* Perceptual MSE level (F.mse_loss): acc (fp64) += sum (a-b)^2 / n; with
 * g != NULL, g = scale*2*(a-b) (scale = weight/n). */
int upr_t_mse(const float* a, const float* b, size_t n, double* acc, float* g, float scale, void* stream);
/* The same over two fp16 tensors (n % 4 == 0, 8-byte aligned; g 16-byte aligned or NULL), else
 * UPR_ERR_UNSUPPORTED: the frozen VGG's fp16-only features under autocast. */
int upr_t_mse16(const void* a16, const void* b16, size_t n, double* acc, float* g, float scale, void* stream);
/* (x NCHW - mean) / std -> NHWC [B,H,W,3]; bwd: g_x (NCHW) += g_y / std. */
int upr_t_vgg_norm(const float* x, float* y, int B, int H, int W, void* stream);
int upr_t_vgg_norm_bwd(const float* g_y, float* g_x, int B, int H, int W, void* stream);
/* FrequencyLoss (:447-487) on complex spectra Ze, Zl (interleaved re/im,
 * [B*3][H][W]): acc[1] += sum w*(|Ze|-|Zl|)^2 with w = 1 (dist > r) / 0.5;
 * with G != NULL, G = scale*2*w*(|Ze|-|Zl|) * Ze/|Ze| (0 where |Ze| = 0). */
int upr_t_freq(const float* Ze, const float* Zl, int BC, int H, int W, double* acc, float* G, float scale,
               void* stream);
/* ... with FrequencyLoss(weight_high, weight_low) (upr_t_freq: 1, 0.5). */
int upr_t_freq_p(const float* Ze, const float* Zl, int BC, int H, int W, double* acc, float* G, float scale,
                 float w_high, float w_low, void* stream);
/* g (+)= scale * Re(z) (z interleaved complex, n elements). */
int upr_t_add_real(const float* z, float* g, size_t n, float scale, void* stream);
/* out[i] = scale * acc[i], i < n (device-side finalisation of a reduction). */
int upr_t_scale_acc(const double* acc, int n, float scale, float* out, void* stream);
/* terms[9] = [exposure, smoothness, color, spatial, decouple, perceptual,
 * frequency, total, smooth_weight]: terms[7] = the weighted sum of
 * TotalLoss.forward (loss.py:722-729) with the fixed weights w[7] and
 * terms[8] as the smoothness weight. */
int upr_t_loss_total(float* terms, float w_exp, float w_col, float w_spa, float w_dec, float w_per, float w_freq,
                     void* stream);

/* ---- optimiser (torch.nn.utils.clip_grad_norm_ + torch.optim.Adam) ------ */
/* GradScaler.unscale_ (trainers/train.py:84-86 with use_amp; torch.amp.GradScaler):
 * g[i] *= 1 / *scale over n elements; *found_inf (caller-zeroed) = 1 when any
 * unscaled value is inf or nan.  scale and found_inf are device fp32 scalars. */
int upr_t_unscale(float* g, size_t n, const float* scale, float* found_inf, void* stream);
/* acc (fp64, zeroed) += sum g^2 over n elements. */
int upr_t_sqsum(const float* g, size_t n, double* acc, void* stream);
/* One Adam step over a flat parameter buffer with the clip_grad_norm_(max_norm)
 * coefficient computed on the device from sqsum: g' = g*min(1, max_norm/(sqrt(sqsum)+1e-6))
 * + wd*p; m,v moments; bias-corrected update (train.py:84-103, Adam L2 decay).
 * norm_out (nullable) receives sqrt(sqsum). */
int upr_t_adam(float* p, const float* g, float* m, float* v, size_t n, const double* sqsum, float max_norm, float lr,
               float beta1, float beta2, float eps, float weight_decay, int step, float* norm_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* UPR_TRAIN_H_ */
