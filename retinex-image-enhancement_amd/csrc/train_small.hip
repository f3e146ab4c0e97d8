// Small-channel convolutions of the training step (the convs whose Cin or Cout
// is not a multiple of 32, so they cannot take the MFMA implicit-GEMM path):
// the 3-channel 3x3 input convs (ResidualIENet.input_layer and the three
// multi-scale branch convs, models/model.py:293,419-425; VGG-19 conv1_1 of the
// perceptual loss, losses/loss.py:198-211), the 32->3 / 32->1 heads
// (model.py:402,326), the 7x7 2->1 spatial attention and the channel-attention
// squeeze convs of EnhancedFAM (model.py:47-59).
//
// Round 1 ran them as one thread per OUTPUT ELEMENT with 64-bit index math
// (26 % of the bs-8 512^2 step).  Here:
//   * forward (3 -> COUT 3x3): fp32 MFMA over 16-pixel groups, the filter in
//     registers, 16-byte stores straight from the accumulators;
//   * input gradient (stride 1): one thread per input pixel accumulates all
//     CIN input-channel gradients over (tap, Cout), weights broadcast from LDS;
//   * weight gradient (Cout <= 32): a GEMM over pixels on
//     v_mfma_f32_32x32x2_f32 (D[co][k] += dy[p][co] * im2col[p][k], two
//     pixels per MFMA, k = ci*kh*kw + ky*kw + kx = PyTorch's weight layout,
//     plus a ones column for the bias), per-block LDS reduction into a
//     partial row per block, summed in block order by a second kernel.
// All fp32 (exact-fp32 MFMA); only the summation order differs from a serial
// loop.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "upr_common.h"
#include "../../include/upr.h"
#include "../../include/upr_train.h"

namespace upr {

typedef float f32x4_t2 __attribute__((ext_vector_type(4)));
typedef float f32x16_t2 __attribute__((ext_vector_type(16)));

struct SV {
  float* d;
  long long sb, sh, sw, sc;
  __device__ __forceinline__ long long at(int b, int y, int x, int c) const {
    return b * sb + y * sh + x * sw + c * sc;
  }
};

static SV mksv(const UprView* u) {
  SV v;
  v.d = (float*)u->data;
  v.sb = u->sb; v.sh = u->sh; v.sw = u->sw; v.sc = u->sc;
  return v;
}

// ---------------------------------------------------------------------------
// forward: 3 -> COUT (32 / 64), 3x3, stride 1, dilation 1, on fp32 MFMA
// (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation).  The
// kernel above reads every weight from LDS once per output pixel (432
// ds_read_b128 per thread for 64 channels: 0.26 ms, 1 TB/s, for VGG conv1_1 at
// bs 8 512^2).  Here a wave walks 16-pixel groups: lane (pixel l & 15, k-group
// l >> 4) gathers the 7 input values k = kg + 4s (k = ci*9 + ky*3 + kx, 27
// padded to 28) straight from HBM, the filter lives in registers as the A
// operand (COUT/16 tiles x 7 k-steps, one float per lane each), and the
// accumulator of tile t holds channels 16t + 4(l >> 4) .. +3 of pixel l & 15:
// 16-byte fp32 / 8-byte fp16 stores from registers.
// ---------------------------------------------------------------------------
template <int COUT>
__global__ __launch_bounds__(256) void c3k3_mfma_kernel(SV x, int B, int H, int W, const float* __restrict__ w,
                                                       const float* __restrict__ bias, int p, SV y, int Ho, int Wo,
                                                       int relu, int accum, half_t* __restrict__ y16, int skip32) {
  constexpr int NT = COUT / 16;
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, kg = lane >> 4;
  float wa[NT][7];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int st = 0; st < 7; ++st) {
      const int k = kg + 4 * st;
      wa[t][st] = k < 27 ? w[(t * 16 + fr) * 27 + k] : 0.f;
    }
  f32x4_t2 bv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[t][i] = bias ? bias[t * 16 + kg * 4 + i] : 0.f;
  const long long P = (long long)B * Ho * Wo;
  const long long ngroups = (P + 15) / 16;
  const long long gstride = (long long)gridDim.x * 4;
  // inputs of group g (the next group's are loaded before this group's MFMAs)
  auto gather = [&](long long g, float (&xin)[7], int& b, int& oy, int& ox, bool& pok) {
    const long long pix = g * 16 + fr;
    pok = g < ngroups && pix < P;
    b = 0; oy = 0; ox = 0;
    if (pok) {
      ox = (int)(pix % Wo);
      const long long r = pix / Wo;
      oy = (int)(r % Ho);
      b = (int)(r / Ho);
    }
#pragma unroll
    for (int st = 0; st < 7; ++st) {
      const int k = kg + 4 * st;
      const int ci = k / 9, ky = (k % 9) / 3, kx = k % 3;
      const int iy = oy - p + ky, ix = ox - p + kx;
      xin[st] = (pok && k < 27 && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) ? x.d[x.at(b, iy, ix, ci)]
                                                                                           : 0.f;
    }
  };
  long long g = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  float xn[7];
  int nb, noy, nox;
  bool npok;
  gather(g, xn, nb, noy, nox, npok);
  for (; g < ngroups; g += gstride) {
    float xin[7];
#pragma unroll
    for (int st = 0; st < 7; ++st) xin[st] = xn[st];
    const int b = nb, oy = noy, ox = nox;
    const bool pok = npok;
    const long long pix = g * 16 + fr;
    gather(g + gstride, xn, nb, noy, nox, npok);
    f32x4_t2 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      acc[t] = bv[t];
#pragma unroll
      for (int st = 0; st < 7; ++st) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[t][st], xin[st], acc[t], 0, 0, 0);
    }
    if (!pok) continue;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int co = t * 16 + kg * 4;
      f32x4_t2 v = acc[t];
      f32x4_t2* dst = (f32x4_t2*)(y.d + y.at(b, oy, ox, co));
      if (accum) v += *dst;
      if (relu) {
        v[0] = fmaxf(v[0], 0.f); v[1] = fmaxf(v[1], 0.f); v[2] = fmaxf(v[2], 0.f); v[3] = fmaxf(v[3], 0.f);
      }
      if (!skip32) *dst = v;
      if (y16) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        *(h4*)(y16 + (size_t)pix * COUT + co) = h4{(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
      }
    }
  }
}

// ---------------------------------------------------------------------------
// forward, COUT <= 4 output channels (32->3 / 32->1 1x1 heads, 7x7 2->1
// spatial attention): one thread per output pixel, all taps and input channels
// (16-byte loads when the input rows are channel-contiguous and aligned)
// ---------------------------------------------------------------------------
template <int COUT>
__global__ __launch_bounds__(256) void small_fwd_kernel(SV x, int B, int H, int W, int Cin,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        int kh, int kw, int s, int p, int d, SV y, int Ho, int Wo,
                                                        int relu, int accum, int xvec) {
  extern __shared__ __attribute__((aligned(16))) float smf[];  // [tap][ci][COUT]
  const int taps = kh * kw;
  const int nw = COUT * Cin * taps;
  for (int i = threadIdx.x; i < nw; i += 256) {
    const int co = i / (Cin * taps);
    const int rem = i - co * Cin * taps;
    const int ci = rem / taps, tap = rem - ci * taps;
    smf[(tap * Cin + ci) * COUT + co] = w[i];
  }
  __syncthreads();
  const int P = B * Ho * Wo;
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= P) return;
  const int ox = pix % Wo;
  const int r = pix / Wo;
  const int oy = r % Ho, b = r / Ho;
  float acc[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) acc[c] = bias ? bias[c] : 0.f;
  for (int ky = 0; ky < kh; ++ky) {
    const int iy = oy * s - p + ky * d;
    if (iy < 0 || iy >= H) continue;
    for (int kx = 0; kx < kw; ++kx) {
      const int ix = ox * s - p + kx * d;
      if (ix < 0 || ix >= W) continue;
      const float* xp = x.d + x.at(b, iy, ix, 0);
      const float* wt = smf + (ky * kw + kx) * Cin * COUT;
      int ci = 0;
      if (xvec) {
        for (; ci + 4 <= Cin; ci += 4) {
          const f32x4_t2 v = *(const f32x4_t2*)(xp + ci);
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int c = 0; c < COUT; ++c) acc[c] = fmaf(v[e], wt[(ci + e) * COUT + c], acc[c]);
        }
      }
      for (; ci < Cin; ++ci) {
        const float v = xp[ci * x.sc];
#pragma unroll
        for (int c = 0; c < COUT; ++c) acc[c] = fmaf(v, wt[ci * COUT + c], acc[c]);
      }
    }
  }
  float* yp = y.d + y.at(b, oy, ox, 0);
#pragma unroll
  for (int c = 0; c < COUT; ++c) {
    float v = acc[c];
    if (accum) v += yp[c * y.sc];
    if (relu) v = fmaxf(v, 0.f);
    yp[c * y.sc] = v;
  }
}

// ---------------------------------------------------------------------------
// forward, 1x1 heads of <= 4 outputs over 16 / 32 / 64 channel-contiguous
// inputs (32 -> 3 / 32 -> 1 at 512^2: models/model.py:335, 440).  The
// one-pixel-per-thread kernel above has each lane walk its own 128-byte pixel
// (0.25 ms, 1 TB/s); here a wave reads 64 pixels as consecutive 16-byte
// chunks (lane = (pixel, channel quad), LPP = Cin / 4 lanes per pixel), each
// lane forms the quad's partial dot products and the LPP lanes of a pixel sum
// them with xor shuffles.
// ---------------------------------------------------------------------------
template <int COUT, int LPP>
__global__ __launch_bounds__(256) void head1x1_kernel(SV x, int P, int Ho, int Wo, const float* __restrict__ w,
                                                      const float* __restrict__ bias, SV y, int relu, int accum) {
  const int lane = threadIdx.x & 63;
  const long long gw = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int q = lane % LPP;
  constexpr int CIN = LPP * 4;
  float wv[4][COUT];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int c = 0; c < COUT; ++c) wv[e][c] = w[c * CIN + q * 4 + e];
#pragma unroll
  for (int j = 0; j < LPP; ++j) {
    const long long pix = gw * 64 + (j * 64 + lane) / LPP;
    const bool in = pix < P;
    int b = 0, oy = 0, ox = 0;
    f32x4_t2 v = f32x4_t2{0.f, 0.f, 0.f, 0.f};
    if (in) {
      ox = (int)(pix % Wo);
      const long long r = pix / Wo;
      oy = (int)(r % Ho);
      b = (int)(r / Ho);
      v = *(const f32x4_t2*)(x.d + x.at(b, oy, ox, q * 4));
    }
    float part[COUT];
#pragma unroll
    for (int c = 0; c < COUT; ++c) {
      part[c] = v[0] * wv[0][c];
#pragma unroll
      for (int e = 1; e < 4; ++e) part[c] = fmaf(v[e], wv[e][c], part[c]);
    }
#pragma unroll
    for (int off = LPP / 2; off >= 1; off >>= 1)
#pragma unroll
      for (int c = 0; c < COUT; ++c) part[c] += __shfl_xor(part[c], off);
    if (in && q == 0) {
      float* yp = y.d + y.at(b, oy, ox, 0);
#pragma unroll
      for (int c = 0; c < COUT; ++c) {
        float o = part[c] + (bias ? bias[c] : 0.f);
        if (accum) o += yp[c * y.sc];
        if (relu) o = fmaxf(o, 0.f);
        yp[c * y.sc] = o;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// input gradient, stride 1: dx[b,iy,ix,ci] (+)= sum_{ky,kx,co} dy[b,iy+p-ky*d,ix+p-kx*d,co] w[co][ci][ky][kx]
// ---------------------------------------------------------------------------
template <int CIN, int COUTT>
__global__ __launch_bounds__(256) void small_dgrad_kernel(SV dy, int Ho, int Wo, const float* __restrict__ w, int B,
                                                          int H, int W, int Cout, int kh, int kw, int p, int d, SV dx,
                                                          int accum, int vec, int dvec) {
  extern __shared__ __attribute__((aligned(16))) float smd[];  // [tap][co][CIN]
  const int taps = kh * kw;
  const int nw = Cout * taps * CIN;
  for (int i = threadIdx.x; i < nw; i += 256) {
    const int co = i / (CIN * taps);
    const int rem = i - co * CIN * taps;
    const int ci = rem / taps, tap = rem - ci * taps;
    smd[(tap * Cout + co) * CIN + ci] = w[i];
  }
  __syncthreads();
  const int P = B * H * W;
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= P) return;
  const int ix = pix % W;
  const int r = pix / W;
  const int iy = r % H, b = r / H;
  float acc[CIN];
#pragma unroll
  for (int c = 0; c < CIN; ++c) acc[c] = 0.f;
  for (int ky = 0; ky < kh; ++ky) {
    const int oy = iy + p - ky * d;
    if (oy < 0 || oy >= Ho) continue;
    for (int kx = 0; kx < kw; ++kx) {
      const int ox = ix + p - kx * d;
      if (ox < 0 || ox >= Wo) continue;
      const float* dyp = dy.d + dy.at(b, oy, ox, 0);
      const float* wt = smd + (ky * kw + kx) * Cout * CIN;
      int co = 0;
      if (COUTT > 0 && dvec) {  // compile-time Cout: the tap's loads all in flight, then the FMAs
        f32x4_t2 g4[COUTT > 0 ? COUTT / 4 : 1];
#pragma unroll
        for (int q = 0; q < COUTT / 4; ++q) g4[q] = *(const f32x4_t2*)(dyp + 4 * q);
#pragma unroll
        for (int q = 0; q < COUTT / 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int c = 0; c < CIN; ++c) acc[c] = fmaf(g4[q][e], wt[(4 * q + e) * CIN + c], acc[c]);
        co = COUTT;
      }
      if (dvec) {  // channel-contiguous, 16-byte aligned dy rows: 4 channels per load
        for (; co + 4 <= Cout; co += 4) {
          const f32x4_t2 g4 = *(const f32x4_t2*)(dyp + co);
          const float* wc = wt + co * CIN;
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int c = 0; c < CIN; ++c) acc[c] = fmaf(g4[q], wc[q * CIN + c], acc[c]);
        }
      }
      for (; co < Cout; ++co) {
        const float g = dyp[co * dy.sc];
        const float* wc = wt + co * CIN;
#pragma unroll
        for (int c = 0; c < CIN; ++c) acc[c] = fmaf(g, wc[c], acc[c]);
      }
    }
  }
  float* xp = dx.d + dx.at(b, iy, ix, 0);
  if (CIN % 4 == 0 && vec) {  // channel-contiguous, 16-byte aligned rows (host-checked)
#pragma unroll
    for (int c = 0; c < CIN; c += 4) {
      f32x4_t2 v = f32x4_t2{acc[c], acc[c + 1], acc[c + 2], acc[c + 3]};
      if (accum) v += *(const f32x4_t2*)(xp + c);
      *(f32x4_t2*)(xp + c) = v;
    }
  } else {
#pragma unroll
    for (int c = 0; c < CIN; ++c) {
      float v = acc[c];
      if (accum) v += xp[c * dx.sc];
      xp[c * dx.sc] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// weight gradient, Cout <= 32: D[co][k] = sum_p dy[p][co] * col[p][k] on
// v_mfma_f32_32x32x2_f32 (A = dy rows, B = im2col rows, K = 2 pixels)
// ---------------------------------------------------------------------------
// pixel pairs in flight per wave
template <int NT>
constexpr int sw_unroll() { return NT == 2 ? 16 : 8; }

template <int NT>
__global__ __launch_bounds__(256) void small_wgrad_mfma_kernel(SV x, SV dy, int B, int H, int W, int Cin, int Ho,
                                                               int Wo, int Cout, int kh, int kw, int s, int p, int d,
                                                               int pairs_per_wave, float* __restrict__ part, SV ym) {
  // ym.d != nullptr: dy masked by ym > 0 on the fly (the producing ReLU's
  // backward, for a gradient whose only reader is this weight gradient)
  __shared__ __attribute__((aligned(16))) float red[4][NT][16][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, half = lane >> 5;
  const int taps = kh * kw;
  const int KC = Cin * taps;
  const int P = B * Ho * Wo;
  // per lane, per 32-column tile: this lane's im2col column k = t*32 + j
  int c_off[NT], c_dy[NT], c_dx[NT], c_kind[NT];  // kind: 0 zero, 1 pixel value, 2 ones (bias)
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int k = t * 32 + j;
    c_kind[t] = 0; c_off[t] = 0; c_dy[t] = 0; c_dx[t] = 0;
    if (k < KC) {
      const int ci = k / taps, tap = k - ci * taps;
      const int ky = tap / kw, kx = tap - ky * kw;
      c_kind[t] = 1;
      c_off[t] = ci;
      c_dy[t] = ky * d - p;
      c_dx[t] = kx * d - p;
    } else if (k == KC) {  // the bias column (kept only when the layer has a bias)
      c_kind[t] = 2;
    }
  }
  f32x16_t2 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  // 32-bit pixel math (P < 2^31, host-checked): the 64-bit div / mod per
  // pixel dominated these kernels
  const int gw = blockIdx.x * 4 + wave;
  const int pair0 = gw * pairs_per_wave;
  constexpr int SW_UNROLL = sw_unroll<NT>();
  for (int u0 = 0; u0 < pairs_per_wave; u0 += SW_UNROLL) {
    float av[SW_UNROLL], bv[SW_UNROLL][NT];
#pragma unroll
    for (int u = 0; u < SW_UNROLL; ++u) {
      const int pix = (pair0 + u0 + u) * 2 + half;
      av[u] = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) bv[u][t] = 0.f;
      if (u0 + u < pairs_per_wave && pix < P) {
        const int ox = pix % Wo;
        const int r = pix / Wo;
        const int oy = r % Ho, b = r / Ho;
        if (j < Cout) {
          av[u] = dy.d[dy.at(b, oy, ox, j)];
          if (ym.d && !(ym.d[ym.at(b, oy, ox, j)] > 0.f)) av[u] = 0.f;
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          if (c_kind[t] == 1) {
            const int iy = oy * s + c_dy[t], ix = ox * s + c_dx[t];
            if (iy >= 0 && iy < H && ix >= 0 && ix < W) bv[u][t] = x.d[x.at(b, iy, ix, c_off[t])];
          } else if (c_kind[t] == 2) {
            bv[u][t] = 1.f;
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < SW_UNROLL; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u][t], acc[t], 0, 0, 0);
  }
  // block reduction over the 4 waves into this block's partial row
  // part[block][co * (KC + 1) + k] (k == KC: the bias column); summed over the
  // blocks in order by small_wgrad_fin_kernel -- deterministic, and no
  // same-address atomics (which serialised ~1000 blocks per weight)
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) red[wave][t][e][lane] = acc[t][e];
  __syncthreads();
  for (int idx = tid; idx < NT * 16 * 64; idx += 256) {
    const int t = idx / (16 * 64);
    const int rem = idx - t * 16 * 64;
    const int e = rem / 64, l = rem - e * 64;
    const float v = red[0][t][e][l] + red[1][t][e][l] + red[2][t][e][l] + red[3][t][e][l];
    // 32x32 accumulator map: column = l & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (l >> 5)
    const int co = (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
    const int k = t * 32 + (l & 31);
    if (co >= Cout || k > KC) continue;
    part[((size_t)blockIdx.x * Cout + co) * (KC + 1) + k] = v;
  }
}

// dw[co][k] += sum over blocks of part[block][co][k]; the bias column into
// dbias.  One block per output: thread t adds blocks t, t + 256, ... in order,
// then a fixed LDS tree -- deterministic, and no long serial load chain
__global__ __launch_bounds__(256) void small_wgrad_fin_kernel(const float* __restrict__ part, int blocks, int Cout,
                                                              int KC, float* __restrict__ dw,
                                                              float* __restrict__ dbias) {
  __shared__ float red[256];
  const int i = blockIdx.x;  // co * (KC + 1) + k
  const int n = Cout * (KC + 1);
  const int co = i / (KC + 1), k = i - co * (KC + 1);
  if (k == KC && !dbias) return;
  float t = 0.f;
  for (int b = threadIdx.x; b < blocks; b += 256) t += part[(size_t)b * n + i];
  red[threadIdx.x] = t;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (k < KC) dw[(size_t)co * KC + k] += red[0];
    else dbias[co] += red[0];
  }
}

// ---------------------------------------------------------------------------
// input gradient of a 3 -> COUT (32 / 64) 3x3 / s1 / p1 conv under autocast
// (VGG-19 conv1_1's gradient w.r.t. the normalised enhanced image,
// losses/loss.py:198-211): dy in fp16 (the masked gradient's copy,
// upr_t_relu_mask16), weights rounded to fp16, fp32 accumulation on
// v_mfma_f32_16x16x32_f16 -- D[ci][pixel] = sum over (tap, co) of
// w[co][ci][tap'] * dy[pixel + tap][co] with the weights as A (rows 0..2 of
// 16 used) and dy as B.  A block owns 4 rows x 64 columns of dx; the dy rows
// and columns it needs (6 x 66 pixels x COUT channels) sit in LDS, the 16-byte
// chunks of a pixel XOR-swizzled by its column (within the pixel's COUT / 8
// chunks) so a fragment read (16 consecutive pixels, one chunk) spreads over
// the banks.  Lanes 0..15 of each 16-pixel group end
// with that pixel's 3 input-channel gradients: 12-byte runs, 192 contiguous
// bytes per group.
// ---------------------------------------------------------------------------
template <int COUT>
__global__ __launch_bounds__(256) void dgrad_c3_mfma_kernel(const half_t* __restrict__ dy, int B, int H, int W,
                                                            const float* __restrict__ w, SV dx, int accum) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int KC = COUT / 32, CH = COUT / 8;  // 32-channel k chunks, 16-byte chunks per pixel
  constexpr int TR = 4, TC = 64, LR = TR + 2, LC = TC + 2;
  __shared__ __attribute__((aligned(16))) half_t tile[LR * LC * COUT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fg = lane >> 4;
  // A = weights: lane (fr = ci, fg) holds w[co = kc*32 + fg*8 + e][ci][tap], tap = 8 - (dr*3 + dc);
  // built once per (persistent) block -- per tile, these 144 scalar loads per lane were
  // most of the kernel's time (0.24 ms for VGG conv1_1 at bs 8 512^2)
  h8 wa[KC][9];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        wa[kc][t][e] = fr < 3 ? (half_t)w[((kc * 32 + fg * 8 + e) * 3 + fr) * 9 + (8 - t)] : (half_t)0.f;
  const int ntx = (W + TC - 1) / TC, nty = (H + TR - 1) / TR;
  const int ntiles = ntx * nty * B;
  // software pipeline: the next tile's dy chunks are loaded into registers
  // while this tile's MFMAs run (the load-then-compute form left the memory
  // idle during the compute: 0.20 ms for VGG conv1_1 at bs 8 512^2)
  constexpr int NQ = (LR * LC * CH + 255) / 256;
  uint4 pre[NQ];
  auto fetch = [&](int tile_id) {
    const int tx = tile_id % ntx, ty = (tile_id / ntx) % nty, b = tile_id / (ntx * nty);
    const int iy0 = ty * TR, ix0 = tx * TC;
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int q = tid + j * 256;
      const int ch = q % CH, rc = q / CH, col = rc % LC, r = rc / LC;
      const int gy = iy0 - 1 + r, gx = ix0 - 1 + col;
      pre[j] = make_uint4(0u, 0u, 0u, 0u);
      if (q < LR * LC * CH && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W)
        pre[j] = *(const uint4*)(dy + (((size_t)b * H + gy) * W + gx) * COUT + ch * 8);
    }
  };
  if (blockIdx.x < ntiles) fetch(blockIdx.x);
  for (int tile_id = blockIdx.x; tile_id < ntiles; tile_id += gridDim.x) {
    const int tx = tile_id % ntx, ty = (tile_id / ntx) % nty, b = tile_id / (ntx * nty);
    const int iy0 = ty * TR, ix0 = tx * TC;
    __syncthreads();  // the previous tile's LDS reads are done
    // dy rows iy0-1 .. iy0+4, columns ix0-1 .. ix0+64 -> LDS
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int q = tid + j * 256;
      const int ch = q % CH, rc = q / CH, col = rc % LC, r = rc / LC;
      if (q < LR * LC * CH) *(uint4*)(tile + (r * LC + col) * COUT + ((ch ^ (col & (CH - 1))) * 8)) = pre[j];
    }
    __syncthreads();
    if (tile_id + (int)gridDim.x < ntiles) fetch(tile_id + gridDim.x);
    const int iy = iy0 + wave;
    f4 acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int dr = t / 3, dc = t % 3;
        const int col = g * 16 + fr + dc;  // LDS column of this lane's pixel, shifted by the tap
        const half_t* row = tile + ((wave + dr) * LC + col) * COUT;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const h8 bv = *(const h8*)(row + (((kc * 4 + fg) ^ (col & (CH - 1))) * 8));
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[kc][t], bv, acc[g], 0, 0, 0);
        }
      }
    if (iy >= H || fg != 0) continue;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ix = ix0 + g * 16 + fr;
      if (ix >= W) continue;
      float* o = dx.d + dx.at(b, iy, ix, 0);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float v = acc[g][c];
        if (accum) v += o[c * dx.sc];
        o[c * dx.sc] = v;
      }
    }
  }
}

int small_conv_dgrad_c3_16(const void* dy16, int B, int H, int W, const float* w, int Cout, const UprView* dxv,
                           int accumulate, hipStream_t st) {
  if ((Cout != 32 && Cout != 64) || ((uintptr_t)dy16 % 16)) return kErrUnsupported;
  if ((long long)B * H * W >= (1ll << 31)) return kErrUnsupported;
  const long long ntiles = (long long)((W + 63) / 64) * ((H + 3) / 4) * B;
  if (ntiles >= (1ll << 31)) return kErrUnsupported;
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // resident blocks per CU: 50 KB of LDS each, and (Cout 64) ~248 VGPRs with the prefetch registers
  const int grid = (int)std::min<long long>(ntiles, (long long)cus * (Cout == 64 ? 2 : 3));
  const SV dx = mksv(dxv);
  if (Cout == 64)
    hipLaunchKernelGGL(dgrad_c3_mfma_kernel<64>, dim3(grid), dim3(256), 0, st, (const half_t*)dy16, B, H, W, w, dx,
                       accumulate);
  else
    hipLaunchKernelGGL(dgrad_c3_mfma_kernel<32>, dim3(grid), dim3(256), 0, st, (const half_t*)dy16, B, H, W, w, dx,
                       accumulate);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// host entries (called from train.hip's upr_t_conv_direct*; kErrUnsupported
// sends the caller to the generic kernels)
// ---------------------------------------------------------------------------
int small_conv_fwd(const UprView* xv, int B, int H, int W, int Cin, const float* w, const float* bias, int Cout,
                   int kh, int kw, int stride, int pad, int dil, const UprView* yv, int Ho, int Wo, int relu,
                   int accumulate, hipStream_t st, void* y16, int skip32) {
  if (y16 && (Cout <= 4 || (uintptr_t)y16 % 8)) return kErrUnsupported;  // fp16 copies: the 3 -> 32 / 64 kernel only
  if (skip32 && !y16) return kErrUnsupported;
  if (Cout <= 4) {
    if ((long long)B * Ho * Wo >= (1ll << 31)) return kErrUnsupported;
    const size_t lds = sizeof(float) * (size_t)Cout * Cin * kh * kw;
    if (lds > 48 * 1024) return kErrUnsupported;
    const SV x = mksv(xv), y = mksv(yv);
    const int xvec = x.sc == 1 && x.sw % 4 == 0 && x.sh % 4 == 0 && x.sb % 4 == 0 && (uintptr_t)x.d % 16 == 0;
    if (xvec && kh == 1 && kw == 1 && stride == 1 && pad == 0 && (Cin == 16 || Cin == 32 || Cin == 64)) {
      const int P = B * Ho * Wo;
      const int hgrid = (P + 255) / 256;
#define UPR_HEAD(C, L) \
  hipLaunchKernelGGL((head1x1_kernel<C, L>), dim3(hgrid), dim3(256), 0, st, x, P, Ho, Wo, w, bias, y, relu, accumulate)
#define UPR_HEAD_C(L)            \
  switch (Cout) {                \
    case 1: UPR_HEAD(1, L); break; \
    case 2: UPR_HEAD(2, L); break; \
    case 3: UPR_HEAD(3, L); break; \
    default: UPR_HEAD(4, L); break; \
  }
      if (Cin == 16) { UPR_HEAD_C(4) } else if (Cin == 32) { UPR_HEAD_C(8) } else { UPR_HEAD_C(16) }
#undef UPR_HEAD_C
#undef UPR_HEAD
      return (int)hipGetLastError();
    }
    const int grid = (B * Ho * Wo + 255) / 256;
#define UPR_SMALL_FWD(C)                                                                                         \
  hipLaunchKernelGGL(small_fwd_kernel<C>, dim3(grid), dim3(256), lds, st, x, B, H, W, Cin, w, bias, kh, kw, stride, \
                     pad, dil, y, Ho, Wo, relu, accumulate, xvec)
    switch (Cout) {
      case 1: UPR_SMALL_FWD(1); break;
      case 2: UPR_SMALL_FWD(2); break;
      case 3: UPR_SMALL_FWD(3); break;
      default: UPR_SMALL_FWD(4); break;
    }
#undef UPR_SMALL_FWD
    return (int)hipGetLastError();
  }
  if (Cin != 3 || kh != 3 || kw != 3 || stride != 1 || dil != 1) return kErrUnsupported;
  if (Cout != 32 && Cout != 64) return kErrUnsupported;
  if (yv->sc != 1 || yv->sw % 4 || yv->sh % 4 || yv->sb % 4 || ((uintptr_t)yv->data % 16)) return kErrUnsupported;
  if ((long long)B * Ho * Wo >= (1ll << 31)) return kErrUnsupported;
  const SV x = mksv(xv), y = mksv(yv);
  const int P = B * Ho * Wo;
  {
    // fp32 MFMA form (16-pixel groups, filter in registers); grid sized for ~8 waves per SIMD
    int cus = 256, dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const long long groups = ((long long)P + 15) / 16;
    const int mgrid = (int)std::min<long long>((groups + 3) / 4, (long long)cus * 8);
    if (Cout == 32)
      hipLaunchKernelGGL(c3k3_mfma_kernel<32>, dim3(mgrid), dim3(256), 0, st, x, B, H, W, w, bias, pad, y, Ho, Wo, relu,
                         accumulate, (half_t*)y16, skip32);
    else
      hipLaunchKernelGGL(c3k3_mfma_kernel<64>, dim3(mgrid), dim3(256), 0, st, x, B, H, W, w, bias, pad, y, Ho, Wo, relu,
                         accumulate, (half_t*)y16, skip32);
    return (int)hipGetLastError();
  }
}

int small_conv_dgrad(const UprView* dyv, int Ho, int Wo, const float* w, int B, int H, int W, int Cin, int Cout,
                     int kh, int kw, int stride, int pad, int dil, const UprView* dxv, int accumulate, hipStream_t st) {
  if (stride != 1) return kErrUnsupported;
  if ((long long)B * H * W >= (1ll << 31)) return kErrUnsupported;
  const size_t lds = sizeof(float) * (size_t)Cout * kh * kw * Cin;
  if (lds > 64 * 1024) return kErrUnsupported;
  const SV dy = mksv(dyv), dx = mksv(dxv);
  const int grid = (B * H * W + 255) / 256;
  const int vec = dx.sc == 1 && dx.sw % 4 == 0 && dx.sh % 4 == 0 && dx.sb % 4 == 0 && (uintptr_t)dx.d % 16 == 0;
  const int dvec = dy.sc == 1 && dy.sw % 4 == 0 && dy.sh % 4 == 0 && dy.sb % 4 == 0 && (uintptr_t)dy.d % 16 == 0;
#define UPR_SMALL_DGRAD(C, CO)                                                                                       \
  hipLaunchKernelGGL((small_dgrad_kernel<C, CO>), dim3(grid), dim3(256), lds, st, dy, Ho, Wo, w, B, H, W, Cout, kh, kw, \
                     pad, dil, dx, accumulate, vec, dvec)
  switch (Cin) {
    case 1: UPR_SMALL_DGRAD(1, 0); break;
    case 2: UPR_SMALL_DGRAD(2, 0); break;
    case 3:
      if (Cout == 64) UPR_SMALL_DGRAD(3, 64);  // VGG-19 conv1_1 (loss.py:198-211)
      else UPR_SMALL_DGRAD(3, 0);
      break;
    case 32: UPR_SMALL_DGRAD(32, 0); break;
    default: return kErrUnsupported;
  }
#undef UPR_SMALL_DGRAD
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// weight gradient of the 7x7 2 -> 1 spatial-attention conv (stride 1, pad 3;
// EnhancedFAM, models/model.py:53,92-95): dW[ci][ky][kx] = sum_p dy[p] *
// x[p + (ky, kx) - 3][ci], db = sum_p dy[p] -- 99 dot products over the
// pixels, 12 bytes per pixel.  The generic MFMA form above spent its time in
// per-pixel index math and per-lane gathers (0.58 ms at bs 8 512^2).  Here a
// block owns an 8 x 64 pixel tile: dy and the (8 + 6) x (64 + 6) x 2 input
// window (zero outside the image) are staged in LDS once, then two threads
// per entry each sum 4 rows of the tile from LDS; one partial row per block
// (part[block][99]), summed in block order by small_wgrad_fin_kernel.
// ---------------------------------------------------------------------------
constexpr int SA_TR = 8, SA_TC = 64, SA_K = 7, SA_P = 3;

__global__ __launch_bounds__(256) void sa_wgrad_kernel(SV x, SV dy, int B, int H, int W, int tiles_x, int tiles_y,
                                                       float* __restrict__ part) {
  constexpr int LR = SA_TR + SA_K - 1, LC = SA_TC + SA_K - 1;
  __shared__ float xs[2][LR][LC + 1];
  __shared__ float ds[SA_TR][SA_TC];
  __shared__ float red[99];
  const int t = threadIdx.x;
  const int tile = blockIdx.x;
  const int tx = tile % tiles_x, rest = tile / tiles_x, ty = rest % tiles_y, b = rest / tiles_y;
  const int y0 = ty * SA_TR, x0 = tx * SA_TC;
  for (int i = t; i < LR * LC; i += 256) {
    const int r = i / LC, c = i - r * LC;  // LDS fill only (once per element)
    const int iy = y0 + r - SA_P, ix = x0 + c - SA_P;
    const bool in = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    xs[0][r][c] = in ? x.d[x.at(b, iy, ix, 0)] : 0.f;
    xs[1][r][c] = in ? x.d[x.at(b, iy, ix, 1)] : 0.f;
  }
  for (int i = t; i < SA_TR * SA_TC; i += 256) {
    const int r = i / SA_TC, c = i - r * SA_TC;
    const int oy = y0 + r, ox = x0 + c;
    ds[r][c] = (oy < H && ox < W) ? dy.d[dy.at(b, oy, ox, 0)] : 0.f;
  }
  if (t < 99) red[t] = 0.f;
  __syncthreads();
  // entry e = ci * 49 + ky * 7 + kx (PyTorch's weight order), e = 98: the bias;
  // threads e and e + 99 take rows 0-3 / 4-7
  float a = 0.f;
  int e = -1;
  if (t < 198) {
    e = t % 99;
    const int r0 = (t / 99) * (SA_TR / 2);
    if (e < 98) {
      const int ci = e / 49, tap = e - ci * 49, ky = tap / 7, kx = tap - ky * 7;
      for (int r = r0; r < r0 + SA_TR / 2; ++r) {
#pragma unroll 8
        for (int c = 0; c < SA_TC; ++c) a = fmaf(ds[r][c], xs[ci][r + ky][c + kx], a);
      }
    } else {
      for (int r = r0; r < r0 + SA_TR / 2; ++r)
#pragma unroll 8
        for (int c = 0; c < SA_TC; ++c) a += ds[r][c];
    }
  }
  // the two halves in a fixed order: rows 0-3 first, then rows 4-7
  if (t < 99) red[t] = a;
  __syncthreads();
  if (t >= 99 && t < 198) red[e] += a;
  __syncthreads();
  if (t < 99) part[(size_t)blockIdx.x * 99 + t] = red[t];
}

// weight gradient of a 1x1 stride-1 conv with Cin * Cout <= 128 (the output
// layer 32 -> 3 and the residual head's 32 -> 1, model.py:326,402):
// dW[co][ci] = sum_p dy[p][co] * x[p][ci] (+ db[co] = sum_p dy[p][co]).  One
// thread per pixel keeps all Cin * Cout (+ Cout) partials in registers; a
// block owns 4 image rows, reduces per entry over its waves (shuffles, then 4
// wave partials in order) into part[block][co * (Cin + 1) + k].
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void pw_wgrad_kernel(SV x, SV dy, int B, int H, int W, int rows_per_block,
                                                       float* __restrict__ part) {
  constexpr int NE = COUT * (CIN + 1);
  __shared__ float wred[4][NE];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  float acc[COUT][CIN + 1];
#pragma unroll
  for (int co = 0; co < COUT; ++co)
#pragma unroll
    for (int k = 0; k <= CIN; ++k) acc[co][k] = 0.f;
  const int row0 = blockIdx.x * rows_per_block;
  const int nrow = B * H;
  for (int rr = 0; rr < rows_per_block; ++rr) {
    const int row = row0 + rr;
    if (row >= nrow) break;
    const int b = row / H, y = row - b * H;  // once per row
    for (int px = t; px < W; px += 256) {
      const float* xp = x.d + x.at(b, y, px, 0);
      float xv[CIN];
#pragma unroll
      for (int c = 0; c < CIN; c += 4) {
        const f32x4_t2 q = *(const f32x4_t2*)(xp + c);
        xv[c] = q[0]; xv[c + 1] = q[1]; xv[c + 2] = q[2]; xv[c + 3] = q[3];
      }
#pragma unroll
      for (int co = 0; co < COUT; ++co) {
        const float g = dy.d[dy.at(b, y, px, co)];
#pragma unroll
        for (int c = 0; c < CIN; ++c) acc[co][c] = fmaf(g, xv[c], acc[co][c]);
        acc[co][CIN] += g;
      }
    }
  }
#pragma unroll
  for (int co = 0; co < COUT; ++co)
#pragma unroll
    for (int k = 0; k <= CIN; ++k) {
      float v = acc[co][k];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) wred[wave][co * (CIN + 1) + k] = v;
    }
  __syncthreads();
  for (int i = t; i < NE; i += 256)
    part[(size_t)blockIdx.x * NE + i] = ((wred[0][i] + wred[1][i]) + wred[2][i]) + wred[3][i];
}

// ---------------------------------------------------------------------------
// weight gradient of the 3 -> 32 3x3 / s1 / p1 image stems with the ReLU
// backward of their output fused: dW[co][ci][tap] = sum_p (dy[p][co] masked by
// y16[p][co] > 0) * x[ci][p + tap], db[co] = sum_p of the masked dy.  A block
// stages a 4 x 64 pixel tile of the masked dy (coalesced 16-byte loads, the
// mask applied on the way into LDS) and the 3 x 6 x 66 input patch, then each
// wave runs v_mfma_f32_32x32x2f32 over its tile row (A = dy rows, B = the
// im2col columns read from the patch at per-lane tap offsets).  Persistent over
// tiles; per-block partials summed in block order by small_wgrad_fin_kernel.
// The generic small_wgrad_mfma_kernel gathered every operand with 4-byte loads
// (0.32 ms per stem at bs 8 512^2, the mask read included).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void stem_wgrad_relu_kernel(SV x, const float* __restrict__ dy,
                                                              const half_t* __restrict__ y16, int B, int H, int W,
                                                              float* __restrict__ part) {
  constexpr int TR = 4, TC = 64, CO = 32, KC = 27;
  __shared__ __attribute__((aligned(16))) float dyl[TR * TC][CO];  // 32 KB; the wave sums reuse it
  __shared__ float xl[3][TR + 2][TC + 2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = lane & 31, kk = lane >> 5;
  // this lane's im2col column n: input channel and tap offsets into the patch
  const int ci = n < KC ? n / 9 : 0, tap = n < KC ? n % 9 : 0, ky = tap / 3, kx = tap % 3;
  f32x16_t2 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  const int ntx = (W + TC - 1) / TC, nty = (H + TR - 1) / TR, ntiles = ntx * nty * B;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tx = t % ntx, ty = (t / ntx) % nty, b = t / (ntx * nty);
    const int iy0 = ty * TR, ix0 = tx * TC;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < (TR * TC * CO / 4) / 256; ++j) {
      const int q = tid + j * 256, px = q >> 3, c4 = (q & 7) * 4;
      const int iy = iy0 + px / TC, ix = ix0 + px % TC;
      f32x4_t2 v = f32x4_t2{0.f, 0.f, 0.f, 0.f};
      if (iy < H && ix < W) {
        const size_t pix = ((size_t)b * H + iy) * W + ix;
        v = *(const f32x4_t2*)(dy + pix * CO + c4);
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        const h4 m = *(const h4*)(y16 + pix * CO + c4);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (!(m[e] > (half_t)0)) v[e] = 0.f;
      }
      *(f32x4_t2*)&dyl[px][c4] = v;
    }
    for (int q = tid; q < 3 * (TR + 2) * (TC + 2); q += 256) {
      const int c = q / ((TR + 2) * (TC + 2)), r = (q / (TC + 2)) % (TR + 2), col = q % (TC + 2);
      const int iy = iy0 - 1 + r, ix = ix0 - 1 + col;
      xl[c][r][col] = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) ? x.d[x.at(b, iy, ix, c)] : 0.f;
    }
    __syncthreads();
    // wave w: tile row w, 32 pixel pairs
#pragma unroll 4
    for (int j = 0; j < TC / 2; ++j) {
      const int col = 2 * j + kk;
      const float a = dyl[wave * TC + col][n];
      const float bv = n < KC ? xl[ci][wave + ky][col + kx] : (n == KC ? 1.f : 0.f);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc, 0, 0, 0);
    }
  }
  __syncthreads();
  float* red = &dyl[0][0];  // [4 waves][16][64]
#pragma unroll
  for (int e = 0; e < 16; ++e) red[(wave * 16 + e) * 64 + lane] = acc[e];
  __syncthreads();
  for (int idx = tid; idx < 16 * 64; idx += 256) {
    const int e = idx >> 6, l = idx & 63;
    const float v = ((red[(0 * 16 + e) * 64 + l] + red[(1 * 16 + e) * 64 + l]) + red[(2 * 16 + e) * 64 + l]) +
                    red[(3 * 16 + e) * 64 + l];
    // 32x32 accumulator map: column = l & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (l >> 5)
    const int co = (e & 3) + 8 * (e >> 2) + 4 * (l >> 5), k = l & 31;
    if (k <= KC) part[(size_t)blockIdx.x * CO * (KC + 1) + co * (KC + 1) + k] = v;
  }
}

int small_stem_wgrad_relu16(const UprView* xv, const float* dy, const void* y16, int B, int H, int W, float* dw,
                            float* dbias, hipStream_t st) {
  if (((uintptr_t)dy % 16) || ((uintptr_t)y16 % 8) || (long long)B * H * W >= (1ll << 31)) return kErrUnsupported;
  const long long ntiles = (long long)((W + 63) / 64) * ((H + 3) / 4) * B;
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = (int)std::min<long long>(ntiles, (long long)cus * 4);
  constexpr int NE = 32 * 28;
  float* part = (float*)scratch(kSlotPart, sizeof(float) * (size_t)grid * NE, st);
  if (!part) return (int)hipErrorOutOfMemory;
  hipLaunchKernelGGL(stem_wgrad_relu_kernel, dim3(grid), dim3(256), 0, st, mksv(xv), dy, (const half_t*)y16, B, H, W,
                     part);
  hipLaunchKernelGGL(small_wgrad_fin_kernel, dim3(NE), dim3(256), 0, st, (const float*)part, grid, 32, 27, dw, dbias);
  return (int)hipGetLastError();
}

int small_conv_wgrad(const UprView* xv, const UprView* dyv, int B, int H, int W, int Cin, int Ho, int Wo, int Cout,
                     int kh, int kw, int stride, int pad, int dil, float* dw, float* dbias, hipStream_t st,
                     const UprView* ymask) {
  if (Cout > 32) return kErrUnsupported;
  SV ym{};
  if (ymask) ym = mksv(ymask);
  if (!ymask) {
    const SV x = mksv(xv), dy = mksv(dyv);
    // the 7x7 spatial-attention conv: LDS-tiled dot products
    if (Cin == 2 && Cout == 1 && kh == SA_K && kw == SA_K && stride == 1 && dil == 1 && pad == SA_P && dbias &&
        Ho == H && Wo == W) {
      const int tx = (W + SA_TC - 1) / SA_TC, ty = (H + SA_TR - 1) / SA_TR;
      const int grid = B * tx * ty;
      float* part = (float*)scratch(kSlotPart, sizeof(float) * (size_t)grid * 99, st);
      if (!part) return (int)hipErrorOutOfMemory;
      hipLaunchKernelGGL(sa_wgrad_kernel, dim3(grid), dim3(256), 0, st, x, dy, B, H, W, tx, ty, part);
      hipLaunchKernelGGL(small_wgrad_fin_kernel, dim3(99), dim3(256), 0, st, (const float*)part, grid, 1, 98, dw,
                         dbias);
      return (int)hipGetLastError();
    }
    // 1x1 heads: one thread per pixel, all partials in registers
    if (kh == 1 && kw == 1 && stride == 1 && pad == 0 && Ho == H && Wo == W && xv->sc == 1 && Cin % 4 == 0 &&
        x.sw % 4 == 0 && x.sh % 4 == 0 && x.sb % 4 == 0 && ((uintptr_t)x.d & 15) == 0 &&
        ((Cin == 32 && (Cout == 1 || Cout == 3)))) {
      const int rows_per_block = 4;
      const int grid = (B * H + rows_per_block - 1) / rows_per_block;
      const int ne = Cout * (Cin + 1);
      float* part = (float*)scratch(kSlotPart, sizeof(float) * (size_t)grid * ne, st);
      if (!part) return (int)hipErrorOutOfMemory;
      if (Cout == 1)
        hipLaunchKernelGGL((pw_wgrad_kernel<32, 1>), dim3(grid), dim3(256), 0, st, x, dy, B, H, W, rows_per_block, part);
      else
        hipLaunchKernelGGL((pw_wgrad_kernel<32, 3>), dim3(grid), dim3(256), 0, st, x, dy, B, H, W, rows_per_block, part);
      hipLaunchKernelGGL(small_wgrad_fin_kernel, dim3(ne), dim3(256), 0, st, (const float*)part, grid, Cout, Cin, dw,
                         dbias);
      return (int)hipGetLastError();
    }
  }
  const int KC = Cin * kh * kw + (dbias ? 1 : 0);
  const int nt = (KC + 31) / 32;
  if (nt > 4) return kErrUnsupported;
  const long long P = (long long)B * Ho * Wo;
  if (P >= (1ll << 30)) return kErrUnsupported;  // the kernel's 32-bit pair / pixel indices
  const long long pairs = (P + 1) / 2;
  // ~4096 waves (16 per CU), pairs per wave a multiple of the unroll
  long long ppw = (pairs + 4095) / 4096;
  const int unroll = nt == 2 ? sw_unroll<2>() : sw_unroll<1>();
  ppw = (ppw + unroll - 1) / unroll * unroll;
  if (ppw < unroll) ppw = unroll;
  const long long waves = (pairs + ppw - 1) / ppw;
  const int grid = (int)((waves + 3) / 4);
  const SV x = mksv(xv), dy = mksv(dyv);
  const int KC0 = Cin * kh * kw;
  float* part = (float*)scratch(kSlotPart, sizeof(float) * (size_t)grid * Cout * (KC0 + 1), st);
  if (!part) return (int)hipErrorOutOfMemory;
#define UPR_SMALL_WGRAD(T)                                                                                          \
  hipLaunchKernelGGL(small_wgrad_mfma_kernel<T>, dim3(grid), dim3(256), 0, st, x, dy, B, H, W, Cin, Ho, Wo, Cout, kh, \
                     kw, stride, pad, dil, (int)ppw, part, ym)
  switch (nt) {
    case 1: UPR_SMALL_WGRAD(1); break;
    case 2: UPR_SMALL_WGRAD(2); break;
    case 3: UPR_SMALL_WGRAD(3); break;
    default: UPR_SMALL_WGRAD(4); break;
  }
#undef UPR_SMALL_WGRAD
  const int nf = Cout * (KC0 + 1);
  hipLaunchKernelGGL(small_wgrad_fin_kernel, dim3(nf), dim3(256), 0, st, (const float*)part, grid, Cout, KC0, dw,
                     dbias);
  return (int)hipGetLastError();
}

}  // namespace upr
