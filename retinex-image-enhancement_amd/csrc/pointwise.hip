// Small fused kernels around the implicit-GEMM convs (gfx950).
//
//  prep_pyramid   bilinear x0.5 / x0.25 (align_corners=False) + MaxPool2 / MaxPool4
//                 inputs of scale2 / scale3 (models/model.py:388,395,421-422)
//  conv3_direct   3->32 3x3 conv + bias + ReLU on a planar 3-channel image
//                 (ie_net.input_layer :298/:335, scale{1,2,3} first conv :382-396)
//  fam_ca         EnhancedFAM channel attention MLP on pooled sums (:47-53, :88)
//  fam_mix        y*ca -> [mean_c, max_c] map + 3-channel head projection (:89-93)
//  fam_sa         7x7 spatial attention conv + sigmoid, scales the projection (:56-59, :94-95)
//  retinex_tail   sigmoid(head) , R = x/(I+1e-6), R*E + (1-R)*E^2 (:411-412, :430-442)
#include <algorithm>
#include <cstdlib>

#include "upr_common.h"

namespace upr {

__device__ __forceinline__ float ldf(const float* p, size_t i) { return p[i]; }
__device__ __forceinline__ float ldf(const half_t* p, size_t i) { return (float)p[i]; }
__device__ __forceinline__ void stf(float* p, size_t i, float v) { p[i] = v; }
__device__ __forceinline__ void stf(half_t* p, size_t i, float v) { p[i] = (half_t)v; }
__device__ __forceinline__ float sigmoidf_(float z) { return 1.f / (1.f + expf(-z)); }

// ---------------------------------------------------------------------------
// prep_pyramid: one thread per (b, c, y, x) of the H/16 image?  No: one thread
// per pixel of the H/4 image; it writes the H/4 pixel and, when (y,x) % 4 == 0
// and in range, also the H/16 pixel.
//   x2  = bilinear(x, 0.5)  -> x2[Y][X]  = mean of x[2Y..2Y+1][2X..2X+1]
//   x2p = MaxPool2(x2)      (H2 = floor(H/2), H4 = floor(H2/2))
//   x3  = bilinear(x, 0.25) -> x3[Y][X]  = mean of x[4Y+1..4Y+2][4X+1..4X+2]
//   x3p = MaxPool4(x3)      (H3 = floor(H/4), H16 = floor(H3/4))
// ---------------------------------------------------------------------------
template <typename TI, typename TO>
__global__ void prep_pyramid_kernel(const TI* __restrict__ x, TO* __restrict__ x2p, TO* __restrict__ x3p,
                                    int B, int H, int W) {
  const int H4 = (H / 2) / 2, W4 = (W / 2) / 2;
  const int H16 = (H / 4) / 4, W16 = (W / 4) / 4;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = B * 3 * H4 * W4;
  if (idx >= total) return;
  const int X = idx % W4;
  const int Y = (idx / W4) % H4;
  const int bc = idx / (W4 * H4);
  const TI* img = x + (size_t)bc * H * W;
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int y2 = 2 * Y + i, x2 = 2 * X + j;  // coords in the H/2 image
      const float a = ldf(img, (size_t)(2 * y2) * W + 2 * x2), b = ldf(img, (size_t)(2 * y2) * W + 2 * x2 + 1);
      const float c = ldf(img, (size_t)(2 * y2 + 1) * W + 2 * x2), d = ldf(img, (size_t)(2 * y2 + 1) * W + 2 * x2 + 1);
      const float v = 0.5f * (0.5f * a + 0.5f * b) + 0.5f * (0.5f * c + 0.5f * d);
      m = fmaxf(m, v);
    }
  stf(x2p, idx, m);
  if ((Y & 3) == 0 && (X & 3) == 0 && (Y >> 2) < H16 && (X >> 2) < W16) {
    const int Ys = Y >> 2, Xs = X >> 2;
    float m3 = -INFINITY;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        const int y3 = 4 * Ys + i, x3 = 4 * Xs + j;  // coords in the H/4 image
        const int r = 4 * y3 + 1, c = 4 * x3 + 1;
        const float a = ldf(img, (size_t)r * W + c), b = ldf(img, (size_t)r * W + c + 1);
        const float cc = ldf(img, (size_t)(r + 1) * W + c), d = ldf(img, (size_t)(r + 1) * W + c + 1);
        const float v = 0.5f * (0.5f * a + 0.5f * b) + 0.5f * (0.5f * cc + 0.5f * d);
        m3 = fmaxf(m3, v);
      }
    stf(x3p, ((size_t)bc * H16 + Ys) * W16 + Xs, m3);
  }
}

// ---------------------------------------------------------------------------
// conv3_direct: planar [B,3,h,w] input -> up to two NHWC [B,h,w,32] outputs,
// each relu(conv3x3(x; w_k) + b_k).  Weights k-major [27][nout*32] fp32, tap k
// in (c,ky,kx) order, read as wave-uniform scalars; channel pairs accumulate with packed
// FMAs.  A block owns 256 consecutive output pixels, whose NHWC rows form one
// contiguous span: results go through LDS and leave as coalesced 16-byte
// chunks (a per-thread 32-channel row store would scatter 16-byte pieces at a
// 64/128-byte lane stride).
// ---------------------------------------------------------------------------
typedef float f2v __attribute__((ext_vector_type(2)));

template <typename TI, typename TO, int NOUT>
__global__ __launch_bounds__(256) void conv3_direct_kernel(const TI* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ bias, TO* __restrict__ out0,
                                                           TO* __restrict__ out1, int B, int h, int wd) {
  constexpr int CPP = 32 * (int)sizeof(TO) / 16;  // 16-byte chunks per output pixel
  constexpr int RS = 9;                           // LDS row stride in 16-byte slots (conflict-free writes)
  __shared__ uint4 stage[256 * RS];
  const int total = B * h * wd;
  const int base = blockIdx.x * 256;
  const int idx = base + threadIdx.x;
  const int npx = total - base < 256 ? total - base : 256;
  float in[27];
  if (idx < total) {
    const int ox = idx % wd, oy = (idx / wd) % h, b = idx / (wd * h);
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int iy = oy + ky - 1, ix = ox + kx - 1;
          in[c * 9 + ky * 3 + kx] = (iy >= 0 && iy < h && ix >= 0 && ix < wd)
                                        ? ldf(x, (((size_t)b * 3 + c) * h + iy) * wd + ix) : 0.f;
        }
  } else {
#pragma unroll
    for (int k = 0; k < 27; ++k) in[k] = 0.f;
  }
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    float r[32];
#pragma unroll
    for (int g = 0; g < 32; g += 2) {
      const int oc = o * 32 + g;
      f2v acc2 = {bias[oc], bias[oc + 1]};
#pragma unroll
      for (int k = 0; k < 27; ++k) {
        const f2v w2 = *(const f2v*)(w + k * (NOUT * 32) + oc);  // k-major weights
        acc2 = __builtin_elementwise_fma((f2v){in[k], in[k]}, w2, acc2);
      }
      r[g] = fmaxf(acc2[0], 0.f);
      r[g + 1] = fmaxf(acc2[1], 0.f);
    }
    uint4* row = stage + threadIdx.x * RS;
#pragma unroll
    for (int c = 0; c < CPP; ++c) {
      uint4 v;
      TO* vv = (TO*)&v;
#pragma unroll
      for (int e = 0; e < 16 / (int)sizeof(TO); ++e) vv[e] = (TO)r[c * (16 / (int)sizeof(TO)) + e];
      row[c] = v;
    }
    __syncthreads();
    uint4* dst = (uint4*)((o == 0 ? out0 : out1) + (size_t)base * 32);
    for (int q = threadIdx.x; q < npx * CPP; q += 256) dst[q] = stage[(q / CPP) * RS + q % CPP];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// fam_ca: ca[b][c] = sigmoid(W2 relu(W1 (pool[b]/HW) + b1) + b2), 32 -> 2 -> 32
// ---------------------------------------------------------------------------
__global__ void fam_ca_kernel(const float* __restrict__ pool, const float* __restrict__ w1,
                              const float* __restrict__ b1, const float* __restrict__ w2,
                              const float* __restrict__ b2, float* __restrict__ ca, int B, float inv_hw) {
  const int b = blockIdx.x;
  const int c = threadIdx.x;  // 32 threads
  if (b >= B || c >= 32) return;
  __shared__ float g[32];
  __shared__ float hdn[2];
  g[c] = pool_get(pool, (size_t)b * 32 + c) * inv_hw;
  __syncthreads();
  if (c < 2) {
    float s = b1[c];
    for (int k = 0; k < 32; ++k) s += w1[c * 32 + k] * g[k];
    hdn[c] = fmaxf(s, 0.f);
  }
  __syncthreads();
  ca[b * 32 + c] = sigmoidf_(b2[c] + w2[c * 2 + 0] * hdn[0] + w2[c * 2 + 1] * hdn[1]);
}

// ---------------------------------------------------------------------------
// fam_mix: per pixel o = y * ca[b]; mm = [mean_c o, max_c o]; p = P o (3 ch)
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void fam_mix_kernel(const T* __restrict__ y, const float* __restrict__ ca,
                                                      const float* __restrict__ P, float* __restrict__ mm,
                                                      float* __restrict__ p, int B, int HW) {
  constexpr int EPC = 16 / (int)sizeof(T);  // channels per 16-byte load
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * HW) return;
  const int b = idx / HW;
  const uint4* yp = (const uint4*)(y + (size_t)idx * 32);
  const float* cab = ca + b * 32;
  float s = 0.f, mx = -INFINITY, p0 = 0.f, p1 = 0.f, p2 = 0.f;
#pragma unroll
  for (int k = 0; k < 32 / EPC; ++k) {
    const uint4 v4 = yp[k];
    const T* v = (const T*)&v4;
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      const int c = k * EPC + e;
      const float o = (float)v[e] * cab[c];
      s += o;
      mx = fmaxf(mx, o);
      p0 += P[c] * o;
      p1 += P[32 + c] * o;
      p2 += P[64 + c] * o;
    }
  }
  *(float2*)(mm + (size_t)idx * 2) = make_float2(s / 32.f, mx);
  p[(size_t)idx * 3] = p0;
  p[(size_t)idx * 3 + 1] = p1;
  p[(size_t)idx * 3 + 2] = p2;
}

// ---------------------------------------------------------------------------
// fam_sa: sa = sigmoid(conv7x7([mean,max]) + b), q = sa * p   (zero padding 3)
// weights w[2][7][7] (channel 0 = mean, 1 = max)
// ---------------------------------------------------------------------------
constexpr int SA_TW = 32, SA_TH = 8;
__global__ __launch_bounds__(256) void fam_sa_kernel(const float* __restrict__ mm, const float* __restrict__ p,
                                                     const float* __restrict__ w, float bias,
                                                     float* __restrict__ q, int B, int h, int wd) {
  // one block = a 32 x 8 output tile; the [mean,max] map of the tile + 3-pixel
  // halo is staged in LDS (zero outside the image = the conv's zero padding)
  constexpr int RW = SA_TW + 6, RH = SA_TH + 6;
  __shared__ float2 reg[RH * RW];
  const int b = blockIdx.z, oy0 = blockIdx.y * SA_TH, ox0 = blockIdx.x * SA_TW;
  const float2* mmb = (const float2*)mm + (size_t)b * h * wd;
  for (int i = threadIdx.x; i < RH * RW; i += 256) {
    const int iy = oy0 - 3 + i / RW, ix = ox0 - 3 + i % RW;
    reg[i] = (iy >= 0 && iy < h && ix >= 0 && ix < wd) ? mmb[(size_t)iy * wd + ix] : make_float2(0.f, 0.f);
  }
  __syncthreads();
  const int ty = threadIdx.x / SA_TW, tx = threadIdx.x % SA_TW;
  const int oy = oy0 + ty, ox = ox0 + tx;
  if (oy >= h || ox >= wd) return;
  float s = bias;
#pragma unroll
  for (int ky = 0; ky < 7; ++ky)
#pragma unroll
    for (int kx = 0; kx < 7; ++kx) {
      const float2 v = reg[(ty + ky) * RW + tx + kx];
      s += w[ky * 7 + kx] * v.x + w[49 + ky * 7 + kx] * v.y;
    }
  const float sa = sigmoidf_(s);
  const size_t idx = ((size_t)b * h + oy) * wd + ox;
  q[idx * 3] = sa * p[idx * 3];
  q[idx * 3 + 1] = sa * p[idx * 3 + 1];
  q[idx * 3 + 2] = sa * p[idx * 3 + 2];
}

// bilinear source coordinate, align_corners=False, size-based (in/out ratio)
__device__ __forceinline__ void src_idx(int d, int in, float scale, int& i0, int& i1, float& l1) {
  float s = scale * (d + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = s - (float)i0;
}

__device__ __forceinline__ float bilerp3(const float* q, int b, int h, int wd, int c, int y0, int y1, float ly,
                                         int x0, int x1, float lx) {
  const float* base = q + (size_t)b * h * wd * 3 + c;
  const float v00 = base[((size_t)y0 * wd + x0) * 3], v01 = base[((size_t)y0 * wd + x1) * 3];
  const float v10 = base[((size_t)y1 * wd + x0) * 3], v11 = base[((size_t)y1 * wd + x1) * 3];
  return (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
}

// ---------------------------------------------------------------------------
// retinex_tail: per output pixel and channel.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void retinex_tail_kernel(const T* __restrict__ x, const float* __restrict__ illu_f32,
                                                           const T* __restrict__ illu_t,
                                                           const float* __restrict__ q1, const float* __restrict__ q2,
                                                           const float* __restrict__ q3, const float* __restrict__ cst,
                                                           T* __restrict__ enh, T* __restrict__ refl,
                                                           int B, int H, int W, int h2, int w2, int h3, int w3,
                                                           int refl_in) {
  // 2-D grid (64 x 4 pixels per block, z = image): no per-pixel div / mod
  const int ox = blockIdx.x * 64 + (threadIdx.x & 63), oy = blockIdx.y * 4 + (threadIdx.x >> 6), b = blockIdx.z;
  if (ox >= W || oy >= H) return;
  const size_t idx = ((size_t)b * H + oy) * W + ox;
  int ay0, ay1, ax0, ax1, by0, by1, bx0, bx1;
  float aly, alx, bly, blx;
  src_idx(oy, h2, (float)h2 / (float)H, ay0, ay1, aly);
  src_idx(ox, w2, (float)w2 / (float)W, ax0, ax1, alx);
  src_idx(oy, h3, (float)h3 / (float)H, by0, by1, bly);
  src_idx(ox, w3, (float)w3 / (float)W, bx0, bx1, blx);
  // refl_in (multi_scale_enhance, models/model.py:415-443): R is the caller's
  // reflectance, read instead of x / (I + 1e-6) and not written
  const float il = refl_in ? 0.f : (illu_t ? ldf(illu_t, idx) : illu_f32[idx]);
  const size_t HW = (size_t)H * W;
  const size_t pix = (size_t)oy * W + ox;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float z = q1[(size_t)idx * 3 + c] + bilerp3(q2, b, h2, w2, c, ay0, ay1, aly, ax0, ax1, alx) +
              bilerp3(q3, b, h3, w3, c, by0, by1, bly, bx0, bx1, blx) + cst[c];
    const float e = sigmoidf_(z);
    const size_t o = ((size_t)b * 3 + c) * HW + pix;
    float r;
    if (refl_in) {
      r = ldf(refl, o);
    } else {
      r = ldf(x, o) / (il + 1e-6f);
      stf(refl, o, r);
    }
    stf(enh, o, r * e + (1.f - r) * (e * e));
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
static inline int grid1d(size_t n) { return (int)((n + 255) / 256); }

int launch_prep(const void* x, void* x2p, void* x3p, int B, int H, int W, int dtype, hipStream_t st) {
  const int n = B * 3 * ((H / 2) / 2) * ((W / 2) / 2);
  if (n <= 0) return kErrShape;
  if (dtype == kF16)
    hipLaunchKernelGGL((prep_pyramid_kernel<half_t, half_t>), dim3(grid1d(n)), dim3(256), 0, st,
                       (const half_t*)x, (half_t*)x2p, (half_t*)x3p, B, H, W);
  else
    hipLaunchKernelGGL((prep_pyramid_kernel<float, float>), dim3(grid1d(n)), dim3(256), 0, st,
                       (const float*)x, (float*)x2p, (float*)x3p, B, H, W);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// fp16 3 -> 32/64 first convs on MFMA (input_layer + scale1.0 in one launch,
// scale2.1 / scale3.1; models/model.py:296, :380-390).  A block owns an 8 x 32
// output tile; the 3 x 10 x 34 input region (planar, zero padded) sits in
// LDS; K = 27 taps x channels padded to 32 = one v_mfma_f32_16x16x32_f16 per
// (16 pixels, 16 outputs), weights as the A operand (in registers), pixels as
// B, so each lane ends with 4 consecutive output channels of one pixel and
// stores 8-byte runs.  Optionally also writes o = relu(bn1(out0)) (the enc1
// PreAct prologue, rounded exactly like OP_PREACT: from the stored fp16 value).
// ---------------------------------------------------------------------------
template <int NO, bool NTS>
__global__ __launch_bounds__(256) void conv3_mfma_kernel(const half_t* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ bias, half_t* __restrict__ out0,
                                                         half_t* __restrict__ out1, half_t* __restrict__ out2,
                                                         const float* __restrict__ ps, const float* __restrict__ ph,
                                                         int h, int wd, int tiles_x, int tiles_y, int nimg) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int NT = NO * 2, RW = 34, RH = 10, RP = RW * RH;
  __shared__ half_t reg[3 * RP];
  __shared__ __attribute__((aligned(16))) half_t tr[4][3][16 * 32];  // per-wave 16-pixel transpose, <= 3 outputs
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fg = lane >> 4;
  const size_t HW = (size_t)h * wd;
  const int ntiles = tiles_x * tiles_y * nimg;
  // persistent: the filter / bias / tap offsets are set up once per block and
  // the next tile's input region is prefetched into registers (4 halves per
  // thread) while the current tile computes and stores
  constexpr int RPT = (3 * RP + 255) / 256;
  auto fetch = [&](int t, half_t (&pre)[RPT]) {
    const int tx = t % tiles_x, ty = (t / tiles_x) % tiles_y, b = t / (tiles_x * tiles_y);
    const int oy0 = ty * 8, ox0 = tx * 32;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int e = tid + j * 256;
      half_t v = (half_t)0.f;
      if (e < 3 * RP) {
        const int c = e / RP, r = e - c * RP, hy = r / RW, hx = r - hy * RW;
        const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
        if ((unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)wd)
          v = x[((size_t)b * 3 + c) * HW + (size_t)iy * wd + ix];
      }
      pre[j] = v;
    }
  };
  half_t pre[RPT];
  int t = blockIdx.x;
  if (t < ntiles) fetch(t, pre);
  h8 wf[NT];
  float bv[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = fg * 8 + e;
      wf[nt][e] = k < 27 ? (half_t)w[k * (NO * 32) + nt * 16 + fr] : (half_t)0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[nt][i] = bias[nt * 16 + fg * 4 + i];
  }
  int koff[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = fg * 8 + e, c = k / 9, ky = (k % 9) / 3, kx = k % 3;
    koff[e] = k < 27 ? c * RP + ky * RW + kx : -1;
  }
  for (; t < ntiles; t += gridDim.x) {
  const int tx = t % tiles_x, ty = (t / tiles_x) % tiles_y, b = t / (tiles_x * tiles_y);
  const int oy0 = ty * 8, ox0 = tx * 32;
  __syncthreads();  // every wave is done with the previous tile's region
#pragma unroll
  for (int j = 0; j < RPT; ++j)
    if (tid + j * 256 < 3 * RP) reg[tid + j * 256] = pre[j];
  __syncthreads();
  if (t + (int)gridDim.x < ntiles) fetch(t + gridDim.x, pre);
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int gy = wave * 2 + (g >> 1), gx = (g & 1) * 16 + fr;
    h8 xf;
#pragma unroll
    for (int e = 0; e < 8; ++e) xf[e] = koff[e] >= 0 ? reg[koff[e] + gy * RW + gx] : (half_t)0.f;
    f4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nt], xf, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    // transpose through this wave's LDS scratch: lane (pixel fr, channels
    // 4fg..4fg+3 of tile nt) -> lane l stores 16 bytes (pixel l/4, channels
    // 8(l%4)..): every store instruction writes the group's 1 KiB run of one
    // output contiguously
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      h4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = (half_t)fmaxf(acc[nt][i] + bv[nt][i], 0.f);
      *(h4*)(&tr[wave][nt >> 1][fr * 32 + (nt & 1) * 16 + fg * 4]) = o;
      if (out2 && nt < 2) {
        h4 q;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = nt * 16 + fg * 4 + i;
          q[i] = (half_t)fmaxf((float)o[i] * ps[c] + ph[c], 0.f);
        }
        *(h4*)(&tr[wave][2][fr * 32 + nt * 16 + fg * 4]) = q;
      }
    }
    const int y = oy0 + gy, xs = ox0 + (g & 1) * 16 + (lane >> 2);
    if (y < h && xs < wd) {
      const size_t off = ((size_t)b * HW + (size_t)y * wd + xs) * 32 + (lane & 3) * 8;
      if constexpr (NTS) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(*(const u4*)(&tr[wave][0][lane * 8]), (u4*)(out0 + off));
        if (NO == 2) __builtin_nontemporal_store(*(const u4*)(&tr[wave][1][lane * 8]), (u4*)(out1 + off));
        if (out2) __builtin_nontemporal_store(*(const u4*)(&tr[wave][2][lane * 8]), (u4*)(out2 + off));
      } else {
        *(h8*)(out0 + off) = *(const h8*)(&tr[wave][0][lane * 8]);
        if (NO == 2) *(h8*)(out1 + off) = *(const h8*)(&tr[wave][1][lane * 8]);
        if (out2) *(h8*)(out2 + off) = *(const h8*)(&tr[wave][2][lane * 8]);
      }
    }
  }
  }
}

int launch_conv3(const void* x, const float* w, const float* bias, void* out0, void* out1, int B, int h, int wd,
                 int dtype, hipStream_t st, void* out2, const float* ps, const float* ph) {
  const int n = B * h * wd;
  if (n <= 0) return kErrShape;
  if (dtype == kF16) {
    const int tx = cdiv(wd, 32), ty = cdiv(h, 8);
    // persistent grid: one wave of resident blocks (108 / 80 VGPRs -> 4 / 6 blocks per CU)
    const int grid = std::min(B * tx * ty, 256 * (out1 ? 4 : 6));
    // non-temporal output stores (measured 0.355 -> 0.313 ms at bs 32 512^2; the
    // three 1 GB outputs do not fit the caches anyway)
    if (out1)
      hipLaunchKernelGGL((conv3_mfma_kernel<2, true>), dim3(grid), dim3(256), 0, st, (const half_t*)x, w, bias,
                         (half_t*)out0, (half_t*)out1, (half_t*)out2, ps, ph, h, wd, tx, ty, B);
    else
      hipLaunchKernelGGL((conv3_mfma_kernel<1, false>), dim3(grid), dim3(256), 0, st, (const half_t*)x, w, bias,
                         (half_t*)out0, (half_t*)nullptr, (half_t*)out2, ps, ph, h, wd, tx, ty, B);
    return (int)hipGetLastError();
  }
  if (out2) return kErrUnsupported;  // the fused PreAct output exists on the MFMA path only
  if (dtype == kF16) {
    if (out1)
      hipLaunchKernelGGL((conv3_direct_kernel<half_t, half_t, 2>), dim3(grid1d(n)), dim3(256), 0, st,
                         (const half_t*)x, w, bias, (half_t*)out0, (half_t*)out1, B, h, wd);
    else
      hipLaunchKernelGGL((conv3_direct_kernel<half_t, half_t, 1>), dim3(grid1d(n)), dim3(256), 0, st,
                         (const half_t*)x, w, bias, (half_t*)out0, (half_t*)nullptr, B, h, wd);
  } else {
    if (out1)
      hipLaunchKernelGGL((conv3_direct_kernel<float, float, 2>), dim3(grid1d(n)), dim3(256), 0, st,
                         (const float*)x, w, bias, (float*)out0, (float*)out1, B, h, wd);
    else
      hipLaunchKernelGGL((conv3_direct_kernel<float, float, 1>), dim3(grid1d(n)), dim3(256), 0, st,
                         (const float*)x, w, bias, (float*)out0, (float*)nullptr, B, h, wd);
  }
  return (int)hipGetLastError();
}

int launch_fam_ca(const float* pool, const float* w1, const float* b1, const float* w2, const float* b2, float* ca,
                  int B, int HW, hipStream_t st) {
  hipLaunchKernelGGL(fam_ca_kernel, dim3(B), dim3(32), 0, st, pool, w1, b1, w2, b2, ca, B, 1.f / (float)HW);
  return (int)hipGetLastError();
}

int launch_fam_mix(const void* y, const float* ca, const float* P, float* mm, float* p, int B, int HW, int dtype,
                   hipStream_t st) {
  const int n = B * HW;
  if (dtype == kF16)
    hipLaunchKernelGGL((fam_mix_kernel<half_t>), dim3(grid1d(n)), dim3(256), 0, st, (const half_t*)y, ca, P, mm, p,
                       B, HW);
  else
    hipLaunchKernelGGL((fam_mix_kernel<float>), dim3(grid1d(n)), dim3(256), 0, st, (const float*)y, ca, P, mm, p, B,
                       HW);
  return (int)hipGetLastError();
}

int launch_fam_sa(const float* mm, const float* p, const float* w, float bias, float* q, int B, int h, int wd,
                  hipStream_t st) {
  if (B <= 0 || h <= 0 || wd <= 0) return kErrShape;
  hipLaunchKernelGGL(fam_sa_kernel, dim3(cdiv(wd, SA_TW), cdiv(h, SA_TH), B), dim3(256), 0, st, mm, p, w, bias, q, B,
                     h, wd);
  return (int)hipGetLastError();
}

int launch_tail(const void* x, const float* illu_f32, const void* illu_t, const float* q1, const float* q2,
                const float* q3, const float* cst, void* enh, void* refl, int B, int H, int W, int h2, int w2, int h3,
                int w3, int dtype, hipStream_t st, int refl_in) {
  if (B <= 0 || H <= 0 || W <= 0) return kErrShape;
  const dim3 grid(cdiv(W, 64), cdiv(H, 4), B);
  if (dtype == kF16)
    hipLaunchKernelGGL((retinex_tail_kernel<half_t>), grid, dim3(256), 0, st, (const half_t*)x, illu_f32,
                       (const half_t*)illu_t, q1, q2, q3, cst, (half_t*)enh, (half_t*)refl, B, H, W, h2, w2, h3, w3,
                       refl_in);
  else
    hipLaunchKernelGGL((retinex_tail_kernel<float>), grid, dim3(256), 0, st, (const float*)x, illu_f32,
                       (const float*)illu_t, q1, q2, q3, cst, (float*)enh, (float*)refl, B, H, W, h2, w2, h3, w3,
                       refl_in);
  return (int)hipGetLastError();
}

// MultiScaleUP_Retinex.retinex_decompose (models/model.py:405-413) called on
// its own: refl = x / (illu + 1e-6) over [B,C,H,W], illu [B,illu_c,H,W] with
// illu_c 1 (broadcast over C, the reference's use) or C; fp32 arithmetic, one
// rounding to the tensor dtype.  Backward: dx = g / d, dillu = -sum_c g*x / d^2
// (the sum over c when illu is broadcast), d = illu + 1e-6.  One thread per
// (image, pixel) walks the channels.
template <typename T>
__global__ __launch_bounds__(256) void decompose_kernel(const T* __restrict__ x, const T* __restrict__ illu,
                                                        T* __restrict__ refl, int B, int C, int HW, int illu_c) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * HW) return;
  const long long b = i / HW, p = i - b * HW;
  for (int c = 0; c < C; ++c) {
    const long long o = (b * C + c) * HW + p;
    const float d = ldf(illu, (b * illu_c + (illu_c == 1 ? 0 : c)) * HW + p) + 1e-6f;
    stf(refl, o, ldf(x, o) / d);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void decompose_bwd_kernel(const T* __restrict__ x, const T* __restrict__ illu,
                                                            const T* __restrict__ g, T* __restrict__ gx,
                                                            T* __restrict__ gillu, int B, int C, int HW, int illu_c) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * HW) return;
  const long long b = i / HW, p = i - b * HW;
  float acc = 0.f;
  for (int c = 0; c < C; ++c) {
    const long long o = (b * C + c) * HW + p;
    const long long io = (b * illu_c + (illu_c == 1 ? 0 : c)) * HW + p;
    const float d = ldf(illu, io) + 1e-6f;
    const float gv = ldf(g, o);
    if (gx) stf(gx, o, gv / d);
    const float gi = -gv * ldf(x, o) / (d * d);
    if (illu_c == 1) acc += gi;
    else if (gillu) stf(gillu, io, gi);
  }
  if (illu_c == 1 && gillu) stf(gillu, b * HW + p, acc);
}

int launch_decompose(const void* x, const void* illu, void* refl, int B, int C, int HW, int illu_c, int dtype,
                     hipStream_t st) {
  const int grid = (int)(((long long)B * HW + 255) / 256);
  if (dtype == kF16)
    hipLaunchKernelGGL((decompose_kernel<half_t>), dim3(grid), dim3(256), 0, st, (const half_t*)x, (const half_t*)illu,
                       (half_t*)refl, B, C, HW, illu_c);
  else
    hipLaunchKernelGGL((decompose_kernel<float>), dim3(grid), dim3(256), 0, st, (const float*)x, (const float*)illu,
                       (float*)refl, B, C, HW, illu_c);
  return (int)hipGetLastError();
}

int launch_decompose_bwd(const void* x, const void* illu, const void* g, void* gx, void* gillu, int B, int C, int HW,
                         int illu_c, int dtype, hipStream_t st) {
  const int grid = (int)(((long long)B * HW + 255) / 256);
  if (dtype == kF16)
    hipLaunchKernelGGL((decompose_bwd_kernel<half_t>), dim3(grid), dim3(256), 0, st, (const half_t*)x,
                       (const half_t*)illu, (const half_t*)g, (half_t*)gx, (half_t*)gillu, B, C, HW, illu_c);
  else
    hipLaunchKernelGGL((decompose_bwd_kernel<float>), dim3(grid), dim3(256), 0, st, (const float*)x,
                       (const float*)illu, (const float*)g, (float*)gx, (float*)gillu, B, C, HW, illu_c);
  return (int)hipGetLastError();
}

// PreActResBlock prologue materialised (models/model.py:164-166):
// o = relu(bn1(x)) with the eval BatchNorm folded to (scale, shift), fp16 NHWC,
// 8 channels per thread (16-byte loads / stores).  Rounds exactly like the
// per-tap prologue of conv.hip / conv_halo.hip (fp32 math, one fp16 rounding).
__global__ __launch_bounds__(256) void preact_kernel(const half_t* __restrict__ x, const float* __restrict__ sc,
                                                     const float* __restrict__ sh, half_t* __restrict__ o, size_t n8,
                                                     int C8) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C8) * 8;
    const h8 v = ((const h8*)x)[i];
    h8 r;
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = (half_t)fmaxf(__builtin_fmaf((float)v[e], sc[c + e], sh[c + e]), 0.f);
    ((h8*)o)[i] = r;
  }
}

int launch_preact_f16(const void* x, const float* sc, const float* sh, void* o, size_t npix, int C, hipStream_t st) {
  if (C % 8) return kErrShape;
  const size_t n8 = npix * (C / 8);
  const int grid = (int)std::min<size_t>((n8 + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(preact_kernel, dim3(grid), dim3(256), 0, st, (const half_t*)x, sc, sh, (half_t*)o, n8, C / 8);
  return (int)hipGetLastError();
}

}  // namespace upr
