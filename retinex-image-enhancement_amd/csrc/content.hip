// Content-aware enhancer kernels (gfx950), enhancers/content_aware.py:19-122.
//
//   gray (cv2 BGR2GRAY 8U) -> |Laplacian ksize=1| (CV_64F, BORDER_REFLECT_101)
//   -> GaussianBlur 15x15 sigma 0 (=> 2.6), CV_64F, REFLECT_101, separable
//   -> min-max normalise (fp64) -> float32 saliency
//   attention = saliency * (1 / (luminance + 0.1)), min-max normalised (fp32)
//   out = clamp(enh * (1 + 0.2 * attention), 0, 1)
// Per image (the reference runs B = 1 and normalises over the whole tensor).
// Built with -ffp-contract=off so the fp64/fp32 operation order follows
// OpenCV's RowFilter / SymmColumnFilter and torch's CPU elementwise ops.
#include <cfloat>
#include <cmath>
#include <cstdlib>

#include "upr_common.h"

namespace upr {

__device__ __forceinline__ float ldf(const float* p, size_t i) { return p[i]; }
__device__ __forceinline__ float ldf(const half_t* p, size_t i) { return (float)p[i]; }
__device__ __forceinline__ void stf(float* p, size_t i, float v) { p[i] = v; }
__device__ __forceinline__ void stf(half_t* p, size_t i, float v) { p[i] = (half_t)v; }

__device__ __forceinline__ int quant_u8c(float v) {
  const float t = v * 255.f;
  if (!(fabsf(t) < 2147483648.f)) return 0;
  return ((int)t) & 255;
}

__device__ __forceinline__ int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * (n - 1) - i;
  return i;
}

template <typename T>
__device__ __forceinline__ int gray_at(const T* img, int H, int W, int y, int x) {
  const size_t HW = (size_t)H * W, p = (size_t)y * W + x;
  const int r = quant_u8c(ldf(img, p)), g = quant_u8c(ldf(img, HW + p)), b = quant_u8c(ldf(img, 2 * HW + p));
  return (b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14;
}

// |Laplacian| of the 8-bit gray image, fp64
template <typename T>
__global__ __launch_bounds__(256) void ca_lap_kernel(const T* __restrict__ x, double* __restrict__ lap, int B, int H,
                                                     int W) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * H * W) return;
  const int b = idx / (H * W), p = idx - b * H * W;
  const int y = p / W, xx = p - y * W;
  const T* img = x + (size_t)b * 3 * H * W;
  const int c = gray_at(img, H, W, y, xx);
  const int u = gray_at(img, H, W, refl101(y - 1, H), xx), d = gray_at(img, H, W, refl101(y + 1, H), xx);
  const int l = gray_at(img, H, W, y, refl101(xx - 1, W)), r = gray_at(img, H, W, y, refl101(xx + 1, W));
  lap[idx] = fabs((double)(u + l - 4 * c + r + d));
}

struct GaussK {
  double k[15];
};

// RowFilter: s = k0*S[x-7] + k1*S[x-6] + ... (tap order)
__global__ __launch_bounds__(256) void ca_gauss_rows(const double* __restrict__ in, double* __restrict__ out, int B,
                                                     int H, int W, GaussK g) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * H * W) return;
  const int row = idx / W, x = idx - row * W;
  const double* s = in + (size_t)row * W;
  double acc = g.k[0] * s[refl101(x - 7, W)];
  for (int k = 1; k < 15; ++k) acc += g.k[k] * s[refl101(x - 7 + k, W)];
  out[idx] = acc;
}

// SymmColumnFilter: s = ky[c]*S[y] + 0.0; s += ky[c+k]*(S[y+k] + S[y-k]); + per-block min/max
__global__ __launch_bounds__(256) void ca_gauss_cols(const double* __restrict__ in, double* __restrict__ out, int H,
                                                     int W, GaussK g, double* __restrict__ part, int nblk) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  double mn = DBL_MAX, mx = -DBL_MAX;
  if (p < H * W) {
    const int y = p / W, x = p - y * W;
    const double* img = in + (size_t)b * H * W;
    double acc = g.k[7] * img[(size_t)y * W + x] + 0.0;
    for (int k = 1; k <= 7; ++k)
      acc += g.k[7 + k] * (img[(size_t)refl101(y + k, H) * W + x] + img[(size_t)refl101(y - k, H) * W + x]);
    out[(size_t)b * H * W + p] = acc;
    mn = mx = acc;
  }
  __shared__ double smn[256], smx[256];
  smn[threadIdx.x] = mn;
  smx[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      smn[threadIdx.x] = fmin(smn[threadIdx.x], smn[threadIdx.x + s]);
      smx[threadIdx.x] = fmax(smx[threadIdx.x], smx[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[((size_t)b * nblk + blockIdx.x) * 2] = smn[0];
    part[((size_t)b * nblk + blockIdx.x) * 2 + 1] = smx[0];
  }
}

// Fused saliency pass (round 6): gray -> |Laplacian| -> 15-tap Gaussian rows
// -> 15-tap Gaussian columns for a 64 x 64 output tile in one block, every
// intermediate in LDS: the tile's gray region (tile + 8 on each side, image
// coordinates reflected 101) is computed from the image once, the Laplacian
// over the tile + 7 (a reflected region position's Laplacian equals the
// Laplacian at the reflected position: the stencil is symmetric), then the
// row and column passes in the order and fp64 arithmetic of ca_gauss_rows /
// ca_gauss_cols (bit-identical outputs).  HBM: the image once (12 B/px, the
// halo from L2) and the fp64 map once (8 B/px), against 52 B/px for the
// three-kernel form.  Per-block fp64 min / max partials as ca_gauss_cols.
// The Laplacian is an integer of at most 2040: LDS holds it as fp32 (exact;
// the row pass widens each value to fp64 as it loads it), and 4-wide rows
// (gray as int4 / lap as float4 reads, rows padded to 80 entries so every
// quad is 16-byte aligned).  The pass is fp64-issue-bound (SQ counters,
// profiles/r6_content_aware_*): 64-row tiles of 512 threads spend 1.25 row-
// pass outputs per pixel against 1.5 for 32-row tiles (the 14-row halo),
// 63 KiB of LDS per block, two blocks (16 waves) per CU.
constexpr int CA_TH = 64, CA_TW = 64, CA_R = 7, CA_NT = 512;
constexpr int CA_GH = CA_TH + 2 * CA_R + 2, CA_GW = CA_TW + 2 * CA_R + 2;  // 48 x 80 gray region
constexpr int CA_LH = CA_TH + 2 * CA_R, CA_LW = CA_TW + 2 * CA_R;          // 46 x 78 Laplacian region
constexpr int CA_LP = 80;                                                  // its padded row
static_assert(CA_GW == CA_LP && CA_LW <= CA_LP, "lap row quads");

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float (&v)[4]);
template <>
__device__ __forceinline__ void ld4<float>(const float* p, float (&v)[4]) {
  const float4 q = *(const float4*)p;
  v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
}
template <>
__device__ __forceinline__ void ld4<half_t>(const half_t* p, float (&v)[4]) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const h4 q = *(const h4*)p;
  v[0] = (float)q[0]; v[1] = (float)q[1]; v[2] = (float)q[2]; v[3] = (float)q[3];
}

template <typename T>
__global__ __launch_bounds__(CA_NT) void ca_sal_fused_kernel(const T* __restrict__ x, double* __restrict__ sal, int H,
                                                           int W, int tiles_x, GaussK g, double* __restrict__ part,
                                                           int nblk) {
  // the gray region and the row-pass output are never live together: one
  // buffer (gray: 15 KiB of its 23 KiB; the lap pass's quad reads of a row's
  // last quad run 4 entries into the next row, or past the last row, inside it)
  __shared__ __attribute__((aligned(16))) double rowg[CA_LH][CA_TW];
  __shared__ __attribute__((aligned(16))) float lap[CA_LH][CA_LP];  // 14.4 KiB
  static_assert(CA_LH * CA_TW * 8 >= (CA_GH * CA_GW + 4) * 4, "gray quad over-read stays in rowg");
  int(*gray)[CA_GW] = (int(*)[CA_GW])&rowg[0][0];
  const int t = threadIdx.x;
  const int b = blockIdx.y;
  const int ty0 = (blockIdx.x / tiles_x) * CA_TH, tx0 = (blockIdx.x % tiles_x) * CA_TW;
  const size_t HW = (size_t)H * W;
  const T* img = x + (size_t)b * 3 * HW;
  const int gy0 = ty0 - CA_R - 1, gx0 = tx0 - CA_R - 1;
  // (1) gray of the region; interior tiles load 4-pixel quads (gx0 is 8-aligned).
  // Every load of a thread is issued before the first gray is formed (one HBM
  // round trip per block: a runtime-trip-count loop waited for each quad's
  // loads in turn and made this pass latency-bound)
  if (gy0 >= 0 && gx0 >= 0 && gy0 + CA_GH <= H && gx0 + CA_GW <= W && (W & 3) == 0) {
    constexpr int QPR = CA_GW / 4, NQ = CA_GH * QPR, NI = (NQ + CA_NT - 1) / CA_NT;
    float r[NI][4], gg[NI][4], bb[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = t + CA_NT * i < NQ ? t + CA_NT * i : NQ - 1;
      const int ry = q / QPR, rq = q - ry * QPR;
      const size_t o = (size_t)(gy0 + ry) * W + gx0 + 4 * rq;
      ld4<T>(img + o, r[i]);
      ld4<T>(img + HW + o, gg[i]);
      ld4<T>(img + 2 * HW + o, bb[i]);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = t + CA_NT * i;
      if (q < NQ) {
        const int ry = q / QPR, rq = q - ry * QPR;
        int4 gq;
        gq.x = (quant_u8c(bb[i][0]) * 1868 + quant_u8c(gg[i][0]) * 9617 + quant_u8c(r[i][0]) * 4899 + (1 << 13)) >> 14;
        gq.y = (quant_u8c(bb[i][1]) * 1868 + quant_u8c(gg[i][1]) * 9617 + quant_u8c(r[i][1]) * 4899 + (1 << 13)) >> 14;
        gq.z = (quant_u8c(bb[i][2]) * 1868 + quant_u8c(gg[i][2]) * 9617 + quant_u8c(r[i][2]) * 4899 + (1 << 13)) >> 14;
        gq.w = (quant_u8c(bb[i][3]) * 1868 + quant_u8c(gg[i][3]) * 9617 + quant_u8c(r[i][3]) * 4899 + (1 << 13)) >> 14;
        *(int4*)&gray[ry][4 * rq] = gq;
      }
    }
  } else {
    constexpr int NP = CA_GH * CA_GW, NI = (NP + CA_NT - 1) / CA_NT;
    float r[NI], gg[NI], bb[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = t + CA_NT * k < NP ? t + CA_NT * k : NP - 1;
      const int ry = i / CA_GW, rx = i - ry * CA_GW;
      const size_t o = (size_t)refl101(gy0 + ry, H) * W + refl101(gx0 + rx, W);
      r[k] = ldf(img, o);
      gg[k] = ldf(img, HW + o);
      bb[k] = ldf(img, 2 * HW + o);
    }
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = t + CA_NT * k;
      if (i < NP) {
        const int ry = i / CA_GW, rx = i - ry * CA_GW;
        gray[ry][rx] = (quant_u8c(bb[k]) * 1868 + quant_u8c(gg[k]) * 9617 + quant_u8c(r[k]) * 4899 + (1 << 13)) >> 14;
      }
    }
  }
  __syncthreads();
  // (2) |Laplacian| over the tile + 7, four consecutive entries per item (the
  // padded entries 78, 79 of a row are never read)
  for (int i = t; i < CA_LH * (CA_LP / 4); i += CA_NT) {
    const int ly = i / (CA_LP / 4), lx = (i - ly * (CA_LP / 4)) * 4;
    int u[8], m[8], d[8];
    *(int4*)&u[0] = *(const int4*)&gray[ly][lx];
    *(int4*)&u[4] = *(const int4*)&gray[ly][lx + 4];
    *(int4*)&m[0] = *(const int4*)&gray[ly + 1][lx];
    *(int4*)&m[4] = *(const int4*)&gray[ly + 1][lx + 4];
    *(int4*)&d[0] = *(const int4*)&gray[ly + 2][lx];
    *(int4*)&d[4] = *(const int4*)&gray[ly + 2][lx + 4];
    float v[4];
#pragma unroll
    for (int o = 0; o < 4; ++o)
      v[o] = (float)abs(u[o + 1] + m[o] - 4 * m[o + 1] + m[o + 2] + d[o + 1]);  // (= fabs((double)...): exact)
    *(float4*)&lap[ly][lx] = make_float4(v[0], v[1], v[2], v[3]);
  }
  __syncthreads();
  // (3) rows: s = k0*S[x-7] + k1*S[x-6] + ... (ca_gauss_rows' order); a thread
  // takes 4 consecutive outputs of a row from one 18-value window in registers
  // (15 LDS reads per output were the pass's limit)
  for (int sgi = t; sgi < CA_LH * (CA_TW / 4); sgi += CA_NT) {
    const int ly = sgi / (CA_TW / 4), x0 = (sgi % (CA_TW / 4)) * 4;
    float wf[20];
#pragma unroll
    for (int i = 0; i < 5; ++i) *(float4*)&wf[4 * i] = *(const float4*)&lap[ly][x0 + 4 * i];
    double w[18];
#pragma unroll
    for (int i = 0; i < 18; ++i) w[i] = (double)wf[i];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      double acc = g.k[0] * w[o];
#pragma unroll
      for (int k = 1; k < 15; ++k) acc += g.k[k] * w[o + k];
      rowg[ly][x0 + o] = acc;
    }
  }
  __syncthreads();
  // (4) columns: s = ky[7]*S[y] + 0.0; s += ky[7+k]*(S[y+k] + S[y-k]); a thread
  // takes 8 consecutive outputs of one column from a 22-value window
  static_assert(CA_NT / 64 * 8 == CA_TH, "one 8-row column window per thread");
  double mn = DBL_MAX, mx = -DBL_MAX;
  {
    const int col = t & 63, yb = (t >> 6) * 8;
    const int xx = tx0 + col;
    double w[22];
#pragma unroll
    for (int i = 0; i < 22; ++i) w[i] = rowg[yb + i][col];
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      const int y = ty0 + yb + o;
      // (SymmColumnFilter's "+ 0.0" is the identity here: every row value is a
      // sum of products of positive taps and |Laplacian| >= +0, never -0)
      double acc = g.k[7] * w[o + CA_R];
#pragma unroll
      for (int k = 1; k <= 7; ++k) acc += g.k[7 + k] * (w[o + CA_R + k] + w[o + CA_R - k]);
      if (y < H && xx < W) {
        sal[(size_t)b * HW + (size_t)y * W + xx] = acc;
        // (compare-selects: fmin / fmax add NaN canonicalisations at the fp64 rate)
        mn = acc < mn ? acc : mn;
        mx = acc > mx ? acc : mx;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double omn = __shfl_xor(mn, o, 64), omx = __shfl_xor(mx, o, 64);
    mn = omn < mn ? omn : mn;
    mx = omx > mx ? omx : mx;
  }
  constexpr int NW = CA_NT / 64;
  __shared__ double red[2][NW];
  if ((t & 63) == 0) { red[0][t >> 6] = mn; red[1][t >> 6] = mx; }
  __syncthreads();
  if (t == 0) {
    double a = red[0][0], z = red[1][0];
#pragma unroll
    for (int k = 1; k < NW; ++k) { a = red[0][k] < a ? red[0][k] : a; z = red[1][k] > z ? red[1][k] : z; }
    part[((size_t)b * nblk + blockIdx.x) * 2] = a;
    part[((size_t)b * nblk + blockIdx.x) * 2 + 1] = z;
  }
}

// the image's min / max from the producer's nblk per-block partial pairs:
// every consumer block reduces them itself (2-4 KiB from L2, read after the
// block's own loads went out) instead of a one-block-per-image reduce launch
// between the passes.  min / max are exact in any order.
template <typename F>
__device__ __forceinline__ void minmax_of_parts(const F* __restrict__ part, int nblk, F (&sh)[2], F& mn, F& mx) {
  if (threadIdx.x < 64) {
    F a = part[0], z = part[1];
    for (int i0 = threadIdx.x; i0 < nblk; i0 += 256) {
      F pa[4], pz[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + 64 * u < nblk ? i0 + 64 * u : 0;
        pa[u] = part[2 * i];
        pz[u] = part[2 * i + 1];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { a = a < pa[u] ? a : pa[u]; z = z > pz[u] ? z : pz[u]; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const F oa = __shfl_xor(a, o, 64), oz = __shfl_xor(z, o, 64);
      a = a < oa ? a : oa;
      z = z > oz ? z : oz;
    }
    if (threadIdx.x == 0) { sh[0] = a; sh[1] = z; }
  }
  // the barrier orders the LDS pair only: the block's HBM loads stay in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  mn = sh[0];
  mx = sh[1];
}

// ca_att_kernel over 4 pixels per thread (HW % 4 == 0): 16-byte loads / stores
template <typename T>
__global__ __launch_bounds__(256) void ca_att4_kernel(const T* __restrict__ x, const double* __restrict__ sal,
                                                      const double* __restrict__ spart, int nsal,
                                                      float* __restrict__ sal_out, float* __restrict__ att,
                                                      float* __restrict__ part, int HW4, int nblk) {
  __shared__ double smm[2];
  const int b = blockIdx.y;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  float mn = FLT_MAX, mx = -FLT_MAX;
  const size_t HW = (size_t)HW4 * 4, p = (size_t)(q < HW4 ? q : HW4 - 1) * 4;
  const double2 s01 = *(const double2*)(sal + b * HW + p), s23 = *(const double2*)(sal + b * HW + p + 2);
  const T* img = x + (size_t)b * 3 * HW;
  float r[4], gg[4], bb[4], so[4], a[4];
  ld4<T>(img + p, r);
  ld4<T>(img + HW + p, gg);
  ld4<T>(img + 2 * HW + p, bb);
  double smin, smax;
  minmax_of_parts<double>(spart + (size_t)b * nsal * 2, nsal, smm, smin, smax);
  if (q < HW4) {
    const double sv[4] = {s01.x, s01.y, s23.x, s23.y};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      so[k] = (float)((sv[k] - smin) / (smax - smin + 1e-8));
      const float lum = 0.299f * r[k] + 0.587f * gg[k] + 0.114f * bb[k];
      a[k] = so[k] * (1.0f / (lum + 0.1f));
      mn = fminf(mn, a[k]);
      mx = fmaxf(mx, a[k]);
    }
    if (sal_out) *(float4*)(sal_out + b * HW + p) = make_float4(so[0], so[1], so[2], so[3]);
    *(float4*)(att + b * HW + p) = make_float4(a[0], a[1], a[2], a[3]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  }
  __shared__ float red[2][4];
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = mn; red[1][threadIdx.x >> 6] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[((size_t)b * nblk + blockIdx.x) * 2] = fminf(fminf(red[0][0], red[0][1]), fminf(red[0][2], red[0][3]));
    part[((size_t)b * nblk + blockIdx.x) * 2 + 1] = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
  }
}

// ca_apply_kernel over 4 pixels per thread (HW % 4 == 0)
template <typename T>
__global__ __launch_bounds__(256) void ca_apply4_kernel(const float* __restrict__ att, const float* __restrict__ apart,
                                                        int natt, float* __restrict__ att_out,
                                                        const T* __restrict__ enh, T* __restrict__ out, int HW4) {
  __shared__ float amm[2];
  const int b = blockIdx.y;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const size_t HW = (size_t)HW4 * 4, p = (size_t)(q < HW4 ? q : HW4 - 1) * 4;
  const float4 av = *(const float4*)(att + b * HW + p);
  float mn, mx;
  minmax_of_parts<float>(apart + (size_t)b * natt * 2, natt, amm, mn, mx);
  if (q >= HW4) return;
  const float a[4] = {(av.x - mn) / (mx - mn + 1e-8f), (av.y - mn) / (mx - mn + 1e-8f), (av.z - mn) / (mx - mn + 1e-8f),
                      (av.w - mn) / (mx - mn + 1e-8f)};
  if (att_out) *(float4*)(att_out + b * HW + p) = make_float4(a[0], a[1], a[2], a[3]);
  if (enh && out) {
    float f[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) f[k] = 1.0f + 0.2f * a[k];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t o = ((size_t)b * 3 + c) * HW + p;
      float v[4];
      ld4<T>(enh + o, v);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = fminf(fmaxf(v[k] * f[k], 0.f), 1.f);
      if constexpr (sizeof(T) == 4) {
        *(float4*)((float*)out + o) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        *(h4*)((half_t*)out + o) = h4{(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
      }
    }
  }
}

template <typename F>
__global__ void reduce_minmax(const F* __restrict__ part, F* __restrict__ res, int nblk) {
  const int b = blockIdx.x;
  __shared__ F smn[256], smx[256];
  F mn = part[(size_t)b * nblk * 2], mx = part[(size_t)b * nblk * 2 + 1];
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) {
    mn = part[((size_t)b * nblk + i) * 2] < mn ? part[((size_t)b * nblk + i) * 2] : mn;
    mx = part[((size_t)b * nblk + i) * 2 + 1] > mx ? part[((size_t)b * nblk + i) * 2 + 1] : mx;
  }
  smn[threadIdx.x] = mn;
  smx[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      if (smn[threadIdx.x + s] < smn[threadIdx.x]) smn[threadIdx.x] = smn[threadIdx.x + s];
      if (smx[threadIdx.x + s] > smx[threadIdx.x]) smx[threadIdx.x] = smx[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) { res[2 * b] = smn[0]; res[2 * b + 1] = smx[0]; }
}

// saliency (normalised, fp32) and raw attention + per-block fp32 min/max
template <typename T>
__global__ __launch_bounds__(256) void ca_att_kernel(const T* __restrict__ x, const double* __restrict__ sal,
                                                     const double* __restrict__ mm, float* __restrict__ sal_out,
                                                     float* __restrict__ att, float* __restrict__ part, int H, int W,
                                                     int nblk) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  float mn = FLT_MAX, mx = -FLT_MAX;
  if (p < H * W) {
    const size_t HW = (size_t)H * W;
    const double smin = mm[2 * b], smax = mm[2 * b + 1];
    const float s = (float)((sal[(size_t)b * HW + p] - smin) / (smax - smin + 1e-8));
    if (sal_out) sal_out[(size_t)b * HW + p] = s;
    const T* img = x + (size_t)b * 3 * HW;
    const float lum = 0.299f * ldf(img, p) + 0.587f * ldf(img, HW + p) + 0.114f * ldf(img, 2 * HW + p);
    const float a = s * (1.0f / (lum + 0.1f));
    att[(size_t)b * HW + p] = a;
    mn = mx = a;
  }
  __shared__ float smn[256], smx[256];
  smn[threadIdx.x] = mn;
  smx[threadIdx.x] = mx;
  __syncthreads();
  for (int s2 = 128; s2 > 0; s2 >>= 1) {
    if (threadIdx.x < s2) {
      smn[threadIdx.x] = fminf(smn[threadIdx.x], smn[threadIdx.x + s2]);
      smx[threadIdx.x] = fmaxf(smx[threadIdx.x], smx[threadIdx.x + s2]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[((size_t)b * nblk + blockIdx.x) * 2] = smn[0];
    part[((size_t)b * nblk + blockIdx.x) * 2 + 1] = smx[0];
  }
}

// attention normalisation (+ optional enhancement)
template <typename T>
__global__ __launch_bounds__(256) void ca_apply_kernel(const float* __restrict__ att, const float* __restrict__ mm,
                                                       float* __restrict__ att_out, const T* __restrict__ enh,
                                                       T* __restrict__ out, int B, int HW) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)B * HW) return;
  const int b = (int)(idx / HW);
  const size_t p = idx - (size_t)b * HW;
  const float mn = mm[2 * b], mx = mm[2 * b + 1];
  const float a = (att[idx] - mn) / (mx - mn + 1e-8f);
  if (att_out) att_out[idx] = a;
  if (enh && out) {
    const float f = 1.0f + 0.2f * a;
    for (int c = 0; c < 3; ++c) {
      const size_t o = ((size_t)b * 3 + c) * HW + p;
      stf(out, o, fminf(fmaxf(ldf(enh, o) * f, 0.f), 1.f));
    }
  }
}

static inline int gd(size_t n) { return (int)((n + 255) / 256); }

static inline int ca_tiles(int H, int W) { return ((W + CA_TW - 1) / CA_TW) * ((H + CA_TH - 1) / CA_TH); }

size_t content_aware_ws(int B, int H, int W) {
  const size_t HW = (size_t)H * W;
  const size_t nblk = (HW + 255) / 256;
  // + the fused form's two partial arrays, side by side (its passes read one
  // while the next writes the other)
  const size_t nb4 = (HW / 4 + 255) / 256;
  return align_up(2 * (size_t)B * HW * 8, 256) + align_up((size_t)B * HW * 4, 256) +
         align_up((size_t)B * nblk * 2 * 8, 256) + align_up((size_t)B * 2 * 8, 256) + align_up((size_t)B * 2 * 4, 256) +
         align_up((size_t)B * ca_tiles(H, W) * 2 * 8, 256) + align_up((size_t)B * nb4 * 2 * 4, 256);
}

int launch_content_aware(const void* x, const void* enh, void* out, float* sal_out, float* att_out, uint8_t* ws,
                         int B, int H, int W, int dtype, hipStream_t st) {
  const size_t HW = (size_t)H * W;
  const int nblk = (int)((HW + 255) / 256);
  double* lap = (double*)ws;
  double* tmp = lap + (size_t)B * HW;
  uint8_t* p = ws + align_up(2 * (size_t)B * HW * 8, 256);
  float* att = (float*)p;
  p += align_up((size_t)B * HW * 4, 256);
  double* part64 = (double*)p;
  float* part32 = (float*)p;
  p += align_up((size_t)B * nblk * 2 * 8, 256);
  double* mm64 = (double*)p;
  p += align_up((size_t)B * 2 * 8, 256);
  float* mm32 = (float*)p;
  p += align_up((size_t)B * 2 * 4, 256);
  double* fpart64 = (double*)p;  // the fused form's partials
  p += align_up((size_t)B * ca_tiles(H, W) * 2 * 8, 256);
  float* fpart32 = (float*)p;
  // Gaussian kernel: getGaussianKernel(15, 0 -> 2.6, CV_64F)
  GaussK g;
  const double sigma = ((15 - 1) * 0.5 - 1) * 0.3 + 0.8;
  const double scale2X = -0.5 / (sigma * sigma);
  double sum = 0.0;
  for (int i = 0; i < 15; ++i) {
    const double xx = i - (15 - 1) * 0.5;
    g.k[i] = std::exp(scale2X * xx * xx);
    sum += g.k[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 15; ++i) g.k[i] *= sum;
  const size_t n = (size_t)B * HW;
  // UPR_CA_FUSED=0: the three-kernel saliency form and the scalar passes (A/B)
  static const bool fused = [] { const char* e = getenv("UPR_CA_FUSED"); return !e || atoi(e) != 0; }();
  if (fused && HW % 4 == 0) {
    // one fused saliency pass (tiles of 64 x 64) + the 4-pixel attention / apply
    // passes, each consumer reducing its producer's per-block min / max itself
    const int tiles_x = (W + CA_TW - 1) / CA_TW, tiles = ca_tiles(H, W);
    const int HW4 = (int)(HW / 4), nb4 = (HW4 + 255) / 256;
    if (dtype == kF16)
      hipLaunchKernelGGL((ca_sal_fused_kernel<half_t>), dim3(tiles, B), dim3(CA_NT), 0, st, (const half_t*)x, lap, H, W,
                         tiles_x, g, fpart64, tiles);
    else
      hipLaunchKernelGGL((ca_sal_fused_kernel<float>), dim3(tiles, B), dim3(CA_NT), 0, st, (const float*)x, lap, H, W,
                         tiles_x, g, fpart64, tiles);
    if (dtype == kF16)
      hipLaunchKernelGGL((ca_att4_kernel<half_t>), dim3(nb4, B), dim3(256), 0, st, (const half_t*)x, lap,
                         (const double*)fpart64, tiles, sal_out, att, fpart32, HW4, nb4);
    else
      hipLaunchKernelGGL((ca_att4_kernel<float>), dim3(nb4, B), dim3(256), 0, st, (const float*)x, lap,
                         (const double*)fpart64, tiles, sal_out, att, fpart32, HW4, nb4);
    if (dtype == kF16)
      hipLaunchKernelGGL((ca_apply4_kernel<half_t>), dim3(nb4, B), dim3(256), 0, st, att, (const float*)fpart32, nb4,
                         att_out, (const half_t*)enh, (half_t*)out, HW4);
    else
      hipLaunchKernelGGL((ca_apply4_kernel<float>), dim3(nb4, B), dim3(256), 0, st, att, (const float*)fpart32, nb4,
                         att_out, (const float*)enh, (float*)out, HW4);
    return (int)hipGetLastError();
  }
  if (dtype == kF16)
    hipLaunchKernelGGL((ca_lap_kernel<half_t>), dim3(gd(n)), dim3(256), 0, st, (const half_t*)x, lap, B, H, W);
  else
    hipLaunchKernelGGL((ca_lap_kernel<float>), dim3(gd(n)), dim3(256), 0, st, (const float*)x, lap, B, H, W);
  hipLaunchKernelGGL(ca_gauss_rows, dim3(gd(n)), dim3(256), 0, st, lap, tmp, B, H, W, g);
  hipLaunchKernelGGL(ca_gauss_cols, dim3(nblk, B), dim3(256), 0, st, tmp, lap, H, W, g, part64, nblk);
  hipLaunchKernelGGL((reduce_minmax<double>), dim3(B), dim3(256), 0, st, part64, mm64, nblk);
  if (dtype == kF16)
    hipLaunchKernelGGL((ca_att_kernel<half_t>), dim3(nblk, B), dim3(256), 0, st, (const half_t*)x, lap, mm64, sal_out,
                       att, part32, H, W, nblk);
  else
    hipLaunchKernelGGL((ca_att_kernel<float>), dim3(nblk, B), dim3(256), 0, st, (const float*)x, lap, mm64, sal_out,
                       att, part32, H, W, nblk);
  hipLaunchKernelGGL((reduce_minmax<float>), dim3(B), dim3(256), 0, st, part32, mm32, nblk);
  if (dtype == kF16)
    hipLaunchKernelGGL((ca_apply_kernel<half_t>), dim3(gd(n)), dim3(256), 0, st, att, mm32, att_out,
                       (const half_t*)enh, (half_t*)out, B, (int)HW);
  else
    hipLaunchKernelGGL((ca_apply_kernel<float>), dim3(gd(n)), dim3(256), 0, st, att, mm32, att_out,
                       (const float*)enh, (float*)out, B, (int)HW);
  return (int)hipGetLastError();
}

}  // namespace upr
