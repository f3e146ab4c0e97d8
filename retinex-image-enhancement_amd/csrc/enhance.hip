// Enhancer kernels (gfx950): integer/histogram work, HBM/latency-bound.
//
//  clahe_hist     float -> u8 cast exactly as numpy's astype(uint8) on x*255
//                 (trunc, wrap mod 256; NaN/|v|>=2^31 -> 0), 8-bit sRGB -> Lab
//                 (enhancers/adaptive_params.py:142,145), per-wave tile histograms
//  clahe_lut      clip + redistribute, CDF -> LUT
//                 (cv2.createCLAHE(2.0,(8,8)).apply, adaptive_params.py:149-152)
//  clahe_apply    bilinear LUT blend of L, Lab -> sRGB 8-bit, /255 back to float
//                 (adaptive_params.py:155-167)
//  gray_hist      8-bit BGR2GRAY histogram (calculate_brightness_features :45-66)
//  ms_sums        multi-scale feature sums (enhancers/multi_scale.py:17-60, :87-94)
//  scale_clamp    clamp(enh * factor[b], 0, 1)  (multi_scale.py:97-98)
#include <utility>

#include "upr_common.h"
#include "lab_tables.h"

#include <mutex>

namespace upr {

struct DevLab {
  uint16_t gamma_b[256];
  uint16_t cbrt_b[3072];
  uint16_t yf_b[512];
  uint16_t invgamma_b[4096];
  int32_t rgb2xyz[9];
  int32_t xyz2rgb[9];
};

// One table copy per device, uploaded on first use (one process per GPU, but
// be correct for several devices in one process too).
static const DevLab* dev_lab_tables(hipStream_t st) {
  static DevLab* ptrs[64] = {nullptr};
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (!ptrs[dev]) {
    const LabTables& t = lab_tables();
    DevLab h;
    for (int i = 0; i < 256; ++i) h.gamma_b[i] = t.gamma_b[i];
    for (int i = 0; i < 3072; ++i) h.cbrt_b[i] = t.cbrt_b[i];
    for (int i = 0; i < 512; ++i) h.yf_b[i] = t.yf_b[i];
    for (int i = 0; i < 4096; ++i) h.invgamma_b[i] = t.invgamma_b[i];
    for (int i = 0; i < 9; ++i) { h.rgb2xyz[i] = t.rgb2xyz[i]; h.xyz2rgb[i] = t.xyz2rgb[i]; }
    DevLab* d = nullptr;
    if (hipMalloc(&d, sizeof(DevLab)) != hipSuccess) return nullptr;
    if (hipMemcpy(d, &h, sizeof(DevLab), hipMemcpyHostToDevice) != hipSuccess) { (void)hipFree(d); return nullptr; }
    ptrs[dev] = d;
  }
  (void)st;
  return ptrs[dev];
}

__device__ __forceinline__ float ldf(const float* p, size_t i) { return p[i]; }
__device__ __forceinline__ float ldf(const half_t* p, size_t i) { return (float)p[i]; }
__device__ __forceinline__ void stf(float* p, size_t i, float v) { p[i] = v; }
__device__ __forceinline__ void stf(half_t* p, size_t i, float v) { p[i] = (half_t)v; }

// numpy: (np.float32 x * 255).astype(np.uint8) on x86-64
__device__ __forceinline__ int quant_u8(float v) {
  const float t = __fmul_rn(v, 255.f);
  if (!(fabsf(t) < 2147483648.f)) return 0;  // NaN, inf, out of int32 range
  return ((int)t) & 255;                      // trunc toward zero, wrap
}

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }
__device__ __forceinline__ int sat_u8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// RGB2Lab_b::operator() (8-bit, sRGB)
__device__ __forceinline__ void rgb2lab_u8(const DevLab* T, int R8, int G8, int B8, int& L, int& A, int& Bb) {
  const int R = T->gamma_b[R8], G = T->gamma_b[G8], B = T->gamma_b[B8];
  const int* c = T->rgb2xyz;
  const int fX = T->cbrt_b[descale(R * c[0] + G * c[1] + B * c[2], 12)];
  const int fY = T->cbrt_b[descale(R * c[3] + G * c[4] + B * c[5], 12)];
  const int fZ = T->cbrt_b[descale(R * c[6] + G * c[7] + B * c[8], 12)];
  const int Lscale = (116 * 255 + 50) / 100;
  const int Lshift = -((16 * 255 * (1 << 15) + 50) / 100);
  L = sat_u8(descale(Lscale * fY + Lshift, 15));
  A = sat_u8(descale(500 * (fX - fY) + 128 * (1 << 15), 15));
  Bb = sat_u8(descale(200 * (fY - fZ) + 128 * (1 << 15), 15));
}

// Lab2RGBinteger::process (8-bit, sRGB)
__device__ __forceinline__ void lab2rgb_u8(const DevLab* T, int L, int A, int Bb, int& R, int& G, int& B) {
  const int BASE = 1 << 14;
  const int y = T->yf_b[L * 2], ify = T->yf_b[L * 2 + 1];
  const int adiv = ((5 * A * 53687 + (1 << 7)) >> 13) - 128 * BASE / 500;
  const int bdiv = ((Bb * 41943 + (1 << 4)) >> 9) - 128 * BASE / 200 + 1;
  const int x = ab_to_xz(ify + adiv);
  const int z = ab_to_xz(ify - bdiv);
  const int* c = T->xyz2rgb;
  int r = descale(c[0] * x + c[1] * y + c[2] * z, 14);
  int g = descale(c[3] * x + c[4] * y + c[5] * z, 14);
  int b = descale(c[6] * x + c[7] * y + c[8] * z, 14);
  r = max(0, min(4095, r)); g = max(0, min(4095, g)); b = max(0, min(4095, b));
  R = T->invgamma_b[r]; G = T->invgamma_b[g]; B = T->invgamma_b[b];
}

// quantise only: NCHW float -> NCHW u8
template <typename T>
__global__ __launch_bounds__(256) void quant_kernel(const T* __restrict__ x, uint8_t* __restrict__ out, size_t n) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < n) out[idx] = (uint8_t)quant_u8(ldf(x, idx));
}

// ---------------------------------------------------------------------------
// CLAHE (cv2.createCLAHE(clip, (tilesX, tilesY)).apply; OpenCV
// imgproc/src/clahe.cpp CLAHE_CalcLut_Body / CLAHE_Interpolation_Body), on the
// L plane of the 8-bit Lab image (adaptive_params.py:142-161) or on a u8 plane.
// The tiles cover the image extended by BORDER_REFLECT_101 to a multiple of
// the tile grid (at most tiles - 1 extra rows / columns: one reflection).
//
//   clahe_hist   one block per (image, tile, row band s of S): quantise + 8-bit
//                Lab of the band's pixels (SRC 0) or the u8 plane (SRC 1); the L
//                / A / B planes are written (SRC 0); every wave counts into its
//                own 256-bin LDS histogram, the 4 copies are summed per bin ->
//                the band's partial histogram (S > 1) or, S == 1, the tile's
//                LUT in the same block
//   clahe_lut    (S > 1) the S partials of a tile summed per bin -> LUT
//   clahe_apply  one block per (image, band of R3 <= tileH rows): the LUT rows
//                the band reads (<= 3 tile rows) and the Lab tables staged in
//                LDS, bilinear LUT blend, Lab -> sRGB 8-bit, /255 (DST 0) or
//                the u8 plane (DST 1)
// Threads walk their (row, column group) items with constant increments: no
// per-pixel division, no reflect loop; V = 4 pixels per item when the rows
// are whole groups of 4 and the tiles too (vector loads / stores).
// ---------------------------------------------------------------------------
struct ClaheArgs {
  int H, W, tilesX, tilesY, tileW, tileH;
  int S, R;      // hist: row bands per tile, rows per band (tileH = S * R)
  int R3;        // apply: rows per block (<= tileH)
  int clip;      // clip limit in counts (0: none)
  float lutScale;
};

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// clip + redistribute + inclusive CDF -> LUT byte of bin t (256 threads, one bin each)
__device__ __forceinline__ uint8_t clahe_lut_bin(int h, int t, int clip, float lutScale, int* red) {
  const int lane = t & 63, w = t >> 6;
  if (clip > 0) {
    const int ex = wave_sum_i(h > clip ? h - clip : 0);
    h = h > clip ? clip : h;
    if (lane == 0) red[w] = ex;
    __syncthreads();
    const int clipped = red[0] + red[1] + red[2] + red[3];
    const int redistBatch = clipped / 256;
    const int residual = clipped - redistBatch * 256;
    h += redistBatch;
    if (residual != 0) {
      // bins 0, step, 2 step, ... take one each until residual runs out
      const int step = max(256 / residual, 1);
      if (t % step == 0 && t / step < residual) h += 1;
    }
    __syncthreads();
  }
  // inclusive scan: within the wave, then the preceding waves' totals
  int c = h;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(c, o, 64);
    if (lane >= o) c += u;
  }
  if (lane == 63) red[4 + w] = c;
  __syncthreads();
  for (int k = 0; k < w; ++k) c += red[4 + k];
  const int r = __float2int_rn(__fmul_rn((float)c, lutScale));  // saturate_cast<uchar>(float)
  return (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
}

template <typename T>
struct Vec4 {};
template <>
struct Vec4<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[4]) {
    const float4 q = *(const float4*)p;
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[4]) {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <>
struct Vec4<half_t> {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ void load(const half_t* p, float (&v)[4]) {
    const h4 q = *(const h4*)p;
    v[0] = (float)q[0]; v[1] = (float)q[1]; v[2] = (float)q[2]; v[3] = (float)q[3];
  }
  static __device__ __forceinline__ void store(half_t* p, const float (&v)[4]) {
    h4 q;
    q[0] = (half_t)v[0]; q[1] = (half_t)v[1]; q[2] = (half_t)v[2]; q[3] = (half_t)v[3];
    *(h4*)p = q;
  }
};

// RGB2Lab_b on LDS copies of the gamma / cube-root tables
__device__ __forceinline__ void rgb2lab_lds(const uint16_t* gam, const uint16_t* cbrt, const int* c, int R8, int G8,
                                            int B8, int& L, int& A, int& Bb) {
  const int R = gam[R8], G = gam[G8], B = gam[B8];
  const int fX = cbrt[descale(R * c[0] + G * c[1] + B * c[2], 12)];
  const int fY = cbrt[descale(R * c[3] + G * c[4] + B * c[5], 12)];
  const int fZ = cbrt[descale(R * c[6] + G * c[7] + B * c[8], 12)];
  const int Lscale = (116 * 255 + 50) / 100;
  const int Lshift = -((16 * 255 * (1 << 15) + 50) / 100);
  L = sat_u8(descale(Lscale * fY + Lshift, 15));
  A = sat_u8(descale(500 * (fX - fY) + 128 * (1 << 15), 15));
  Bb = sat_u8(descale(200 * (fY - fZ) + 128 * (1 << 15), 15));
}

// Lab2RGBinteger on LDS copies of the Y / inverse-gamma tables; igf holds the
// inverse-gamma byte already divided by 255 (__fdiv_rn(ig, 255): the output's
// /255, one lookup instead of two), yf2 the (y, ify) pair of L as one word
__device__ __forceinline__ int ab_to_xz_dev(int v) {
  // lab_tables.h ab_to_xz: the cube branch has v > 3390 > 0, so its signed
  // divisions by 2^14 are shifts (unsigned: no sign fix-ups)
  const int BASE = 1 << 14;
  if (v <= 3390) return v * 108 / 841 - BASE * 16 / 116 * 108 / 841;
  const unsigned u = (unsigned)v;
  return (int)((((u * u) >> 14) * u) >> 14);
}

__device__ __forceinline__ void lab2rgb_lds(const uint32_t* yf2, const float* igf, const int* c, int L, int A, int Bb,
                                            float& R, float& G, float& B) {
  const int BASE = 1 << 14;
  const uint32_t yw = yf2[L];
  const int y = (int)(yw & 0xffffu), ify = (int)(yw >> 16);
  const int adiv = ((5 * A * 53687 + (1 << 7)) >> 13) - 128 * BASE / 500;
  const int bdiv = ((Bb * 41943 + (1 << 4)) >> 9) - 128 * BASE / 200 + 1;
  const int x = ab_to_xz_dev(ify + adiv);
  const int z = ab_to_xz_dev(ify - bdiv);
  int r = descale(c[0] * x + c[1] * y + c[2] * z, 14);
  int g = descale(c[3] * x + c[4] * y + c[5] * z, 14);
  int b = descale(c[6] * x + c[7] * y + c[8] * z, 14);
  r = max(0, min(4095, r)); g = max(0, min(4095, g)); b = max(0, min(4095, b));
  R = igf[r]; G = igf[g]; B = igf[b];
}

// SRC 0: T RGB planes [B,3,H,W] -> L / A / B planes; SRC 1: u8 plane [B,H,W] (src = L)
template <int SRC, typename T, int V>
__global__ __launch_bounds__(256) void clahe_hist_kernel(const void* __restrict__ src, uint8_t* __restrict__ Lp,
                                                         uint8_t* __restrict__ Ap, uint8_t* __restrict__ Bp,
                                                         int* __restrict__ part, uint8_t* __restrict__ lut,
                                                         const DevLab* __restrict__ tab, ClaheArgs g) {
  __shared__ int hist[4][256];
  __shared__ uint16_t gam[SRC == 0 ? 256 : 1];
  __shared__ uint16_t cbrt[SRC == 0 ? 3072 : 1];
  __shared__ int red[8];
  const int t = threadIdx.x, wave = t >> 6;
  const int b = blockIdx.y;
  const int s = blockIdx.x % g.S, tile = blockIdx.x / g.S;  // block-uniform
  const int tx = tile % g.tilesX, ty = tile / g.tilesX;
#pragma unroll
  for (int k = 0; k < 4; ++k) hist[k][t] = 0;
  int c[9];
  if constexpr (SRC == 0) {
    for (int i = t; i < 256; i += 256) gam[i] = tab->gamma_b[i];
    for (int i = t; i < 3072; i += 256) cbrt[i] = tab->cbrt_b[i];
#pragma unroll
    for (int k = 0; k < 9; ++k) c[k] = tab->rgb2xyz[k];
  }
  __syncthreads();
  const int H = g.H, W = g.W;
  const size_t HW = (size_t)H * W;
  const int y0 = ty * g.tileH + s * g.R, x0 = tx * g.tileW;
  const int TWV = g.tileW / V;
  // item cursor (row, column group), advanced by 256 items per iteration
  int row = t / TWV, col = t - (t / TWV) * TWV;
  const int inc_r = 256 / TWV, inc_c = 256 - inc_r * TWV;
  int* hw = hist[wave];
  // (issuing 4 iterations' loads together measured slower twice: 27.5 -> 36.0 us,
  // profiles/r5_enh_kernels_ab.txt -- occupancy halves, the LDS atomics are the limit)
  for (; row < g.R; row += inc_r) {
    const int y = y0 + row;
    const int yr = y < H ? y : 2 * H - 2 - y;  // BORDER_REFLECT_101 (one reflection)
    const int x = x0 + col * V;
    if constexpr (V == 4) {
      // whole groups inside the image (no column padding on this path)
      const size_t o = (size_t)b * (SRC == 0 ? 3 : 1) * HW + (size_t)yr * W + x;
      int Lv[4];
      if constexpr (SRC == 0) {
        const T* img = (const T*)src;
        float r[4], gg[4], bl[4];
        Vec4<T>::load(img + o, r);
        Vec4<T>::load(img + o + HW, gg);
        Vec4<T>::load(img + o + 2 * HW, bl);
        int Av[4], Bv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) rgb2lab_lds(gam, cbrt, c, quant_u8(r[k]), quant_u8(gg[k]), quant_u8(bl[k]), Lv[k],
                                                 Av[k], Bv[k]);
        if (y < H) {
          const size_t q = (size_t)b * HW + (size_t)y * W + x;
          *(uchar4*)(Lp + q) = make_uchar4(Lv[0], Lv[1], Lv[2], Lv[3]);
          *(uchar4*)(Ap + q) = make_uchar4(Av[0], Av[1], Av[2], Av[3]);
          *(uchar4*)(Bp + q) = make_uchar4(Bv[0], Bv[1], Bv[2], Bv[3]);
        }
      } else {
        const uchar4 q = *(const uchar4*)((const uint8_t*)src + o);
        Lv[0] = q.x; Lv[1] = q.y; Lv[2] = q.z; Lv[3] = q.w;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) atomicAdd(&hw[Lv[k]], 1);
    } else {
      const int xr = x < W ? x : 2 * W - 2 - x;
      const size_t o = (size_t)b * (SRC == 0 ? 3 : 1) * HW + (size_t)yr * W + xr;
      int Lv;
      if constexpr (SRC == 0) {
        const T* img = (const T*)src;
        int Av, Bv;
        rgb2lab_lds(gam, cbrt, c, quant_u8(ldf(img, o)), quant_u8(ldf(img, o + HW)), quant_u8(ldf(img, o + 2 * HW)),
                    Lv, Av, Bv);
        if (y < H && x < W) {
          const size_t q = (size_t)b * HW + (size_t)y * W + x;
          Lp[q] = (uint8_t)Lv; Ap[q] = (uint8_t)Av; Bp[q] = (uint8_t)Bv;
        }
      } else {
        Lv = ((const uint8_t*)src)[o];
      }
      atomicAdd(&hw[Lv], 1);
    }
    col += inc_c;
    if (col >= TWV) { col -= TWV; ++row; }
  }
  __syncthreads();
  // (16 sub-histograms, 4 per wave by lane % 4 on padded rows, measured
  // slower: 27.1 -> 30.4 us, profiles/r5_ms_sums3_v2.txt)
  const int h = hist[0][t] + hist[1][t] + hist[2][t] + hist[3][t];
  const size_t tb = (size_t)b * g.tilesX * g.tilesY + tile;
  if (g.S > 1) {
    part[(tb * g.S + s) * 256 + t] = h;
    return;
  }
  lut[tb * 256 + t] = clahe_lut_bin(h, t, g.clip, g.lutScale, red);
}

// S > 1: one block per (image, tile)
__global__ __launch_bounds__(256) void clahe_lut_kernel(const int* __restrict__ part, uint8_t* __restrict__ lut,
                                                        ClaheArgs g) {
  __shared__ int red[8];
  const int t = threadIdx.x;
  const size_t tb = (size_t)blockIdx.y * g.tilesX * g.tilesY + blockIdx.x;
  int h = 0;
  for (int s = 0; s < g.S; ++s) h += part[(tb * g.S + s) * 256 + t];
  lut[tb * 256 + t] = clahe_lut_bin(h, t, g.clip, g.lutScale, red);
}

// DST 0: L / A / B planes -> T RGB planes (/255); DST 1: u8 plane (Lp) -> u8 plane (out)
template <int DST, typename T, int V>
__global__ __launch_bounds__(256) void clahe_apply_kernel(const uint8_t* __restrict__ Lp, const uint8_t* __restrict__ Ap,
                                                          const uint8_t* __restrict__ Bp, const uint8_t* __restrict__ lut,
                                                          const DevLab* __restrict__ tab, void* __restrict__ out,
                                                          ClaheArgs g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  float* igf = (float*)sm;                  // 4096: __fdiv_rn(invgamma_b[i], 255)
  uint32_t* yf2 = (uint32_t*)(igf + 4096);  // 256: (y, ify) of L
  uint8_t* lrows = (uint8_t*)(yf2 + 256);   // <= 3 tile rows of LUTs
  const int t = threadIdx.x;
  const int b = blockIdx.y;
  const int H = g.H, W = g.W;
  const size_t HW = (size_t)H * W;
  const int y0 = blockIdx.x * g.R3;
  const int nrows = min(g.R3, H - y0);
  const float inv_tw = __fdiv_rn(1.0f, (float)g.tileW);
  const float inv_th = __fdiv_rn(1.0f, (float)g.tileH);
  // tile rows the band reads: ty1 of its first row .. ty2 of its last row
  const int ty_lo = max((int)floorf(__fsub_rn(__fmul_rn((float)y0, inv_th), 0.5f)), 0);
  const int ty_hi = min((int)floorf(__fsub_rn(__fmul_rn((float)(y0 + nrows - 1), inv_th), 0.5f)) + 1, g.tilesY - 1);
  const int lbytes = (ty_hi - ty_lo + 1) * g.tilesX * 256;
  const uint8_t* lsrc = lut + ((size_t)b * g.tilesY + ty_lo) * g.tilesX * 256;
  for (int i = t * 16; i < lbytes; i += 256 * 16) *(uint4*)(lrows + i) = *(const uint4*)(lsrc + i);
  int c[9];
  if constexpr (DST == 0) {
    yf2[t] = (uint32_t)tab->yf_b[2 * t] | (uint32_t)tab->yf_b[2 * t + 1] << 16;
    for (int i = t; i < 4096; i += 256) igf[i] = __fdiv_rn((float)tab->invgamma_b[i], 255.f);
#pragma unroll
    for (int k = 0; k < 9; ++k) c[k] = tab->xyz2rgb[k];
  }
  __syncthreads();
  const int WV = W / V;
  int row = t / WV, col = t - (t / WV) * WV;
  const int inc_r = 256 / WV, inc_c = 256 - inc_r * WV;
  // per-column interpolation terms of this thread's V pixels: computed once
  // when every iteration keeps the column (inc_c == 0: W / V divides 256)
  int cx1[V], cx2[V];
  float cxa[V], cxa1[V];
  auto colterms = [&](int cl) {
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const int x = cl * V + k;
      const float txf = __fsub_rn(__fmul_rn((float)x, inv_tw), 0.5f);
      const int tx1 = (int)floorf(txf);
      cxa[k] = __fsub_rn(txf, (float)tx1);
      cxa1[k] = __fsub_rn(1.0f, cxa[k]);
      cx1[k] = max(tx1, 0) * 256;
      cx2[k] = min(tx1 + 1, g.tilesX - 1) * 256;
    }
  };
  if (inc_c == 0) colterms(col);
  for (; row < nrows; row += inc_r) {
    if (inc_c != 0) colterms(col);
    const int y = y0 + row;
    const float tyf = __fsub_rn(__fmul_rn((float)y, inv_th), 0.5f);
    int ty1 = (int)floorf(tyf);
    int ty2 = ty1 + 1;
    const float ya = __fsub_rn(tyf, (float)ty1), ya1 = __fsub_rn(1.0f, ya);
    ty1 = max(ty1, 0) - ty_lo;
    ty2 = min(ty2, g.tilesY - 1) - ty_lo;
    const uint8_t* r1 = lrows + ty1 * g.tilesX * 256;
    const uint8_t* r2 = lrows + ty2 * g.tilesX * 256;
    const size_t q = (size_t)b * HW + (size_t)y * W + col * V;
    int Lv[V], Av[V], Bv[V];
    if constexpr (V == 4) {
      const uchar4 l4 = *(const uchar4*)(Lp + q);
      Lv[0] = l4.x; Lv[1] = l4.y; Lv[2] = l4.z; Lv[3] = l4.w;
      if constexpr (DST == 0) {
        const uchar4 a4 = *(const uchar4*)(Ap + q), b4 = *(const uchar4*)(Bp + q);
        Av[0] = a4.x; Av[1] = a4.y; Av[2] = a4.z; Av[3] = a4.w;
        Bv[0] = b4.x; Bv[1] = b4.y; Bv[2] = b4.z; Bv[3] = b4.w;
      }
    } else {
      Lv[0] = Lp[q];
      if constexpr (DST == 0) { Av[0] = Ap[q]; Bv[0] = Bp[q]; }
    }
    int lc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float xa = cxa[k], xa1 = cxa1[k];
      const int v = Lv[k];
      const float l11 = r1[cx1[k] + v], l12 = r1[cx2[k] + v];
      const float l21 = r2[cx1[k] + v], l22 = r2[cx2[k] + v];
      // res = (l11*xa1 + l12*xa)*ya1 + (l21*xa1 + l22*xa)*ya, no contraction
      const float top = __fadd_rn(__fmul_rn(l11, xa1), __fmul_rn(l12, xa));
      const float bot = __fadd_rn(__fmul_rn(l21, xa1), __fmul_rn(l22, xa));
      const int r = __float2int_rn(__fadd_rn(__fmul_rn(top, ya1), __fmul_rn(bot, ya)));
      lc[k] = r < 0 ? 0 : (r > 255 ? 255 : r);
    }
    if constexpr (DST == 1) {
      uint8_t* o = (uint8_t*)out + q;
      if constexpr (V == 4) *(uchar4*)o = make_uchar4(lc[0], lc[1], lc[2], lc[3]);
      else o[0] = (uint8_t)lc[0];
    } else {
      float R[V], G[V], Bo[V];
#pragma unroll
      for (int k = 0; k < V; ++k) lab2rgb_lds(yf2, igf, c, lc[k], Av[k], Bv[k], R[k], G[k], Bo[k]);
      T* o = (T*)out + (size_t)b * 3 * HW + (size_t)y * W + col * V;
      if constexpr (V == 4) {
        Vec4<T>::store(o, R);
        Vec4<T>::store(o + HW, G);
        Vec4<T>::store(o + 2 * HW, Bo);
      } else {
        stf(o, 0, R[0]);
        stf(o, HW, G[0]);
        stf(o, 2 * HW, Bo[0]);
      }
    }
    col += inc_c;
    if (col >= WV) { col -= WV; ++row; }
  }
}

// Lab <-> RGB standalone kernels (u8 HWC RGB <-> u8 HWC Lab), for API/tests
__global__ void rgb2lab_kernel(const uint8_t* __restrict__ rgb, uint8_t* __restrict__ lab, const DevLab* tab, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int l, a, b;
  rgb2lab_u8(tab, rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2], l, a, b);
  lab[3 * i] = l; lab[3 * i + 1] = a; lab[3 * i + 2] = b;
}
__global__ void lab2rgb_kernel(const uint8_t* __restrict__ lab, uint8_t* __restrict__ rgb, const DevLab* tab, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int r, g, b;
  lab2rgb_u8(tab, lab[3 * i], lab[3 * i + 1], lab[3 * i + 2], r, g, b);
  rgb[3 * i] = r; rgb[3 * i + 1] = g; rgb[3 * i + 2] = b;
}

// ---------------------------------------------------------------------------
// gray histogram: cv2 BGR2GRAY 8-bit = (B*1868 + G*9617 + R*4899 + 2^13) >> 14
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void gray_hist_kernel(const T* __restrict__ img, int* __restrict__ hist, int HW) {
  __shared__ int h[256];
  const int b = blockIdx.y;
  h[threadIdx.x] = 0;
  __syncthreads();
  const T* base = img + (size_t)b * 3 * HW;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    const int r = quant_u8(ldf(base, p)), g = quant_u8(ldf(base, HW + p)), bl = quant_u8(ldf(base, 2 * (size_t)HW + p));
    const int gray = (bl * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14;
    atomicAdd(&h[gray], 1);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[b * 256 + threadIdx.x], h[threadIdx.x]);
}

// ---------------------------------------------------------------------------
// Multi-scale feature sums.  For each image b and scale s (1, 0.5, 0.25):
//   img_s = bilinear(x, size=(int(h*s), int(w*s))) (align_corners=False)
//   f = [img_s (3ch), 0.299R+0.587G+0.114B, sqrt(gx^2+gy^2) (3ch)]
//   sums[b][s] += sum(f)  (double)
// torch.gradient: interior (f[i+1]-f[i-1])/2, one-sided at the edges.
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ float sample_s(const T* img, int H, int W, int hs, int ws, float sy, float sx, int y, int x) {
  if (hs == H && ws == W) return ldf(img, (size_t)y * W + x);
  float fy = sy * (y + 0.5f) - 0.5f; if (fy < 0.f) fy = 0.f;
  float fx = sx * (x + 0.5f) - 0.5f; if (fx < 0.f) fx = 0.f;
  int y0 = (int)fy; if (y0 > H - 1) y0 = H - 1;
  int x0 = (int)fx; if (x0 > W - 1) x0 = W - 1;
  const int y1 = y0 + (y0 < H - 1 ? 1 : 0), x1 = x0 + (x0 < W - 1 ? 1 : 0);
  const float ly = fy - y0, lx = fx - x0;
  const float v00 = ldf(img, (size_t)y0 * W + x0), v01 = ldf(img, (size_t)y0 * W + x1);
  const float v10 = ldf(img, (size_t)y1 * W + x0), v11 = ldf(img, (size_t)y1 * W + x1);
  return (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
}

// One block per (image, 16 x 64 tile of the scaled image): the tile's
// bilinear samples plus a 1-sample halo are computed ONCE into LDS (each is
// read by up to 5 feature terms: value, +-x and +-y neighbours of the
// gradient), then every pixel's 7 features are summed from LDS.  Block sums
// go to the per-(image, scale) accumulator as 64-bit fixed point (2^-24):
// integer atomics, so the total does not depend on block order.
constexpr int MS_TH = 16, MS_TW = 64;
constexpr double kMsFix = 16777216.0;  // 2^24

template <typename T>
__global__ __launch_bounds__(256) void ms_sums_kernel(const T* __restrict__ x, unsigned long long* __restrict__ acc,
                                                      int H, int W, int hs, int ws, int scale_idx, int tiles_x) {
  __shared__ float smp[3][MS_TH + 2][MS_TW + 2];
  __shared__ double red[4];
  const int t = threadIdx.x;
  const int b = blockIdx.y;
  const int ty0 = (blockIdx.x / tiles_x) * MS_TH, tx0 = (blockIdx.x % tiles_x) * MS_TW;  // block-uniform
  const T* img = x + (size_t)b * 3 * H * W;
  const float sy = (float)H / (float)hs, sx = (float)W / (float)ws;
  constexpr int RW = MS_TW + 2, NS = (MS_TH + 2) * RW;
  int r = t / RW, c = t - (t / RW) * RW;
  constexpr int inc_r = 256 / RW, inc_c = 256 - inc_r * RW;
  for (; r < MS_TH + 2; r += inc_r) {
    const int ys = ty0 - 1 + r, xs = tx0 - 1 + c;
    if ((unsigned)ys < (unsigned)hs && (unsigned)xs < (unsigned)ws) {
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) smp[ch][r][c] = sample_s(img + (size_t)ch * H * W, H, W, hs, ws, sy, sx, ys, xs);
    }
    c += inc_c;
    if (c >= RW) { c -= RW; ++r; }
  }
  (void)NS;
  __syncthreads();
  // thread: row t / 16, pixels 4 (t % 16) .. + 3 of the tile
  const int lr = t >> 4, lc0 = (t & 15) * 4;
  const int y = ty0 + lr;
  double a = 0.0;
  if (y < hs) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int xx = tx0 + lc0 + k;
      if (xx >= ws) break;
      const int R = lr + 1, C = lc0 + k + 1;
      float c3[3];
      float fsum = 0.f;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const float v = smp[ch][R][C];
        c3[ch] = v;
        float gx, gy;
        if (ws < 2) gx = 0.f;
        else if (xx == 0) gx = smp[ch][R][C + 1] - v;
        else if (xx == ws - 1) gx = v - smp[ch][R][C - 1];
        else gx = (smp[ch][R][C + 1] - smp[ch][R][C - 1]) / 2.f;
        if (hs < 2) gy = 0.f;
        else if (y == 0) gy = smp[ch][R + 1][C] - v;
        else if (y == hs - 1) gy = v - smp[ch][R - 1][C];
        else gy = (smp[ch][R + 1][C] - smp[ch][R - 1][C]) / 2.f;
        fsum += v + sqrtf(gx * gx + gy * gy);
      }
      fsum += 0.299f * c3[0] + 0.587f * c3[1] + 0.114f * c3[2];
      a += (double)fsum;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if ((t & 63) == 0) red[t >> 6] = a;
  __syncthreads();
  if (t == 0) {
    const double blk = red[0] + red[1] + red[2] + red[3];
    atomicAdd(&acc[b * 3 + scale_idx], (unsigned long long)(long long)llrint(blk * kMsFix));
  }
}

// One pass for all three scales (H % 4 == 0, W % 4 == 0: the 0.5 / 0.25
// bilinear samples are then 2x2 blends of full-resolution pixels, taps at
// rows / columns 2y, 2y + 1 and 4y + 1, 4y + 2, weights exactly 0.5).  A block
// owns a 32 x 64 full-resolution tile = a 16 x 32 half and an 8 x 16 quarter
// tile; it stages the full-resolution region with a 4-pixel halo in LDS
// (every pixel of the image is read from HBM once, halos from L2), forms the
// half / quarter samples (+ their 1-sample halos) from LDS with sample_s's
// arithmetic, and sums the 7 features of all three tiles.  The three block
// sums are stored to the tile's partial slot and the block ends; ms_fin_kernel
// adds an image's partials in tile order (fp64, deterministic) and writes the
// sums and the factor.  (An earlier form ended every block with fixed-point
// atomics and an arrival counter, the last block finishing the image: the
// blocks' atomic tails held their LDS and cost more than the extra launch.)
constexpr int M3_TH = 32, M3_TW = 64, M3_HALO = 4;
constexpr int M3_RH = M3_TH + 2 * M3_HALO, M3_RW = M3_TW + 2 * M3_HALO;
constexpr int M3_H1 = M3_TH / 2 + 2, M3_W1 = M3_TW / 2 + 2, M3_H2 = M3_TH / 4 + 2, M3_W2 = M3_TW / 4 + 2;
// half / quarter sample planes: interior columns from 4 (16-byte aligned
// quads), the 1-sample halo at columns 3 and 4 + width
constexpr int M3_P1 = M3_TW / 2 + 8, M3_P2 = M3_TW / 4 + 8;

__device__ __forceinline__ float blend_half(float v00, float v01, float v10, float v11) {
  const float ly = 0.5f, lx = 0.5f;  // sample_s with fy - y0 = fx - x0 = 0.5
  return (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
}

// the 7 features of pixel (R, C) of an LDS image P (3 planes of PH x PW)
// whose pixel (R, C) is image pixel (y, x) of an hs x ws scale (torch.gradient:
// central differences, one-sided at the borders).  The gradient magnitude
// takes the hardware square root (v_sqrt_f32, <= 1 ulp) instead of the
// correctly rounded expansion (~15 instructions each, 3 per pixel: that
// expansion was a third of this pass's VALU work); the sums feed means over
// >= 10^5 pixels, and the factor stays within 1e-8 of the oracle's (tests
// hold it to 1e-6).  The feature MAPS (ms_features_kernel) keep sqrtf.
template <int PH, int PW>
__device__ __forceinline__ float ms_feat(const float (&P)[3][PH][PW], int R, int C, int y, int x, int hs, int ws) {
  float c3[3];
  float fsum = 0.f;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float v = P[ch][R][C];
    c3[ch] = v;
    float gx, gy;
    if (ws < 2) gx = 0.f;
    else if (x == 0) gx = P[ch][R][C + 1] - v;
    else if (x == ws - 1) gx = v - P[ch][R][C - 1];
    else gx = (P[ch][R][C + 1] - P[ch][R][C - 1]) / 2.f;
    if (hs < 2) gy = 0.f;
    else if (y == 0) gy = P[ch][R + 1][C] - v;
    else if (y == hs - 1) gy = v - P[ch][R - 1][C];
    else gy = (P[ch][R + 1][C] - P[ch][R - 1][C]) / 2.f;
    fsum += v + __builtin_amdgcn_sqrtf(gx * gx + gy * gy);
  }
  fsum += 0.299f * c3[0] + 0.587f * c3[1] + 0.114f * c3[2];
  return fsum;
}

// the features of the 4 pixels (R, C .. C + 3) (C 16-byte aligned) of image
// row y, columns x .. x + 3, summed in fp64 as ms_feat's per-pixel floats
// (same expression, same order: bit-identical to ms_feat on every pixel).
// Every lane of the wave calls it (DPP below): lanes whose quad lies outside
// the hs x ws image contribute 0, as do the pixels of a quad past ws.  A
// lane's quads sit along a DPP row of 16 lanes: the left / right neighbour
// columns come from the adjacent lanes' quads (row_shr / row_shl by 1) and
// only a row's first / last lane (first / last) reads them from LDS -- the
// stride-4 single-float LDS reads were 4-way bank conflicts on every lane.
// Image borders: a missing neighbour is replaced by the centre pixel and the
// difference is not halved (torch.gradient's one-sided edge difference).
__device__ __forceinline__ float dpp_from_left(float v) {  // lane i <- lane i - 1 within its row of 16
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x111, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_from_right(float v) {  // lane i <- lane i + 1 within its row of 16
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x101, 0xF, 0xF, false));
}

// EDGE false: the caller's block holds no image border (block-uniform), so
// none of the border selects are needed
template <bool EDGE, int PH, int PW>
__device__ __forceinline__ double ms_quad(const float (&P)[3][PH][PW], int R, int C, int y, int x, int hs, int ws,
                                          bool first, bool last) {
  const bool top = EDGE && y == 0, bot = EDGE && y >= hs - 1;  // (hs < 2: both)
  const float sy = top || bot ? 1.f : 0.5f;
  float fs[4] = {0.f, 0.f, 0.f, 0.f}, c3[3][4];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float4 ce = *(const float4*)&P[ch][R][C];
    float4 up = *(const float4*)&P[ch][R - 1][C];
    float4 dn = *(const float4*)&P[ch][R + 1][C];
    float l = dpp_from_left(ce.w), r = dpp_from_right(ce.x);
    if (first) l = P[ch][R][C - 1];
    if (last) r = P[ch][R][C + 4];
    if (top) up = ce;
    if (bot) dn = ce;
    const float v[6] = {l, ce.x, ce.y, ce.z, ce.w, r};
    const float u[4] = {up.x, up.y, up.z, up.w}, d[4] = {dn.x, dn.y, dn.z, dn.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool lft = EDGE && x + k == 0, rgt = EDGE && x + k >= ws - 1;
      const float a = lft ? v[k + 1] : v[k], b = rgt ? v[k + 1] : v[k + 2];
      const float gx = (b - a) * (lft || rgt ? 1.f : 0.5f);
      const float gy = (d[k] - u[k]) * sy;
      fs[k] += v[k + 1] + __builtin_amdgcn_sqrtf(gx * gx + gy * gy);
      c3[ch][k] = v[k + 1];
    }
  }
  double a = 0.0;
  if (!EDGE || y < hs) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (!EDGE || x + k < ws) a += (double)(fs[k] + (0.299f * c3[0][k] + 0.587f * c3[1][k] + 0.114f * c3[2][k]));
  }
  return a;
}

// the block's feature quads: 512 of the full tile (2 per thread), 128 half
// (threads 0-127), 32 quarter (128-159)
template <bool E>
__device__ __forceinline__ void ms_tile_quads(const float (&full)[3][M3_RH][M3_RW], const float (&s1)[3][M3_H1][M3_P1],
                                              const float (&s2)[3][M3_H2][M3_P2], int t, int ty0, int tx0, int H,
                                              int W, double& a0, double& a1, double& a2) {
  a0 = 0.0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = t + 256 * k, r = i >> 4, q = i & 15;
    a0 += ms_quad<E>(full, r + M3_HALO, 4 * q + M3_HALO, ty0 + r, tx0 + 4 * q, H, W, q == 0, q == 15);
  }
  // (one value selected afterwards: assigning a1 / a2 inside the branches
  // became a dynamically indexed scratch pair)
  double ah = 0.0;
  if (t < 128) {  // (waves 0, 1: whole)
    const int r = t >> 3, q = t & 7;
    ah = ms_quad<E>(s1, r + 1, 4 * q + 4, ty0 / 2 + r, tx0 / 2 + 4 * q, H / 2, W / 2, q == 0, q == 7);
  } else if (t < 160) {  // (lanes 0-31 of wave 2: two whole DPP rows)
    const int r = (t - 128) >> 2, q = (t - 128) & 3;
    ah = ms_quad<E>(s2, r + 1, 4 * q + 4, ty0 / 4 + r, tx0 / 4 + 4 * q, H / 4, W / 4, q == 0, q == 3);
  }
  a1 = t < 128 ? ah : 0.0;
  a2 = t < 128 ? 0.0 : ah;
}

__device__ __forceinline__ double ms_factor(const double* sums, int b, double n0, double n1, double n2);

template <typename T>
__global__ __launch_bounds__(256) void ms_sums3_kernel(const T* __restrict__ x, double* __restrict__ part, int H,
                                                       int W, int tiles_x) {
  __shared__ float full[3][M3_RH][M3_RW];
  __shared__ __attribute__((aligned(16))) float s1[3][M3_H1][M3_P1];
  __shared__ __attribute__((aligned(16))) float s2[3][M3_H2][M3_P2];
  __shared__ double red[4][3];
  const int t = threadIdx.x;
  // tiles in XCD-contiguous order (blocks i, i + 8, ... share an XCD: they take
  // neighbouring tiles, whose 4-pixel halo lines then come from that XCD's L2;
  // dealt round-robin, every tile's halos were fetched from HBM twice)
  const int nb = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, k8 = bid >> 3;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + k8;
  const int b = tile / gridDim.x, tin = tile - b * gridDim.x;
  const int ty0 = (tin / tiles_x) * M3_TH, tx0 = (tin % tiles_x) * M3_TW;
  const size_t HW = (size_t)H * W;
  const T* img = x + (size_t)b * 3 * HW;
  // full-resolution region: rows ty0 - 4 .., columns tx0 - 4 .. in 4-pixel quads
  // every quad's load is issued before the first LDS store (NLD loads in
  // flight per thread: one HBM round trip per block, not one per quad).  (A
  // persistent form loading tile j + 1 under tile j's work measured no faster:
  // 0.074 vs 0.071 ms)
  // thread (lr, lq) = quad lq of region rows lr + 14 k (k < 3 covers the 40
  // rows), all three channels: the 9 loads' offsets are compile-time steps
  // from one base (the per-quad division / modulo of a flat index was a fifth
  // of this pass's VALU work)
  constexpr int QPR = M3_RW / 4, LR = 256 / QPR, NK = (M3_RH + LR - 1) / LR;
  const int lr = t / QPR, lq = t - lr * QPR;
  const bool lact = t < LR * QPR;
  const int xs = tx0 - M3_HALO + 4 * lq, ys0 = ty0 - M3_HALO + lr;
  const bool xok = lact && (unsigned)xs < (unsigned)W;
  float v[3][NK][4];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int ys = ys0 + LR * k;
    const bool ok = xok && lr + LR * k < M3_RH && (unsigned)ys < (unsigned)H;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      v[ch][k][0] = v[ch][k][1] = v[ch][k][2] = v[ch][k][3] = 0.f;
      if (ok) Vec4<T>::load(img + ch * HW + (size_t)ys * W + xs, v[ch][k]);
    }
  }
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    if (lact && lr + LR * k < M3_RH) {
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
        *(float4*)&full[ch][lr + LR * k][4 * lq] = make_float4(v[ch][k][0], v[ch][k][1], v[ch][k][2], v[ch][k][3]);
    }
  }
  __syncthreads();
  const int h1 = H / 2, w1 = W / 2, h2 = H / 4, w2 = W / 4;
  // half / quarter samples with their 1-sample halos (LDS rows of sample r:
  // 2r + 2, 2r + 3 / 4r + 1, 4r + 2 of the region, by the halo of 4); sample
  // column c at plane column c + 3.  Half: thread (r0, c) = (t / 34, t % 34)
  // takes rows r0 + 7 j (j < 3); quarter: threads 238.. and a second pass
  {
    constexpr int R1 = 256 / M3_W1;  // 7 half rows per pass
    const int r0 = t / M3_W1, c = t - r0 * M3_W1;
    const int xs1 = tx0 / 2 - 1 + c;
    if (t < R1 * M3_W1 && (unsigned)xs1 < (unsigned)w1) {
#pragma unroll
      for (int j = 0; j < (M3_H1 + R1 - 1) / R1; ++j) {
        const int r = r0 + R1 * j, ys = ty0 / 2 - 1 + r;
        if (r < M3_H1 && (unsigned)ys < (unsigned)h1) {
#pragma unroll
          for (int ch = 0; ch < 3; ++ch)
            s1[ch][r][c + 3] = blend_half(full[ch][2 * r + 2][2 * c + 2], full[ch][2 * r + 2][2 * c + 3],
                                          full[ch][2 * r + 3][2 * c + 2], full[ch][2 * r + 3][2 * c + 3]);
        }
      }
    }
    // quarter: 10 x 18 samples over threads 0..179
    const int r2 = t / M3_W2, c2 = t - r2 * M3_W2;
    const int ys2 = ty0 / 4 - 1 + r2, xs2 = tx0 / 4 - 1 + c2;
    if (t < M3_H2 * M3_W2 && (unsigned)ys2 < (unsigned)h2 && (unsigned)xs2 < (unsigned)w2) {
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
        s2[ch][r2][c2 + 3] = blend_half(full[ch][4 * r2 + 1][4 * c2 + 1], full[ch][4 * r2 + 1][4 * c2 + 2],
                                        full[ch][4 * r2 + 2][4 * c2 + 1], full[ch][4 * r2 + 2][4 * c2 + 2]);
    }
  }
  __syncthreads();
  double a0, a1, a2;
  // a tile touching no image border (at any of the three scales: the half /
  // quarter tiles' borders are the full tile's) takes the select-free form
  if (ty0 == 0 || tx0 == 0 || ty0 + M3_TH >= H || tx0 + M3_TW >= W)
    ms_tile_quads<true>(full, s1, s2, t, ty0, tx0, H, W, a0, a1, a2);
  else
    ms_tile_quads<false>(full, s1, s2, t, ty0, tx0, H, W, a0, a1, a2);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a0 += __shfl_xor(a0, o, 64);
    a1 += __shfl_xor(a1, o, 64);
    a2 += __shfl_xor(a2, o, 64);
  }
  if ((t & 63) == 0) { red[t >> 6][0] = a0; red[t >> 6][1] = a1; red[t >> 6][2] = a2; }
  __syncthreads();
  // the block's three sums, plain stores: no atomics or arrival counter to
  // wait for at the end of every block (ms_fin_kernel adds them in order)
  if (t < 3) part[((size_t)b * gridDim.x + tin) * 3 + t] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
}

// Register-streaming form of the one-pass multi-scale sums (round 6): one
// WAVE owns a strip of 256 full-resolution columns (a 4-pixel quad per lane)
// of a band of MSR_BH rows and walks the band's rows top to bottom (plus 3
// halo rows above and below), all three scales from registers -- no LDS, no
// barriers.  Row j's quads arrive MSR_PF rows ahead of their use; full-row
// features take the rows above / below from the register window and the
// left / right neighbour columns from the adjacent lanes (DPP wave_shr:1 /
// wave_shl:1), lane 0 / 63 from a quad of the neighbouring strip that only they
// load.  Half samples (rows 2h, 2h + 1, columns 2c, 2c + 1) and quarter samples
// (rows 4q + 1, 4q + 2, columns 4c + 1, 4c + 2) are blended in registers as rows
// complete and take their neighbours the same way.  Per pixel the arithmetic
// is ms_quad's (bit-identical features); the wave's three fp64 sums go to its
// partial slot, ms_fin_kernel adds an image's slots in order.  (The tiled
// ms_sums3_kernel staged a 40 x 72 region, its half / quarter planes and ran
// three barrier-separated phases per block: 44 us for 32 x 512^2.)
constexpr int MSR_BH = 16, MSR_PF = 2, MSR_NR = MSR_BH + 6;

template <typename F, int... S>
__device__ __forceinline__ void ms_steps(F&& f, std::integer_sequence<int, S...>) {
  (f(std::integral_constant<int, S>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void ms_sfor(F&& f) {  // f(0) .. f(N - 1), each index a compile-time constant
  ms_steps(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ float wave_from_left(float v, float edge) {  // lane i <- lane i - 1; lane 0 <- edge
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_from_right(float v, float edge) {  // lane i <- lane i + 1; lane 63 <- edge
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v), 0x130, 0xF, 0xF, false));
}

// features of N consecutive pixels of one row (c[ch][k], neighbours l / r of
// the first / last, rows u / d above / below), ms_quad's expression per pixel
// a value select (an lvalue ?: between array elements became a pointer phi
// that kept the arrays in scratch)
__device__ __forceinline__ float fsel(bool p, float a, float b) { return p ? a : b; }

template <int N>
__device__ __forceinline__ double ms_row_feat(const float (&c)[3][N], const float (&u)[3][N], const float (&d)[3][N],
                                              const float (&l)[3], const float (&r)[3], int y, int x, int hs, int ws) {
  // y is wave-uniform: rows off the image contribute nothing, and only the
  // image's first / last row takes the one-sided vertical difference (a
  // uniform branch); horizontally (W % 4 == 0, aligned quads) only a run's
  // first pixel can sit on column 0 and only its last on column ws - 1, and a
  // run lies wholly inside or outside the image
  if (y < 0 || y >= hs) return 0.0;
  const bool top = y == 0, bot = y >= hs - 1;
  float fs[N];
#pragma unroll
  for (int k = 0; k < N; ++k) fs[k] = 0.f;
  auto body = [&](auto VB_) {
    constexpr bool VB = decltype(VB_)::value;  // vertical border row
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      ms_sfor<N>([&](auto K_) {
        constexpr int k = decltype(K_)::value;
        float vl, vr;
        if constexpr (k == 0) vl = l[ch]; else vl = c[ch][k - 1];
        if constexpr (k == N - 1) vr = r[ch]; else vr = c[ch][k + 1];
        const float v = c[ch][k];
        float gx;
        if constexpr (k == 0 || k == N - 1) {
          const bool lft = k == 0 && x == 0, rgt = k == N - 1 && x + k >= ws - 1;
          const float a = fsel(lft, v, vl), b = fsel(rgt, v, vr);
          gx = (b - a) * fsel(lft || rgt, 1.f, 0.5f);
        } else {
          gx = (vr - vl) * 0.5f;
        }
        float gy;
        if constexpr (VB) {
          const float uu = fsel(top, v, u[ch][k]), dd = fsel(bot, v, d[ch][k]);
          gy = (dd - uu) * fsel(top || bot, 1.f, 0.5f);
        } else {
          gy = (d[ch][k] - u[ch][k]) * 0.5f;
        }
        fs[k] += v + __builtin_amdgcn_sqrtf(gx * gx + gy * gy);
      });
    }
  };
  if (top || bot) body(std::true_type{});
  else body(std::false_type{});
  double a = 0.0;
  if (x < ws) {
#pragma unroll
    for (int k = 0; k < N; ++k) a += (double)(fs[k] + (0.299f * c[0][k] + 0.587f * c[1][k] + 0.114f * c[2][k]));
  }
  return a;
}

template <typename T>
__global__ __launch_bounds__(256, 2) void ms_rows_kernel(const T* __restrict__ x, double* __restrict__ part, int B,
                                                      int H, int W, int strips, int nwav) {
  const int lane = threadIdx.x & 63;
  // waves in XCD-contiguous order over (image, wave): blocks i, i + 8, ... share
  // an XCD and take neighbouring bands, whose halo rows then hit that L2
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, k8 = bid >> 3;
  const int blk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + k8;
  // global wave = image * nwav + wave; readfirstlane: everything derived from
  // it is wave-uniform (SGPRs), or every buffer load became a waterfall loop
  const int gw = blk * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int b = gw / nwav, wv = gw - b * nwav;
  if (b >= B) return;  // (the last block's spare waves)
  const int band = wv / strips, strip = wv - band * strips;
  const int y0 = band * MSR_BH, xs = strip * 256, xq = xs + 4 * lane;
  const int hs1 = H / 2, ws1 = W / 2, hs2 = H / 4, ws2 = W / 4;
  const size_t HW = (size_t)H * W;
  const T* img = x + (size_t)b * 3 * HW;
  const bool qin = xq < W;
  // the neighbouring strip's quad of the edge lanes: lane 0 cols xs - 4 .. xs - 1, lane 63 xs + 256 .. + 259
  const int xe = lane == 0 ? xs - 4 : xs + 256;  // (fp32 reads 3 columns from xe + 1 / xe on lane 0 / 63)
  const bool ein = (lane == 0 || lane == 63) && xe >= 0 && xe < W;
  // row j of the window = image row y0 - 3 + j; V: the lane's quad, E: the edge quad's
  // three columns that the neighbours use (lane 0: xs - 3, xs - 2, xs - 1; lane 63: xs + 256 .. + 258)
  float V[MSR_NR][3][4], E[MSR_NR][3][3];
  // loads are unconditional, from clamped (always valid) addresses, and zeroed
  // by a select after the fact: a load under a divergent branch came with a
  // vmcnt(0) at the branch's merge, serialising every row's loads.  They are
  // buffer loads: a per-lane 32-bit column offset fixed for the wave + a
  // wave-uniform row offset (64-bit per-lane addresses for every row of the
  // unrolled walk took 264 registers)
  // the buffer's range is the image: a lane whose quad lies off the image (and
  // every lane but 0 / 63 for the edge load) reads at an offset past it, which
  // returns zeros without a memory access
  const int ib = 3 * (int)HW * (int)sizeof(T);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)img, 0, ib, 0x00020000);
  constexpr int kOff = 0x40000000;
  const int vq = qin ? xq * (int)sizeof(T) : kOff;
  const int ve = ein ? (sizeof(T) == 4 && lane == 0 ? xe + 1 : xe) * (int)sizeof(T) : kOff;
  auto bld = [&](int voff, int soff, float (&v)[4]) {
    if constexpr (sizeof(T) == 4) {
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
      v[0] = __uint_as_float(q[0]); v[1] = __uint_as_float(q[1]); v[2] = __uint_as_float(q[2]); v[3] = __uint_as_float(q[3]);
    } else {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
      const h4 hv = __builtin_bit_cast(h4, q);
      v[0] = (float)hv[0]; v[1] = (float)hv[1]; v[2] = (float)hv[2]; v[3] = (float)hv[3];
    }
  };
  auto load_row = [&](auto J_) {
    constexpr int j = decltype(J_)::value;
    const int y = y0 - 3 + j;
    const bool yin = y >= 0 && y < H;  // (wave-uniform)
    // rows off the image: every lane's offset out of range (the range check is
    // on the per-lane offset; the row's soffset stays a valid one)
    const int ro = yin ? y * W : 0;
    const int vqr = yin ? vq : kOff, ver = yin ? ve : kOff;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      float v[4];
      const int so = (ch * (int)HW + ro) * (int)sizeof(T);
      bld(vqr, so, v);
#pragma unroll
      for (int k = 0; k < 4; ++k) V[j][ch][k] = v[k];
      if constexpr (sizeof(T) == 4) {
        // the three edge columns straight from one 12-byte load (lane 0: xs - 3 ..; lane 63: xs + 256 ..)
        typedef unsigned u32x3 __attribute__((ext_vector_type(3)));
        const u32x3 q = __builtin_amdgcn_raw_buffer_load_b96(rs, ver, so, 0);
#pragma unroll
        for (int k = 0; k < 3; ++k) E[j][ch][k] = __uint_as_float(q[k]);
      } else {
        float e[4];
        bld(ver, so, e);
        const bool l0 = lane == 0;
        E[j][ch][0] = fsel(l0, e[1], e[0]);
        E[j][ch][1] = fsel(l0, e[2], e[1]);
        E[j][ch][2] = fsel(l0, e[3], e[2]);
      }
    }
  };
  // half samples: sample row k (k = 0 .. MSR_BH / 2 + 1) = half row y0 / 2 - 1 + k from window rows 1 + 2k, 2 + 2k;
  // quarter sample row k (k = 0 .. MSR_BH / 4 + 1) = quarter row y0 / 4 - 1 + k from window rows 4k, 4k + 1
  float S1[MSR_BH / 2 + 2][3][2], S1e[MSR_BH / 2 + 2][3];  // the lane's 2 half pixels, the edge lane's neighbour
  float S2[MSR_BH / 4 + 2][3], S2e[MSR_BH / 4 + 2][3];
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  ms_sfor<MSR_PF + 1>([&](auto J_) { load_row(J_); });
  ms_sfor<MSR_NR>([&](auto J_) {
    constexpr int j = decltype(J_)::value;
    // (a compiler-only fence per row: without it every row's loads were hoisted
    // to the top -- 316 registers, one wave per SIMD)
    asm volatile("" ::: "memory");
    if constexpr (j + MSR_PF + 1 < MSR_NR) load_row(std::integral_constant<int, j + MSR_PF + 1>{});
    // full features of window row j - 1 (image rows y0 .. y0 + MSR_BH - 1: j - 1 in 3 .. MSR_BH + 2)
    if constexpr (j - 1 >= 3 && j - 1 < MSR_BH + 3) {
      constexpr int m = j - 1;
      float l[3], r[3];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        l[ch] = wave_from_left(V[m][ch][3], E[m][ch][2]);
        r[ch] = wave_from_right(V[m][ch][0], E[m][ch][0]);
      }
      a0 += ms_row_feat<4>(V[m], V[m - 1], V[m + 1], l, r, y0 - 3 + m, xq, H, W);
    }
    // half sample row k once window row 2 + 2k is in
    if constexpr (j >= 2 && j % 2 == 0) {
      constexpr int k = (j - 2) / 2;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        S1[k][ch][0] = blend_half(V[j - 1][ch][0], V[j - 1][ch][1], V[j][ch][0], V[j][ch][1]);
        S1[k][ch][1] = blend_half(V[j - 1][ch][2], V[j - 1][ch][3], V[j][ch][2], V[j][ch][3]);
        const bool l0 = lane == 0;  // (value selects: a ?: of two blend calls became pointer phis into scratch)
        S1e[k][ch] = blend_half(fsel(l0, E[j - 1][ch][1], E[j - 1][ch][0]), fsel(l0, E[j - 1][ch][2], E[j - 1][ch][1]),
                                fsel(l0, E[j][ch][1], E[j][ch][0]), fsel(l0, E[j][ch][2], E[j][ch][1]));
      }
      // half features of sample row k - 1 (half rows y0 / 2 .. y0 / 2 + MSR_BH / 2 - 1: k - 1 in 1 .. MSR_BH / 2)
      if constexpr (k - 1 >= 1 && k - 1 <= MSR_BH / 2) {
        constexpr int m = k - 1;
        float l[3], r[3];
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          l[ch] = wave_from_left(S1[m][ch][1], S1e[m][ch]);
          r[ch] = wave_from_right(S1[m][ch][0], S1e[m][ch]);
        }
        a1 += ms_row_feat<2>(S1[m], S1[m - 1], S1[m + 1], l, r, y0 / 2 - 1 + m, xq / 2, hs1, ws1);
      }
    }
    // quarter sample row k once window row 4k + 1 is in
    if constexpr (j % 4 == 1) {
      constexpr int k = (j - 1) / 4;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        S2[k][ch] = blend_half(V[j - 1][ch][1], V[j - 1][ch][2], V[j][ch][1], V[j][ch][2]);
        const bool l0 = lane == 0;
        S2e[k][ch] = blend_half(fsel(l0, E[j - 1][ch][0], E[j - 1][ch][1]), fsel(l0, E[j - 1][ch][1], E[j - 1][ch][2]),
                                fsel(l0, E[j][ch][0], E[j][ch][1]), fsel(l0, E[j][ch][1], E[j][ch][2]));
      }
      if constexpr (k - 1 >= 1 && k - 1 <= MSR_BH / 4) {
        constexpr int m = k - 1;
        float l[3], r[3], c1[3][1], u1[3][1], d1[3][1];
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          l[ch] = wave_from_left(S2[m][ch], S2e[m][ch]);
          r[ch] = wave_from_right(S2[m][ch], S2e[m][ch]);
          c1[ch][0] = S2[m][ch];
          u1[ch][0] = S2[m - 1][ch];
          d1[ch][0] = S2[m + 1][ch];
        }
        a2 += ms_row_feat<1>(c1, u1, d1, l, r, y0 / 4 - 1 + m, xq / 4, hs2, ws2);
      }
    }
  });
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a0 += __shfl_xor(a0, o, 64);
    a1 += __shfl_xor(a1, o, 64);
    a2 += __shfl_xor(a2, o, 64);
  }
  if (lane < 3) part[((size_t)b * nwav + wv) * 3 + lane] = lane == 0 ? a0 : lane == 1 ? a1 : a2;
}

// One CHANNEL per wave (round 6, the default): the register-streaming walk of
// ms_rows_kernel over one colour plane.  SQ counters on ms_rows_kernel
// (profiles/r6_ms_rows_sq_counters.txt) showed its waves issue-stalled (47% of
// their cycles waiting on dependent VALU results, 27% issuing) at two waves
// per SIMD (256 VGPRs: three planes' windows and loads in flight): with one
// plane a wave needs a third of the registers, and four-plus waves per SIMD
// hide each other's dependency chains.  The 7 features of a pixel are summed
// as sum over channels of (v + |grad v|) plus the luminance, and the
// luminance's sum is linear in the planes: 0.299f * sum r + 0.587f * sum g +
// 0.114f * sum b (the sampled half / quarter planes are linear blends too).
// So a wave keeps, per scale, the sum of v + |grad v| and the sum of v over
// its pixels (fp32 over a lane's run of a row, fp64 across rows and lanes),
// and ms_fin1_kernel combines an image's 3 planes in a fixed order.  The
// rounding differs from ms_rows_kernel's per-pixel fp32 sum of the 7 terms
// at the 1e-7 relative level (the sums test holds 1e-6 vs the oracle's maps).
template <int N>
__device__ __forceinline__ void ms_row_feat1(const float (&c)[N], const float (&u)[N], const float (&d)[N], float l,
                                             float r, int y, int x, int hs, int ws, double& af, double& av) {
  if (y < 0 || y >= hs) return;  // (wave-uniform)
  const bool top = y == 0, bot = y >= hs - 1;
  float fs = 0.f, vs = 0.f;
  auto body = [&](auto VB_) {
    constexpr bool VB = decltype(VB_)::value;  // vertical border row
    ms_sfor<N>([&](auto K_) {
      constexpr int k = decltype(K_)::value;
      float vl, vr;
      if constexpr (k == 0) vl = l; else vl = c[k - 1];
      if constexpr (k == N - 1) vr = r; else vr = c[k + 1];
      const float v = c[k];
      float gx;
      if constexpr (k == 0 || k == N - 1) {
        const bool lft = k == 0 && x == 0, rgt = k == N - 1 && x + k >= ws - 1;
        const float a = fsel(lft, v, vl), b = fsel(rgt, v, vr);
        gx = (b - a) * fsel(lft || rgt, 1.f, 0.5f);
      } else {
        gx = (vr - vl) * 0.5f;
      }
      float gy;
      if constexpr (VB) {
        const float uu = fsel(top, v, u[k]), dd = fsel(bot, v, d[k]);
        gy = (dd - uu) * fsel(top || bot, 1.f, 0.5f);
      } else {
        gy = (d[k] - u[k]) * 0.5f;
      }
      fs += v + __builtin_amdgcn_sqrtf(gx * gx + gy * gy);
      vs += v;
    });
  };
  if (top || bot) body(std::true_type{});
  else body(std::false_type{});
  if (x < ws) {
    af += (double)fs;
    av += (double)vs;
  }
}

template <typename T, int BH>
__global__ __launch_bounds__(256, 4) void ms_rows1_kernel(const T* __restrict__ x, double* __restrict__ part, int B,
                                                       int H, int W, int strips, int nwav) {
  constexpr int NR = BH + 6;
  static_assert(BH % 4 == 0, "bands of whole quarter rows");
  const int lane = threadIdx.x & 63;
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, k8 = bid >> 3;
  const int blk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + k8;
  // global wave = (image * 3 + channel) * nwav + wave (readfirstlane: wave-uniform)
  const int gw = blk * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int bc = gw / nwav, wv = gw - bc * nwav;
  if (bc >= 3 * B) return;  // (the last block's spare waves)
  const int band = wv / strips, strip = wv - band * strips;
  const int y0 = band * BH, xs = strip * 256, xq = xs + 4 * lane;
  const int hs1 = H / 2, ws1 = W / 2, hs2 = H / 4, ws2 = W / 4;
  const size_t HW = (size_t)H * W;
  const T* plane = x + (size_t)bc * HW;
  const bool qin = xq < W;
  const int xe = lane == 0 ? xs - 4 : xs + 256;
  const bool ein = (lane == 0 || lane == 63) && xe >= 0 && xe < W;
  float V[NR][4], E[NR][3];
  // buffer over the plane: off-image lanes read zeros without a memory access
  // (ms_rows_kernel's scheme, one plane)
  const int ib = (int)HW * (int)sizeof(T);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)plane, 0, ib, 0x00020000);
  constexpr int kOff = 0x40000000;
  const int vq = qin ? xq * (int)sizeof(T) : kOff;
  const int ve = ein ? (sizeof(T) == 4 && lane == 0 ? xe + 1 : xe) * (int)sizeof(T) : kOff;
  auto load_row = [&](auto J_) {
    constexpr int j = decltype(J_)::value;
    const int y = y0 - 3 + j;
    const bool yin = y >= 0 && y < H;  // (wave-uniform)
    const int so = (yin ? y * W : 0) * (int)sizeof(T);
    const int vqr = yin ? vq : kOff, ver = yin ? ve : kOff;
    if constexpr (sizeof(T) == 4) {
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      typedef unsigned u32x3 __attribute__((ext_vector_type(3)));
      const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, vqr, so, 0);
      const u32x3 e = __builtin_amdgcn_raw_buffer_load_b96(rs, ver, so, 0);
#pragma unroll
      for (int k = 0; k < 4; ++k) V[j][k] = __uint_as_float(q[k]);
#pragma unroll
      for (int k = 0; k < 3; ++k) E[j][k] = __uint_as_float(e[k]);
    } else {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      const h4 hv = __builtin_bit_cast(h4, __builtin_amdgcn_raw_buffer_load_b64(rs, vqr, so, 0));
      const h4 he = __builtin_bit_cast(h4, __builtin_amdgcn_raw_buffer_load_b64(rs, ver, so, 0));
#pragma unroll
      for (int k = 0; k < 4; ++k) V[j][k] = (float)hv[k];
      const bool l0 = lane == 0;
      E[j][0] = fsel(l0, (float)he[1], (float)he[0]);
      E[j][1] = fsel(l0, (float)he[2], (float)he[1]);
      E[j][2] = fsel(l0, (float)he[3], (float)he[2]);
    }
  };
  float S1[BH / 2 + 2][2], S1e[BH / 2 + 2];
  float S2[BH / 4 + 2], S2e[BH / 4 + 2];
  double f0 = 0.0, v0 = 0.0, f1 = 0.0, v1 = 0.0, f2 = 0.0, v2 = 0.0;
  ms_sfor<MSR_PF + 1>([&](auto J_) { load_row(J_); });
  ms_sfor<NR>([&](auto J_) {
    constexpr int j = decltype(J_)::value;
    asm volatile("" ::: "memory");
    if constexpr (j + MSR_PF + 1 < NR) load_row(std::integral_constant<int, j + MSR_PF + 1>{});
    if constexpr (j - 1 >= 3 && j - 1 < BH + 3) {
      constexpr int m = j - 1;
      const float l = wave_from_left(V[m][3], E[m][2]), r = wave_from_right(V[m][0], E[m][0]);
      ms_row_feat1<4>(V[m], V[m - 1], V[m + 1], l, r, y0 - 3 + m, xq, H, W, f0, v0);
    }
    if constexpr (j >= 2 && j % 2 == 0) {
      constexpr int k = (j - 2) / 2;
      S1[k][0] = blend_half(V[j - 1][0], V[j - 1][1], V[j][0], V[j][1]);
      S1[k][1] = blend_half(V[j - 1][2], V[j - 1][3], V[j][2], V[j][3]);
      const bool l0 = lane == 0;
      S1e[k] = blend_half(fsel(l0, E[j - 1][1], E[j - 1][0]), fsel(l0, E[j - 1][2], E[j - 1][1]),
                          fsel(l0, E[j][1], E[j][0]), fsel(l0, E[j][2], E[j][1]));
      if constexpr (k - 1 >= 1 && k - 1 <= BH / 2) {
        constexpr int m = k - 1;
        const float l = wave_from_left(S1[m][1], S1e[m]), r = wave_from_right(S1[m][0], S1e[m]);
        ms_row_feat1<2>(S1[m], S1[m - 1], S1[m + 1], l, r, y0 / 2 - 1 + m, xq / 2, hs1, ws1, f1, v1);
      }
    }
    if constexpr (j % 4 == 1) {
      constexpr int k = (j - 1) / 4;
      S2[k] = blend_half(V[j - 1][1], V[j - 1][2], V[j][1], V[j][2]);
      const bool l0 = lane == 0;
      S2e[k] = blend_half(fsel(l0, E[j - 1][0], E[j - 1][1]), fsel(l0, E[j - 1][1], E[j - 1][2]),
                          fsel(l0, E[j][0], E[j][1]), fsel(l0, E[j][1], E[j][2]));
      if constexpr (k - 1 >= 1 && k - 1 <= BH / 4) {
        constexpr int m = k - 1;
        const float l = wave_from_left(S2[m], S2e[m]), r = wave_from_right(S2[m], S2e[m]);
        const float c1[1] = {S2[m]}, u1[1] = {S2[m - 1]}, d1[1] = {S2[m + 1]};
        ms_row_feat1<1>(c1, u1, d1, l, r, y0 / 4 - 1 + m, xq / 4, hs2, ws2, f2, v2);
      }
    }
  });
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    f0 += __shfl_xor(f0, o, 64);
    v0 += __shfl_xor(v0, o, 64);
    f1 += __shfl_xor(f1, o, 64);
    v1 += __shfl_xor(v1, o, 64);
    f2 += __shfl_xor(f2, o, 64);
    v2 += __shfl_xor(v2, o, 64);
  }
  // slot (image, channel, wave): the 3 scales' (sum of v + |grad|, sum of v)
  if (lane < 6) {
    const double o = lane == 0 ? f0 : lane == 1 ? v0 : lane == 2 ? f1 : lane == 3 ? v1 : lane == 4 ? f2 : v2;
    part[(size_t)gw * 6 + lane] = o;
  }
}

__device__ __forceinline__ double ms_factor(const double* sums, int b, double n0, double n1, double n2);

// per image: the (channel, wave) slots of ms_rows1_kernel added in a fixed
// order -- thread t takes waves t, t + 256, ... of every (channel, scale,
// kind), a fixed tree over the block -- then sum_s = sum_ch F[ch][s] +
// 0.299f * V[r][s] + 0.587f * V[g][s] + 0.114f * V[b][s] (the luminance
// weights as the fp32 constants the per-pixel form multiplies by)
__global__ __launch_bounds__(256) void ms_fin1_kernel(const double* __restrict__ part, int nwav,
                                                      double* __restrict__ sums, double* __restrict__ factor, double n0,
                                                      double n1, double n2) {
  __shared__ double red[18][4];
  const int b = blockIdx.x, t = threadIdx.x;
  double a[18];
#pragma unroll
  for (int k = 0; k < 18; ++k) a[k] = 0.0;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch)
    for (int i = t; i < nwav; i += 256) {
      const double* p = part + (((size_t)b * 3 + ch) * nwav + i) * 6;
#pragma unroll
      for (int k = 0; k < 6; ++k) a[ch * 6 + k] += p[k];
    }
  // fixed xor tree within each wave, then the 4 wave sums in order
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int k = 0; k < 18; ++k) a[k] += __shfl_xor(a[k], o, 64);
  if ((t & 63) == 0)
#pragma unroll
    for (int k = 0; k < 18; ++k) red[k][t >> 6] = a[k];
  __syncthreads();
  if (t == 0) {
#pragma unroll
    for (int k = 0; k < 18; ++k) red[k][0] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
    const double wl[3] = {(double)0.299f, (double)0.587f, (double)0.114f};
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      double f = 0.0, l = 0.0;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        f += red[ch * 6 + 2 * s][0];
        l += wl[ch] * red[ch * 6 + 2 * s + 1][0];
      }
      sums[b * 3 + s] = f + l;
    }
    if (factor) factor[b] = ms_factor(sums, b, n0, n1, n2);
  }
}

// per image: the tile partials of ms_sums3_kernel added in a fixed order (one
// block per image; deterministic fp64), then sums and the factor
__global__ __launch_bounds__(256) void ms_fin_kernel(const double* __restrict__ part, int nblk, double* __restrict__ sums,
                                                     double* __restrict__ factor, double n0, double n1, double n2) {
  __shared__ double red[3][256];
  const int b = blockIdx.x, t = threadIdx.x;
  double a[3] = {0.0, 0.0, 0.0};
  for (int i = t; i < nblk; i += 256)
#pragma unroll
    for (int k = 0; k < 3; ++k) a[k] += part[((size_t)b * nblk + i) * 3 + k];
#pragma unroll
  for (int k = 0; k < 3; ++k) red[k][t] = a[k];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o)
#pragma unroll
      for (int k = 0; k < 3; ++k) red[k][t] += red[k][t + o];
    __syncthreads();
  }
  if (t == 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) sums[b * 3 + k] = red[k][0];
    if (factor) factor[b] = ms_factor(sums, b, n0, n1, n2);
  }
}

// fixed-point accumulators -> fp64 sums (in place) and the factor
// factor[b] = 1 + sum_i w_i * mean_i * 0.1, mean_i = float32(sums[b][i] / (7*h_i*w_i))
// (torch.mean returns a float32 tensor; .item() widens it; Python accumulates in
// double, multi_scale.py:310-314)
__device__ __forceinline__ double ms_factor(const double* sums, int b, double n0, double n1, double n2) {
  double f = 1.0;
  f += 0.5 * (double)(float)(sums[b * 3 + 0] / n0) * 0.1;
  f += 0.3 * (double)(float)(sums[b * 3 + 1] / n1) * 0.1;
  f += 0.2 * (double)(float)(sums[b * 3 + 2] / n2) * 0.1;
  return f;
}

__global__ void ms_factor_kernel(double* __restrict__ sums, double* __restrict__ factor, int B, double n0, double n1,
                                 double n2) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  for (int i = 0; i < 3; ++i) {
    const long long q = (long long)((const unsigned long long*)sums)[b * 3 + i];
    sums[b * 3 + i] = (double)q / kMsFix;
  }
  if (factor) factor[b] = ms_factor(sums, b, n0, n1, n2);
}

// clamp(enh * float(factor), 0, 1)   (multi_scale.py:317-318); grid (chunks, B)
template <typename T, int V>
__global__ __launch_bounds__(256) void scale_clamp_kernel(const T* __restrict__ enh, T* __restrict__ out,
                                                          const double* __restrict__ factor, int CHW) {
  const int b = blockIdx.y;
  const float f = (float)factor[b];
  const size_t base = (size_t)b * CHW;
  for (int i = (blockIdx.x * 256 + threadIdx.x) * V; i < CHW; i += gridDim.x * 256 * V) {
    if constexpr (V == 4) {
      float v[4];
      Vec4<T>::load(enh + base + i, v);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = fminf(fmaxf(__fmul_rn(v[k], f), 0.f), 1.f);
      Vec4<T>::store(out + base + i, v);
    } else {
      stf(out, base + i, fminf(fmaxf(__fmul_rn(ldf(enh, base + i), f), 0.f), 1.f));
    }
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
static inline int g1(size_t n) { return (int)((n + 255) / 256); }

// tile geometry of OpenCV's CLAHE_Impl::apply + the band split of the launches
static ClaheArgs clahe_args(int B, int H, int W, float clipLimit, int tilesX, int tilesY, bool split) {
  ClaheArgs g;
  g.H = H; g.W = W; g.tilesX = tilesX; g.tilesY = tilesY;
  const int Hp = (H % tilesY) ? H + tilesY - (H % tilesY) : H;
  const int Wp = (W % tilesX) ? W + tilesX - (W % tilesX) : W;
  g.tileW = Wp / tilesX; g.tileH = Hp / tilesY;
  const int area = g.tileW * g.tileH;
  g.lutScale = 255.0f / (float)area;
  g.clip = 0;
  if (clipLimit > 0.0f) {
    g.clip = (int)(clipLimit * area / 256);
    if (g.clip < 1) g.clip = 1;
  }
  // histogram blocks: (image, tile, band).  With few images, split each tile
  // into S row bands (S | tileH) so the launch still fills the chip, keeping
  // >= ~2048 pixels per block; S = 1 computes the LUT in the same block
  g.S = 1;
  if (split) {
    const long long tiles = (long long)B * tilesX * tilesY;
    for (int S = 2; S <= g.tileH; ++S) {
      if (g.tileH % S) continue;
      if (tiles * (g.S) >= 1024 || (long long)(g.tileH / S) * g.tileW < 2048) break;
      g.S = S;
    }
  }
  g.R = g.tileH / g.S;
  // apply blocks: R3 rows (<= tileH: the band reads <= 3 tile rows of LUTs),
  // ~1024 blocks per launch
  long long r3 = ((long long)B * H + 1023) / 1024;
  r3 = r3 < 1 ? 1 : (r3 > 32 ? 32 : r3);
  g.R3 = (int)(r3 > g.tileH ? g.tileH : r3);
  return g;
}

static size_t clahe_apply_lds(const ClaheArgs& g) { return 4096 * 4 + 256 * 4 + (size_t)3 * g.tilesX * 256; }

// the three launches; src: T RGB planes (SRC 0) or a u8 plane (SRC 1, then L = src)
template <int SRC, typename T>
static int clahe_launch(const void* src, void* out, uint8_t* L, uint8_t* A, uint8_t* Bc, uint8_t* lut, int* part,
                        const DevLab* tab, int B, const ClaheArgs& g, hipStream_t st) {
  if (g.tilesX > 64 || g.tilesY > 64) return kErrUnsupported;  // LDS of the apply kernel's LUT rows
  // 4-pixel items: whole groups of 4 per tile row (no column padding) and per image row
  const bool v4h = g.tileW % 4 == 0 && g.tileW * g.tilesX == g.W;
  const bool v4a = g.W % 4 == 0;
  const dim3 gh(g.tilesX * g.tilesY * g.S, B);
  if (v4h)
    hipLaunchKernelGGL((clahe_hist_kernel<SRC, T, 4>), gh, dim3(256), 0, st, src, L, A, Bc, part, lut, tab, g);
  else
    hipLaunchKernelGGL((clahe_hist_kernel<SRC, T, 1>), gh, dim3(256), 0, st, src, L, A, Bc, part, lut, tab, g);
  UPR_CHECK_HIP(hipGetLastError());
  if (g.S > 1) {
    hipLaunchKernelGGL(clahe_lut_kernel, dim3(g.tilesX * g.tilesY, B), dim3(256), 0, st, (const int*)part, lut, g);
    UPR_CHECK_HIP(hipGetLastError());
  }
  const dim3 ga((g.H + g.R3 - 1) / g.R3, B);
  const size_t lds = clahe_apply_lds(g);
  const uint8_t* Lsrc = SRC == 0 ? L : (const uint8_t*)src;
  constexpr int DST = SRC;
  if (v4a)
    hipLaunchKernelGGL((clahe_apply_kernel<DST, T, 4>), ga, dim3(256), lds, st, Lsrc, A, Bc, lut, tab, out, g);
  else
    hipLaunchKernelGGL((clahe_apply_kernel<DST, T, 1>), ga, dim3(256), lds, st, Lsrc, A, Bc, lut, tab, out, g);
  return (int)hipGetLastError();
}

static size_t clahe_part_bytes(const ClaheArgs& g, int B) {
  return g.S > 1 ? (size_t)B * g.tilesX * g.tilesY * g.S * 256 * sizeof(int) : 0;
}

// workspace: L, A, B planes | LUTs | partial histograms (S > 1)
size_t clahe_pipeline_ws(int B, int H, int W, int tilesX, int tilesY) {
  const ClaheArgs g = clahe_args(B, H, W, 2.0f, tilesX, tilesY, true);
  const size_t planes = ((size_t)B * H * W * 3 + 15) & ~(size_t)15;
  const size_t luts = ((size_t)B * tilesX * tilesY * 256 + 15) & ~(size_t)15;
  return planes + luts + clahe_part_bytes(g, B);
}

int launch_clahe_pipeline(const void* enh, void* out, uint8_t* ws, int B, int H, int W, float clip, int tilesX,
                          int tilesY, int dtype, hipStream_t st) {
  const DevLab* tab = dev_lab_tables(st);
  if (!tab) return kErrUnsupported;
  const ClaheArgs g = clahe_args(B, H, W, clip, tilesX, tilesY, true);
  const size_t HW = (size_t)H * W;
  uint8_t* L = ws;
  uint8_t* A = L + B * HW;
  uint8_t* Bc = A + B * HW;
  uint8_t* lut = ws + (((size_t)B * HW * 3 + 15) & ~(size_t)15);
  int* part = (int*)(lut + (((size_t)B * tilesX * tilesY * 256 + 15) & ~(size_t)15));
  if (dtype == kF16) return clahe_launch<0, half_t>(enh, out, L, A, Bc, lut, part, tab, B, g, st);
  return clahe_launch<0, float>(enh, out, L, A, Bc, lut, part, tab, B, g, st);
}

// u8 plane -> u8 plane (upr_clahe_u8: the caller's workspace holds the LUTs only, so S = 1)
int launch_clahe_u8(const uint8_t* src, uint8_t* dst, uint8_t* lut, int B, int H, int W, float clip, int tilesX,
                    int tilesY, hipStream_t st) {
  const ClaheArgs g = clahe_args(B, H, W, clip, tilesX, tilesY, false);
  return clahe_launch<1, float>(src, dst, nullptr, nullptr, nullptr, lut, nullptr, nullptr, B, g, st);
}

int launch_rgb2lab(const uint8_t* rgb, uint8_t* lab, size_t npix, hipStream_t st) {
  const DevLab* tab = dev_lab_tables(st);
  if (!tab) return kErrUnsupported;
  hipLaunchKernelGGL(rgb2lab_kernel, dim3(g1(npix)), dim3(256), 0, st, rgb, lab, tab, npix);
  return (int)hipGetLastError();
}

int launch_lab2rgb(const uint8_t* lab, uint8_t* rgb, size_t npix, hipStream_t st) {
  const DevLab* tab = dev_lab_tables(st);
  if (!tab) return kErrUnsupported;
  hipLaunchKernelGGL(lab2rgb_kernel, dim3(g1(npix)), dim3(256), 0, st, lab, rgb, tab, npix);
  return (int)hipGetLastError();
}

int launch_quantize(const void* x, uint8_t* out, size_t n, int dtype, hipStream_t st) {
  if (dtype == kF16)
    hipLaunchKernelGGL((quant_kernel<half_t>), dim3(g1(n)), dim3(256), 0, st, (const half_t*)x, out, n);
  else
    hipLaunchKernelGGL((quant_kernel<float>), dim3(g1(n)), dim3(256), 0, st, (const float*)x, out, n);
  return (int)hipGetLastError();
}

int launch_gray_hist(const void* img, int* hist, int B, int H, int W, int dtype, hipStream_t st) {
  UPR_CHECK_HIP(hipMemsetAsync(hist, 0, sizeof(int) * 256 * B, st));
  const int HW = H * W;
  const int gx = min(g1(HW), 256);
  if (dtype == kF16)
    hipLaunchKernelGGL((gray_hist_kernel<half_t>), dim3(gx, B), dim3(256), 0, st, (const half_t*)img, hist, HW);
  else
    hipLaunchKernelGGL((gray_hist_kernel<float>), dim3(gx, B), dim3(256), 0, st, (const float*)img, hist, HW);
  return (int)hipGetLastError();
}

int launch_multiscale(const void* x, const void* enh, void* out, double* sums, double* factor, int B, int H, int W,
                      int dtype, hipStream_t st) {
  const int hs[3] = {H, (int)(H * 0.5), (int)(H * 0.25)};
  const int wsz[3] = {W, (int)(W * 0.5), (int)(W * 0.25)};
  for (int s = 0; s < 3; ++s)
    if (hs[s] < 1 || wsz[s] < 1) return kErrShape;
  const double n0 = 7.0 * hs[0] * wsz[0], n1 = 7.0 * hs[1] * wsz[1], n2 = 7.0 * hs[2] * wsz[2];
  // the clamp needs the factor: use the caller's buffer, else a per-device scratch one
  double* fac = factor;
  if (!fac && enh && out) {
    fac = (double*)scratch(kSlotTmp, sizeof(double) * B, st);
    if (!fac) return (int)hipErrorOutOfMemory;
  }
  // UPR_MS_ROWS=0: the tiled single pass (ms_sums3_kernel); 1: the three-plane
  // register-streaming walk (ms_rows_kernel); default 2: one plane per wave (A/B)
  static const int rows = [] { const char* e = getenv("UPR_MS_ROWS"); return e ? atoi(e) : 2; }();
  if (rows == 2 && H % 4 == 0 && W % 4 == 0 && (uintptr_t)x % (dtype == kF16 ? 8 : 16) == 0) {
    const int strips = (W + 255) / 256, nwav = strips * ((H + MSR_BH - 1) / MSR_BH);
    double* part = (double*)scratch(kSlotMs, (size_t)B * 3 * nwav * 6 * sizeof(double), st);
    if (!part) return (int)hipErrorOutOfMemory;
    // (bands of 20 / 24 / 32 rows measured the same within noise, profiles/r6_ms_rows1_ab.txt)
    const int nblk = (B * 3 * nwav + 3) / 4;
    if (dtype == kF16)
      hipLaunchKernelGGL((ms_rows1_kernel<half_t, MSR_BH>), dim3(nblk), dim3(256), 0, st, (const half_t*)x, part, B,
                         H, W, strips, nwav);
    else
      hipLaunchKernelGGL((ms_rows1_kernel<float, MSR_BH>), dim3(nblk), dim3(256), 0, st, (const float*)x, part, B, H,
                         W, strips, nwav);
    UPR_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(ms_fin1_kernel, dim3(B), dim3(256), 0, st, (const double*)part, nwav, sums, fac, n0, n1, n2);
    UPR_CHECK_HIP(hipGetLastError());
  } else if (rows == 1 && H % 4 == 0 && W % 4 == 0 && (uintptr_t)x % (dtype == kF16 ? 8 : 16) == 0) {
    const int strips = (W + 255) / 256, nwav = strips * ((H + MSR_BH - 1) / MSR_BH);
    double* part = (double*)scratch(kSlotMs, (size_t)B * nwav * 3 * sizeof(double), st);
    if (!part) return (int)hipErrorOutOfMemory;
    const int nblk = (B * nwav + 3) / 4;
    if (dtype == kF16)
      hipLaunchKernelGGL((ms_rows_kernel<half_t>), dim3(nblk), dim3(256), 0, st, (const half_t*)x, part, B, H, W,
                         strips, nwav);
    else
      hipLaunchKernelGGL((ms_rows_kernel<float>), dim3(nblk), dim3(256), 0, st, (const float*)x, part, B, H, W, strips,
                         nwav);
    UPR_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(ms_fin_kernel, dim3(B), dim3(256), 0, st, (const double*)part, nwav, sums, fac, n0, n1, n2);
    UPR_CHECK_HIP(hipGetLastError());
  } else if (H % 4 == 0 && W % 4 == 0 && (uintptr_t)x % (dtype == kF16 ? 8 : 16) == 0) {
    // single pass (ms_sums3_kernel): per-tile partials in a scratch slot,
    // added in order by ms_fin_kernel.  (A streamed form -- 64-column strips
    // walked in 4-row bands through LDS row rings, one band of prefetch --
    // measured 0.281 ms against this kernel's 0.085: too little in flight per
    // block, profiles/r5_ms_strip_vs_tiled.txt)
    const int tx = (W + M3_TW - 1) / M3_TW;
    const int nblk = tx * ((H + M3_TH - 1) / M3_TH);
    double* part = (double*)scratch(kSlotMs, (size_t)B * nblk * 3 * sizeof(double), st);
    if (!part) return (int)hipErrorOutOfMemory;
    if (dtype == kF16)
      hipLaunchKernelGGL((ms_sums3_kernel<half_t>), dim3(nblk, B), dim3(256), 0, st, (const half_t*)x, part, H, W, tx);
    else
      hipLaunchKernelGGL((ms_sums3_kernel<float>), dim3(nblk, B), dim3(256), 0, st, (const float*)x, part, H, W, tx);
    UPR_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(ms_fin_kernel, dim3(B), dim3(256), 0, st, (const double*)part, nblk, sums, fac, n0, n1, n2);
    UPR_CHECK_HIP(hipGetLastError());
  } else {
    UPR_CHECK_HIP(hipMemsetAsync(sums, 0, sizeof(double) * 3 * B, st));
    for (int s = 0; s < 3; ++s) {
      const int tx = (wsz[s] + MS_TW - 1) / MS_TW, ty = (hs[s] + MS_TH - 1) / MS_TH;
      unsigned long long* acc = (unsigned long long*)sums;
      if (dtype == kF16)
        hipLaunchKernelGGL((ms_sums_kernel<half_t>), dim3(tx * ty, B), dim3(256), 0, st, (const half_t*)x, acc, H, W,
                           hs[s], wsz[s], s, tx);
      else
        hipLaunchKernelGGL((ms_sums_kernel<float>), dim3(tx * ty, B), dim3(256), 0, st, (const float*)x, acc, H, W,
                           hs[s], wsz[s], s, tx);
    }
    hipLaunchKernelGGL(ms_factor_kernel, dim3((B + 63) / 64), dim3(64), 0, st, sums, fac, B, n0, n1, n2);
  }
  if (enh && out) {
    const int CHW = 3 * H * W;
    const bool v4 = CHW % 4 == 0 && ((uintptr_t)enh | (uintptr_t)out) % (dtype == kF16 ? 8 : 16) == 0;
    const int per = v4 ? 1024 : 256;
    const int gx = min((CHW + per - 1) / per, 1024);
    if (dtype == kF16) {
      if (v4)
        hipLaunchKernelGGL((scale_clamp_kernel<half_t, 4>), dim3(gx, B), dim3(256), 0, st, (const half_t*)enh,
                           (half_t*)out, (const double*)fac, CHW);
      else
        hipLaunchKernelGGL((scale_clamp_kernel<half_t, 1>), dim3(gx, B), dim3(256), 0, st, (const half_t*)enh,
                           (half_t*)out, (const double*)fac, CHW);
    } else {
      if (v4)
        hipLaunchKernelGGL((scale_clamp_kernel<float, 4>), dim3(gx, B), dim3(256), 0, st, (const float*)enh,
                           (float*)out, (const double*)fac, CHW);
      else
        hipLaunchKernelGGL((scale_clamp_kernel<float, 1>), dim3(gx, B), dim3(256), 0, st, (const float*)enh,
                           (float*)out, (const double*)fac, CHW);
    }
  }
  return (int)hipGetLastError();
}

// Feature maps of one scale: out [B,7,hs,ws] = [img_s (3), luminance, |grad| (3)]
// (MultiScaleEnhancer.extract_multi_scale_features, multi_scale.py:17-60)
template <typename T>
__global__ __launch_bounds__(256) void ms_features_kernel(const T* __restrict__ x, T* __restrict__ out, int B, int H,
                                                          int W, int hs, int ws) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * hs * ws) return;
  const int b = idx / (hs * ws), p = idx - b * hs * ws;
  const int y = p / ws, xx = p - y * ws;
  const T* img = x + (size_t)b * 3 * H * W;
  const float sy = (float)H / (float)hs, sx = (float)W / (float)ws;
  T* o = out + (size_t)b * 7 * hs * ws + p;
  const size_t plane = (size_t)hs * ws;
  float c3[3];
  for (int c = 0; c < 3; ++c) {
    const T* ch = img + (size_t)c * H * W;
    const float v = sample_s(ch, H, W, hs, ws, sy, sx, y, xx);
    c3[c] = v;
    float gx, gy;
    if (ws < 2) gx = 0.f;
    else if (xx == 0) gx = sample_s(ch, H, W, hs, ws, sy, sx, y, 1) - v;
    else if (xx == ws - 1) gx = v - sample_s(ch, H, W, hs, ws, sy, sx, y, ws - 2);
    else gx = (sample_s(ch, H, W, hs, ws, sy, sx, y, xx + 1) - sample_s(ch, H, W, hs, ws, sy, sx, y, xx - 1)) / 2.f;
    if (hs < 2) gy = 0.f;
    else if (y == 0) gy = sample_s(ch, H, W, hs, ws, sy, sx, 1, xx) - v;
    else if (y == hs - 1) gy = v - sample_s(ch, H, W, hs, ws, sy, sx, hs - 2, xx);
    else gy = (sample_s(ch, H, W, hs, ws, sy, sx, y + 1, xx) - sample_s(ch, H, W, hs, ws, sy, sx, y - 1, xx)) / 2.f;
    stf(o, c * plane, v);
    stf(o, (4 + c) * plane, sqrtf(gx * gx + gy * gy));
  }
  stf(o, 3 * plane, 0.299f * c3[0] + 0.587f * c3[1] + 0.114f * c3[2]);
}

int launch_ms_features(const void* x, void* out, int B, int H, int W, int scale_idx, int dtype, hipStream_t st) {
  const double sc = scale_idx == 0 ? 1.0 : (scale_idx == 1 ? 0.5 : 0.25);
  const int hs = scale_idx == 0 ? H : (int)(H * sc), wsz = scale_idx == 0 ? W : (int)(W * sc);
  if (hs < 1 || wsz < 1) return kErrShape;
  const size_t n = (size_t)B * hs * wsz;
  if (dtype == kF16)
    hipLaunchKernelGGL((ms_features_kernel<half_t>), dim3(g1(n)), dim3(256), 0, st, (const half_t*)x, (half_t*)out, B,
                       H, W, hs, wsz);
  else
    hipLaunchKernelGGL((ms_features_kernel<float>), dim3(g1(n)), dim3(256), 0, st, (const float*)x, (float*)out, B,
                       H, W, hs, wsz);
  return (int)hipGetLastError();
}

}  // namespace upr

// ---------------------------------------------------------------------------
// letterbox (utils/letterbox.py:9-102): quantise (float CHW source: the
// reference's (x*255).astype(uint8)), cv2.resize INTER_LINEAR in OpenCV's
// 8-bit fixed point (11-bit coefficients; horizontal pass in int, vertical as
// VResizeLinearVec_32s8u: >>4, two >>16 products, (v+2)>>2), grey border, and
// the output store (float CHW /255 or u8 HWC) -- one thread per output pixel.
// xtab / ytab: [4][n] = source index 0, source index 1, weight 0, weight 1
// (host-built, as OpenCV builds them); NULL when the unpadded size equals the
// source size (no resize).
// ---------------------------------------------------------------------------
namespace upr {

__device__ __forceinline__ int lb_src(const void* src, int kind, int H, int W, int y, int x, int c) {
  if (kind == 0) return ((const uint8_t*)src)[((size_t)y * W + x) * 3 + c];
  return quant_u8(((const float*)src)[((size_t)c * H + y) * W + x]);
}

__global__ __launch_bounds__(256) void letterbox_kernel(const void* __restrict__ src, int src_kind, int H, int W,
                                                        int top, int left, int nh, int nw, int Ho, int Wo,
                                                        const int* __restrict__ xtab, const int* __restrict__ ytab,
                                                        int color, void* __restrict__ out, int out_kind) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= Ho * Wo) return;
  const int y = p / Wo, x = p - y * Wo;
  const int yy = y - top, xx = x - left;
  const bool inside = yy >= 0 && yy < nh && xx >= 0 && xx < nw;
  int v[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (!inside) {
      v[c] = (color >> (8 * c)) & 255;
    } else if (!xtab) {
      v[c] = lb_src(src, src_kind, H, W, yy, xx, c);
    } else {
      const int x0 = xtab[xx], x1 = xtab[nw + xx], a0 = xtab[2 * nw + xx], a1 = xtab[3 * nw + xx];
      const int y0 = ytab[yy], y1 = ytab[nh + yy], b0 = ytab[2 * nh + yy], b1 = ytab[3 * nh + yy];
      const int r0 = (lb_src(src, src_kind, H, W, y0, x0, c) * a0 + lb_src(src, src_kind, H, W, y0, x1, c) * a1) >> 4;
      const int r1 = (lb_src(src, src_kind, H, W, y1, x0, c) * a0 + lb_src(src, src_kind, H, W, y1, x1, c) * a1) >> 4;
      const int s = ((r0 * b0) >> 16) + ((r1 * b1) >> 16);
      v[c] = sat_u8((s + 2) >> 2);
    }
  }
  if (out_kind == 0) {
#pragma unroll
    for (int c = 0; c < 3; ++c) ((float*)out)[(size_t)c * Ho * Wo + p] = (float)v[c] / 255.f;
  } else {
#pragma unroll
    for (int c = 0; c < 3; ++c) ((uint8_t*)out)[(size_t)p * 3 + c] = (uint8_t)v[c];
  }
}

int launch_letterbox(const void* src, int src_kind, int H, int W, int top, int left, int nh, int nw, int Ho, int Wo,
                     const int* xtab, const int* ytab, int color, void* out, int out_kind, hipStream_t st) {
  const int n = Ho * Wo;
  hipLaunchKernelGGL(letterbox_kernel, dim3((n + 255) / 256), dim3(256), 0, st, src, src_kind, H, W, top, left, nh,
                     nw, Ho, Wo, xtab, ytab, color, out, out_kind);
  return (int)hipGetLastError();
}

}  // namespace upr

// ---------------------------------------------------------------------------
// save_image / create_comparison pixels (enhancers/simple_enhance.py:65-132):
// np.clip(x, 0, 1) then (x*255).astype(np.uint8), CHW -> HWC, a 1-channel map
// replicated to RGB.  NaN -> 0 (clip keeps NaN, the cast maps it to 0; here
// the clamp already yields 0 -- same byte).
// ---------------------------------------------------------------------------
namespace upr {

template <typename T>
__global__ __launch_bounds__(256) void to_u8_hwc_kernel(const T* __restrict__ x, int C, size_t HW,
                                                        uint8_t* __restrict__ out) {
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= HW) return;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = ldf(x, (size_t)(C == 1 ? 0 : c) * HW + p);
    out[p * 3 + c] = (uint8_t)quant_u8(fminf(fmaxf(v, 0.f), 1.f));
  }
}

int launch_to_u8_hwc(const void* x, int C, int H, int W, int dtype, uint8_t* out, hipStream_t st) {
  const size_t HW = (size_t)H * W;
  const int grid = (int)((HW + 255) / 256);
  if (dtype == kF16)
    hipLaunchKernelGGL((to_u8_hwc_kernel<half_t>), dim3(grid), dim3(256), 0, st, (const half_t*)x, C, HW, out);
  else
    hipLaunchKernelGGL((to_u8_hwc_kernel<float>), dim3(grid), dim3(256), 0, st, (const float*)x, C, HW, out);
  return (int)hipGetLastError();
}

}  // namespace upr
