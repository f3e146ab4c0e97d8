// Enhancer kernels (gfx950): integer/histogram work, HBM/latency-bound.
//
//  quant_lab      float -> u8 cast exactly as numpy's astype(uint8) on x*255
//                 (trunc, wrap mod 256; NaN/|v|>=2^31 -> 0), then 8-bit sRGB ->
//                 Lab (enhancers/adaptive_params.py:142,145)
//  clahe_lut      per-tile 256-bin LDS histogram, clip + redistribute, CDF -> LUT
//                 (cv2.createCLAHE(2.0,(8,8)).apply, adaptive_params.py:149-152)
//  clahe_lab2rgb  bilinear LUT blend of L, Lab -> sRGB 8-bit, /255 back to float
//                 (adaptive_params.py:155-167)
//  gray_hist      8-bit BGR2GRAY histogram (calculate_brightness_features :45-66)
//  ms_sums        multi-scale feature sums (enhancers/multi_scale.py:17-60, :87-94)
//  scale_clamp    clamp(enh * factor[b], 0, 1)  (multi_scale.py:97-98)
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

// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void quant_lab_kernel(const T* __restrict__ img, const DevLab* __restrict__ tab,
                                                        uint8_t* __restrict__ L, uint8_t* __restrict__ A,
                                                        uint8_t* __restrict__ Bc, int B, int HW) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * HW) return;
  const int b = idx / HW, p = idx - b * HW;
  const T* base = img + (size_t)b * 3 * HW + p;
  const int r = quant_u8(ldf(base, 0)), g = quant_u8(ldf(base, HW)), bl = quant_u8(ldf(base, 2 * HW));
  int l, a, bb;
  rgb2lab_u8(tab, r, g, bl, l, a, bb);
  L[idx] = (uint8_t)l;
  A[idx] = (uint8_t)a;
  Bc[idx] = (uint8_t)bb;
}

// quantise only: NCHW float -> NCHW u8
template <typename T>
__global__ __launch_bounds__(256) void quant_kernel(const T* __restrict__ x, uint8_t* __restrict__ out, size_t n) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < n) out[idx] = (uint8_t)quant_u8(ldf(x, idx));
}

// ---------------------------------------------------------------------------
// CLAHE LUT: one 256-thread block per (image, tile).  Tiles cover the image
// extended by BORDER_REFLECT_101 to a multiple of the tile grid
// (CLAHE_Impl::apply + CLAHE_CalcLut_Body, OpenCV imgproc/src/clahe.cpp).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * (n - 1) - i;
  return i;
}

__global__ __launch_bounds__(256) void clahe_lut_kernel(const uint8_t* __restrict__ L, uint8_t* __restrict__ lut,
                                                        int H, int W, int tilesX, int tilesY, int tileW, int tileH,
                                                        int clipLimit, float lutScale) {
  const int tile = blockIdx.x;
  const int b = blockIdx.y;
  const int tx = tile % tilesX, ty = tile / tilesX;
  __shared__ int hist[256];
  __shared__ int red[256];
  const int t = threadIdx.x;
  hist[t] = 0;
  __syncthreads();
  const uint8_t* img = L + (size_t)b * H * W;
  const int n = tileW * tileH;
  for (int i = t; i < n; i += 256) {
    const int yy = reflect101(ty * tileH + i / tileW, H);
    const int xx = reflect101(tx * tileW + i % tileW, W);
    atomicAdd(&hist[img[(size_t)yy * W + xx]], 1);
  }
  __syncthreads();
  int h = hist[t];
  if (clipLimit > 0) {
    const int ex = h > clipLimit ? h - clipLimit : 0;
    h = h > clipLimit ? clipLimit : h;
    red[t] = ex;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (t < s) red[t] += red[t + s];
      __syncthreads();
    }
    const int clipped = red[0];
    const int redistBatch = clipped / 256;
    const int residual = clipped - redistBatch * 256;
    h += redistBatch;
    if (residual != 0) {
      const int step = max(256 / residual, 1);
      // bins 0, step, 2*step, ... take one each until residual runs out
      if (t % step == 0 && t / step < residual) h += 1;
    }
    __syncthreads();
  }
  // inclusive prefix sum (Hillis-Steele over 256 bins)
  red[t] = h;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const int v = t >= off ? red[t - off] : 0;
    __syncthreads();
    red[t] += v;
    __syncthreads();
  }
  const float v = __fmul_rn((float)red[t], lutScale);
  const int r = __float2int_rn(v);  // saturate_cast<uchar>(float): cvRound then clamp
  lut[((size_t)b * tilesX * tilesY + tile) * 256 + t] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
}

// CLAHE_Interpolation_Body + Lab -> sRGB 8-bit + /255
template <typename T>
__global__ __launch_bounds__(256) void clahe_lab2rgb_kernel(const uint8_t* __restrict__ L, const uint8_t* __restrict__ A,
                                                            const uint8_t* __restrict__ Bc,
                                                            const uint8_t* __restrict__ lut,
                                                            const DevLab* __restrict__ tab, T* __restrict__ out,
                                                            int B, int H, int W, int tilesX, int tilesY, int tileW,
                                                            int tileH) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * H * W) return;
  const int HW = H * W;
  const int b = idx / HW, p = idx - b * HW;
  const int y = p / W, x = p - y * W;
  const float inv_tw = __fdiv_rn(1.0f, (float)tileW);
  const float inv_th = __fdiv_rn(1.0f, (float)tileH);
  const float txf = __fsub_rn(__fmul_rn((float)x, inv_tw), 0.5f);
  int tx1 = (int)floorf(txf);
  int tx2 = tx1 + 1;
  const float xa = __fsub_rn(txf, (float)tx1), xa1 = __fsub_rn(1.0f, xa);
  tx1 = max(tx1, 0);
  tx2 = min(tx2, tilesX - 1);
  const float tyf = __fsub_rn(__fmul_rn((float)y, inv_th), 0.5f);
  int ty1 = (int)floorf(tyf);
  int ty2 = ty1 + 1;
  const float ya = __fsub_rn(tyf, (float)ty1), ya1 = __fsub_rn(1.0f, ya);
  ty1 = max(ty1, 0);
  ty2 = min(ty2, tilesY - 1);
  const uint8_t* lb = lut + (size_t)b * tilesX * tilesY * 256;
  const int v = L[idx];
  const float l11 = lb[(ty1 * tilesX + tx1) * 256 + v], l12 = lb[(ty1 * tilesX + tx2) * 256 + v];
  const float l21 = lb[(ty2 * tilesX + tx1) * 256 + v], l22 = lb[(ty2 * tilesX + tx2) * 256 + v];
  // res = (l11*xa1 + l12*xa)*ya1 + (l21*xa1 + l22*xa)*ya, no contraction
  const float top = __fadd_rn(__fmul_rn(l11, xa1), __fmul_rn(l12, xa));
  const float bot = __fadd_rn(__fmul_rn(l21, xa1), __fmul_rn(l22, xa));
  const float res = __fadd_rn(__fmul_rn(top, ya1), __fmul_rn(bot, ya));
  int lc = __float2int_rn(res);
  lc = lc < 0 ? 0 : (lc > 255 ? 255 : lc);
  int R, G, Bo;
  lab2rgb_u8(tab, lc, A[idx], Bc[idx], R, G, Bo);
  T* o = out + (size_t)b * 3 * HW + p;
  stf(o, 0, __fdiv_rn((float)R, 255.f));
  stf(o, HW, __fdiv_rn((float)G, 255.f));
  stf(o, 2 * (size_t)HW, __fdiv_rn((float)Bo, 255.f));
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

// CLAHE interpolation alone (u8 -> u8), for API/tests
__global__ void clahe_apply_kernel(const uint8_t* __restrict__ L, const uint8_t* __restrict__ lut,
                                   uint8_t* __restrict__ out, int B, int H, int W, int tilesX, int tilesY,
                                   int tileW, int tileH) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * H * W) return;
  const int HW = H * W;
  const int b = idx / HW, p = idx - b * HW;
  const int y = p / W, x = p - y * W;
  const float inv_tw = __fdiv_rn(1.0f, (float)tileW);
  const float inv_th = __fdiv_rn(1.0f, (float)tileH);
  const float txf = __fsub_rn(__fmul_rn((float)x, inv_tw), 0.5f);
  int tx1 = (int)floorf(txf);
  int tx2 = tx1 + 1;
  const float xa = __fsub_rn(txf, (float)tx1), xa1 = __fsub_rn(1.0f, xa);
  tx1 = max(tx1, 0);
  tx2 = min(tx2, tilesX - 1);
  const float tyf = __fsub_rn(__fmul_rn((float)y, inv_th), 0.5f);
  int ty1 = (int)floorf(tyf);
  int ty2 = ty1 + 1;
  const float ya = __fsub_rn(tyf, (float)ty1), ya1 = __fsub_rn(1.0f, ya);
  ty1 = max(ty1, 0);
  ty2 = min(ty2, tilesY - 1);
  const uint8_t* lb = lut + (size_t)b * tilesX * tilesY * 256;
  const int v = L[idx];
  const float l11 = lb[(ty1 * tilesX + tx1) * 256 + v], l12 = lb[(ty1 * tilesX + tx2) * 256 + v];
  const float l21 = lb[(ty2 * tilesX + tx1) * 256 + v], l22 = lb[(ty2 * tilesX + tx2) * 256 + v];
  const float top = __fadd_rn(__fmul_rn(l11, xa1), __fmul_rn(l12, xa));
  const float bot = __fadd_rn(__fmul_rn(l21, xa1), __fmul_rn(l22, xa));
  const float res = __fadd_rn(__fmul_rn(top, ya1), __fmul_rn(bot, ya));
  int lc = __float2int_rn(res);
  out[idx] = (uint8_t)(lc < 0 ? 0 : (lc > 255 ? 255 : lc));
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

template <typename T>
__global__ __launch_bounds__(256) void ms_sums_kernel(const T* __restrict__ x, double* __restrict__ sums, int H, int W,
                                                      int hs, int ws, int scale_idx) {
  const int b = blockIdx.y;
  const T* img = x + (size_t)b * 3 * H * W;
  const float sy = (float)H / (float)hs, sx = (float)W / (float)ws;
  double acc = 0.0;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < hs * ws; p += gridDim.x * blockDim.x) {
    const int y = p / ws, xx = p - y * ws;
    float c3[3];
    float fsum = 0.f;
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
      fsum += v + sqrtf(gx * gx + gy * gy);
    }
    fsum += 0.299f * c3[0] + 0.587f * c3[1] + 0.114f * c3[2];
    acc += (double)fsum;
  }
  // block reduce
  __shared__ double red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(&sums[b * 3 + scale_idx], red[0]);
}

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

__global__ void ms_factor_kernel(const double* __restrict__ sums, double* __restrict__ factor, int B, double n0,
                                 double n1, double n2) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) factor[b] = ms_factor(sums, b, n0, n1, n2);
}

// clamp(enh * float(factor), 0, 1)   (multi_scale.py:317-318)
template <typename T>
__global__ __launch_bounds__(256) void scale_clamp_kernel(const T* __restrict__ enh, T* __restrict__ out,
                                                          const double* __restrict__ sums, double n0, double n1,
                                                          double n2, int CHW, int B) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)B * CHW) return;
  const int b = (int)(idx / CHW);
  const float f = (float)ms_factor(sums, b, n0, n1, n2);
  const float v = __fmul_rn(ldf(enh, idx), f);
  stf(out, idx, fminf(fmaxf(v, 0.f), 1.f));
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
static inline int g1(size_t n) { return (int)((n + 255) / 256); }

struct ClaheGeom {
  int tilesX, tilesY, tileW, tileH, clip;
  float lutScale;
};
static ClaheGeom clahe_geom(int H, int W, float clipLimit, int tilesX, int tilesY) {
  ClaheGeom g;
  g.tilesX = tilesX; g.tilesY = tilesY;
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
  return g;
}

int launch_clahe_pipeline(const void* enh, void* out, uint8_t* ws, int B, int H, int W, float clip, int tilesX,
                          int tilesY, int dtype, hipStream_t st) {
  const DevLab* tab = dev_lab_tables(st);
  if (!tab) return kErrUnsupported;
  const size_t HW = (size_t)H * W;
  uint8_t* L = ws;
  uint8_t* A = L + B * HW;
  uint8_t* Bc = A + B * HW;
  uint8_t* lut = Bc + B * HW;
  const ClaheGeom g = clahe_geom(H, W, clip, tilesX, tilesY);
  const int n = (int)(B * HW);
  if (dtype == kF16)
    hipLaunchKernelGGL((quant_lab_kernel<half_t>), dim3(g1(n)), dim3(256), 0, st, (const half_t*)enh, tab, L, A, Bc, B,
                       (int)HW);
  else
    hipLaunchKernelGGL((quant_lab_kernel<float>), dim3(g1(n)), dim3(256), 0, st, (const float*)enh, tab, L, A, Bc, B,
                       (int)HW);
  hipLaunchKernelGGL(clahe_lut_kernel, dim3(tilesX * tilesY, B), dim3(256), 0, st, L, lut, H, W, tilesX, tilesY,
                     g.tileW, g.tileH, g.clip, g.lutScale);
  if (dtype == kF16)
    hipLaunchKernelGGL((clahe_lab2rgb_kernel<half_t>), dim3(g1(n)), dim3(256), 0, st, L, A, Bc, lut, tab,
                       (half_t*)out, B, H, W, tilesX, tilesY, g.tileW, g.tileH);
  else
    hipLaunchKernelGGL((clahe_lab2rgb_kernel<float>), dim3(g1(n)), dim3(256), 0, st, L, A, Bc, lut, tab,
                       (float*)out, B, H, W, tilesX, tilesY, g.tileW, g.tileH);
  return (int)hipGetLastError();
}

size_t clahe_pipeline_ws(int B, int H, int W, int tilesX, int tilesY) {
  return (size_t)B * H * W * 3 + (size_t)B * tilesX * tilesY * 256;
}

int launch_clahe_u8(const uint8_t* src, uint8_t* dst, uint8_t* lut, int B, int H, int W, float clip, int tilesX,
                    int tilesY, hipStream_t st) {
  const ClaheGeom g = clahe_geom(H, W, clip, tilesX, tilesY);
  hipLaunchKernelGGL(clahe_lut_kernel, dim3(tilesX * tilesY, B), dim3(256), 0, st, src, lut, H, W, tilesX, tilesY,
                     g.tileW, g.tileH, g.clip, g.lutScale);
  hipLaunchKernelGGL(clahe_apply_kernel, dim3(g1((size_t)B * H * W)), dim3(256), 0, st, src, lut, dst, B, H, W,
                     tilesX, tilesY, g.tileW, g.tileH);
  return (int)hipGetLastError();
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
  UPR_CHECK_HIP(hipMemsetAsync(sums, 0, sizeof(double) * 3 * B, st));
  const int hs[3] = {H, (int)(H * 0.5), (int)(H * 0.25)};
  const int wsz[3] = {W, (int)(W * 0.5), (int)(W * 0.25)};
  for (int s = 0; s < 3; ++s) {
    if (hs[s] < 1 || wsz[s] < 1) return kErrShape;
    const int gx = min(g1((size_t)hs[s] * wsz[s]), 512);
    if (dtype == kF16)
      hipLaunchKernelGGL((ms_sums_kernel<half_t>), dim3(gx, B), dim3(256), 0, st, (const half_t*)x, sums, H, W, hs[s],
                         wsz[s], s);
    else
      hipLaunchKernelGGL((ms_sums_kernel<float>), dim3(gx, B), dim3(256), 0, st, (const float*)x, sums, H, W, hs[s],
                         wsz[s], s);
  }
  const double n0 = 7.0 * hs[0] * wsz[0], n1 = 7.0 * hs[1] * wsz[1], n2 = 7.0 * hs[2] * wsz[2];
  if (factor)
    hipLaunchKernelGGL(ms_factor_kernel, dim3((B + 63) / 64), dim3(64), 0, st, (const double*)sums, factor, B, n0, n1,
                       n2);
  if (enh && out) {
    const size_t n = (size_t)B * 3 * H * W;
    if (dtype == kF16)
      hipLaunchKernelGGL((scale_clamp_kernel<half_t>), dim3(g1(n)), dim3(256), 0, st, (const half_t*)enh,
                         (half_t*)out, sums, n0, n1, n2, 3 * H * W, B);
    else
      hipLaunchKernelGGL((scale_clamp_kernel<float>), dim3(g1(n)), dim3(256), 0, st, (const float*)enh, (float*)out,
                         sums, n0, n1, n2, 3 * H * W, B);
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
