// Training kernels for gfx950: the backward pass of MultiScaleUP_Retinex, the
// TotalLoss terms with their gradients, and the clip + Adam optimiser step
// (reference trainers/train.py:63-103, losses/loss.py:12-753, models/model.py).
// Contract of every entry: include/upr_train.h.
//
// Layout: activations are addressed through UprView strides (NCHW inputs,
// NHWC activations, channel slices of concat buffers).  Everything computes in
// fp32; per-channel / per-image reductions accumulate in fp64 (block partials
// in registers + LDS, one fp64 atomic per block and channel).
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <mutex>
#include <thread>

#include "upr_common.h"
#include "../../include/upr.h"
#include "../../include/upr_train.h"

namespace upr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct V {
  float* d;
  long long sb, sh, sw, sc;
  __device__ __forceinline__ long long at(int b, int y, int x, int c) const {
    return b * sb + y * sh + x * sw + c * sc;
  }
};

static V mkv(const UprView* u) {
  V v;
  v.d = (float*)u->data;
  v.sb = u->sb; v.sh = u->sh; v.sw = u->sw; v.sc = u->sc;
  return v;
}

// channel-contiguous view with 32-bit strides: the 4-channels-per-thread
// resampling / copy kernels (the generic V kernels' 64-bit div/mod per element
// run below 1 TB/s)
struct V4 {
  float* d;
  int sb, sh, sw;
  __device__ __forceinline__ float* at(int b, int y, int x, int c) const { return d + b * sb + y * sh + x * sw + c; }
};

// usable as a V4 over [B, H, W, C]: unit channel stride, C and the strides
// multiples of 4, 16-byte aligned, every offset below 2^31
static bool vec4_view_ok(const UprView* v, int B, int H, int W, int C) {
  if (v->sc != 1 || C % 4 || (uintptr_t)v->data % 16 || v->sw % 4 || v->sh % 4 || v->sb % 4) return false;
  if ((long long)B * H * W * C >= (1LL << 31)) return false;
  const long long ext = (long long)(B - 1) * v->sb + (long long)(H - 1) * v->sh + (long long)(W - 1) * v->sw + C;
  return ext < (1LL << 31) && v->sb < (1LL << 31) && v->sh < (1LL << 31) && v->sw < (1LL << 31);
}

// 4 consecutive channels as floats, from fp32 or an fp16 copy
__device__ __forceinline__ float4 ld4f(const float* p) { return *(const float4*)p; }
__device__ __forceinline__ float4 ld4f(const half_t* p) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const h4 v = *(const h4*)p;
  return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}

static V4 mkv4(const UprView* u) {
  V4 v;
  v.d = (float*)u->data;
  v.sb = (int)u->sb; v.sh = (int)u->sh; v.sw = (int)u->sw;
  return v;
}

static inline int grid_for(long long n, int per = 256, int cap = 65536) {
  long long g = (n + per - 1) / per;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

#define GSTRIDE(i, n) for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (n); \
                           i += (long long)gridDim.x * blockDim.x)

#define LAUNCH_CHECK() return (int)hipGetLastError()

// train_small.hip: pixel-tiled / MFMA forms of the small-channel convs
int small_conv_fwd(const UprView* xv, int B, int H, int W, int Cin, const float* w, const float* bias, int Cout,
                   int kh, int kw, int stride, int pad, int dil, const UprView* yv, int Ho, int Wo, int relu,
                   int accumulate, hipStream_t st, void* y16 = nullptr, int skip32 = 0);
int small_stem_wgrad_relu16(const UprView* xv, const float* dy, const void* y16, int B, int H, int W, float* dw,
                            float* dbias, hipStream_t st);
int small_conv_dgrad(const UprView* dyv, int Ho, int Wo, const float* w, int B, int H, int W, int Cin, int Cout,
                     int kh, int kw, int stride, int pad, int dil, const UprView* dxv, int accumulate, hipStream_t st);
int small_conv_dgrad_c3_16(const void* dy16, int B, int H, int W, const float* w, int Cout, const UprView* dxv,
                           int accumulate, hipStream_t st);
int small_conv_wgrad(const UprView* xv, const UprView* dyv, int B, int H, int W, int Cin, int Ho, int Wo, int Cout,
                     int kh, int kw, int stride, int pad, int dil, float* dw, float* dbias, hipStream_t st,
                     const UprView* ymask = nullptr);
// train_wgrad.hip: split-K GEMM weight gradient (the conv_wgrad_kernel below takes the shapes it does not)
int wgrad_gemm(const float* x, int B, int H, int W, int Cin, int x_cs, int x_coff, const float* dy, int Ho, int Wo,
               int Cout, int dy_cs, int dy_coff, int kh, int kw, int stride, int pad, int dil, float* dwp,
               hipStream_t st, int torch_ci = 0);
int wgrad16_gemm(const void* x16, int B, int H, int W, int Cin, const float* dy, int Ho, int Wo, int Cout, int dy_cs,
                 int dy_coff, int kh, int kw, int stride, int pad, int dil, float* dwp, hipStream_t st,
                 int torch_ci = 0, const void* dy16 = nullptr);

// scratch(): see upr_common.h
void* scratch(int slot, size_t bytes, hipStream_t st, bool* fresh) {
  struct Entry {
    int dev;
    hipStream_t st;
    void* p[kSlotCount];
    size_t n[kSlotCount];
    std::thread::id owner;     // the one thread that used the entry (unless shared)
    bool shared;               // used by more than one thread: never reclaimed
    unsigned long long tick;   // last use (LRU)
  };
  static std::mutex mu;
  static Entry tab[kScratchStreams];
  static int used = 0;
  static unsigned long long clock = 0;
  if (fresh) *fresh = false;
  if (slot < 0 || slot >= kSlotCount) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  const std::thread::id me = std::this_thread::get_id();
  std::lock_guard<std::mutex> lock(mu);
  Entry* e = nullptr;
  for (int i = 0; i < used; ++i)
    if (tab[i].dev == dev && tab[i].st == st) e = &tab[i];
  if (!e) {
    if (used < kScratchStreams) {
      e = &tab[used++];
    } else {
      // full: reclaim the least recently used entry that only THIS thread
      // ever used.  Its buffers went out only in this thread's earlier calls,
      // which returned after enqueueing their launches, so once the device is
      // idle nobody reads them (another thread's entries may be mid-call:
      // their pointers can still be waiting for a launch, so they are never
      // taken).  The device synchronise is not allowed while the caller's
      // stream is being captured: then the call fails as before.
      Entry* v = nullptr;
      for (int i = 0; i < used; ++i)
        if (!tab[i].shared && tab[i].owner == me && tab[i].dev == dev && (!v || tab[i].tick < v->tick)) v = &tab[i];
      hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
      if (!v || hipStreamIsCapturing(st, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) {
        (void)hipGetLastError();
        return nullptr;
      }
      if (hipDeviceSynchronize() != hipSuccess) return nullptr;
      for (int k = 0; k < kSlotCount; ++k)
        if (v->p[k]) (void)hipFree(v->p[k]);
      e = v;
    }
    *e = Entry{};
    e->dev = dev;
    e->st = st;
    e->owner = me;
  } else if (e->owner != me) {
    e->shared = true;
  }
  e->tick = ++clock;
  if (bytes == 0) bytes = 16;
  if (e->n[slot] < bytes) {
    if (e->p[slot]) {
      if (hipStreamSynchronize(st) != hipSuccess) return nullptr;  // earlier kernels may still read it
      (void)hipFree(e->p[slot]);
      e->p[slot] = nullptr;
      e->n[slot] = 0;
    }
    const size_t grow = bytes + bytes / 4;  // headroom: one growth covers nearby sizes
    if (hipMalloc(&e->p[slot], grow) != hipSuccess) {
      (void)hipGetLastError();
      e->p[slot] = nullptr;
      return nullptr;
    }
    e->n[slot] = grow;
    if (fresh) *fresh = true;
  }
  return e->p[slot];
}

// ---------------------------------------------------------------------------
// Direct convolution (small channel counts): forward / dgrad / wgrad
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_direct_kernel(V x, int B, int H, int W, int Cin, const float* __restrict__ w,
                                                          const float* __restrict__ bias, int Cout, int kh, int kw,
                                                          int s, int p, int d, V y, int Ho, int Wo, int relu,
                                                          int accum) {
  const long long n = (long long)B * Ho * Wo * Cout;
  GSTRIDE(i, n) {
    const int co = (int)(i % Cout);
    long long r = i / Cout;
    const int ox = (int)(r % Wo); r /= Wo;
    const int oy = (int)(r % Ho);
    const int b = (int)(r / Ho);
    float a = bias ? bias[co] : 0.f;
    const float* wc = w + (size_t)co * Cin * kh * kw;
    for (int ci = 0; ci < Cin; ++ci) {
      for (int ky = 0; ky < kh; ++ky) {
        const int iy = oy * s - p + ky * d;
        if (iy < 0 || iy >= H) continue;
        for (int kx = 0; kx < kw; ++kx) {
          const int ix = ox * s - p + kx * d;
          if (ix < 0 || ix >= W) continue;
          a = fmaf(x.d[x.at(b, iy, ix, ci)], wc[(ci * kh + ky) * kw + kx], a);
        }
      }
    }
    float* yp = y.d + y.at(b, oy, ox, co);
    if (accum) a += *yp;
    if (relu) a = fmaxf(a, 0.f);
    *yp = a;
  }
}

// 3-input-channel 3x3 stride-1 dilation-1 form (the input layers 3->32 and
// VGG-19 conv1_1 3->64 at full resolution): compile-time tap loops, the 27
// weights in registers, one base pointer per tap row -- the generic kernel's
// per-access 64-bit four-stride index arithmetic dominated its time
__global__ __launch_bounds__(256) void conv_direct_c3k3_kernel(V x, int B, int H, int W, const float* __restrict__ w,
                                                               const float* __restrict__ bias, int Cout, int p, V y,
                                                               int Ho, int Wo, int relu, int accum) {
  const long long n = (long long)B * Ho * Wo * Cout;
  GSTRIDE(i, n) {
    const int co = (int)(i % Cout);
    long long r = i / Cout;
    const int ox = (int)(r % Wo); r /= Wo;
    const int oy = (int)(r % Ho);
    const int b = (int)(r / Ho);
    const float* wc = w + (size_t)co * 27;
    float a = bias ? bias[co] : 0.f;
    // same accumulation order as conv_direct_kernel: ci outer, then ky, kx
#pragma unroll
    for (int ci = 0; ci < 3; ++ci) {
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int iy = oy - p + ky;
        if (iy < 0 || iy >= H) continue;
        const float* row = x.d + b * x.sb + iy * x.sh + ci * x.sc;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int ix = ox - p + kx;
          if (ix < 0 || ix >= W) continue;
          a = fmaf(row[ix * x.sw], wc[(ci * 3 + ky) * 3 + kx], a);
        }
      }
    }
    float* yp = y.d + y.at(b, oy, ox, co);
    if (accum) a += *yp;
    if (relu) a = fmaxf(a, 0.f);
    *yp = a;
  }
}

__global__ __launch_bounds__(256) void conv_direct_dgrad_kernel(V dy, int Ho, int Wo, const float* __restrict__ w,
                                                                int B, int H, int W, int Cin, int Cout, int kh,
                                                                int kw, int s, int p, int d, V dx, int accum) {
  const long long n = (long long)B * H * W * Cin;
  GSTRIDE(i, n) {
    const int ci = (int)(i % Cin);
    long long r = i / Cin;
    const int ix = (int)(r % W); r /= W;
    const int iy = (int)(r % H);
    const int b = (int)(r / H);
    float a = 0.f;
    for (int ky = 0; ky < kh; ++ky) {
      const int yn = iy + p - ky * d;
      if (yn < 0 || yn % s) continue;
      const int oy = yn / s;
      if (oy >= Ho) continue;
      for (int kx = 0; kx < kw; ++kx) {
        const int xn = ix + p - kx * d;
        if (xn < 0 || xn % s) continue;
        const int ox = xn / s;
        if (ox >= Wo) continue;
        for (int co = 0; co < Cout; ++co)
          a = fmaf(dy.d[dy.at(b, oy, ox, co)], w[(((size_t)co * Cin + ci) * kh + ky) * kw + kx], a);
      }
    }
    float* xp = dx.d + dx.at(b, iy, ix, ci);
    if (accum) a += *xp;
    *xp = a;
  }
}

// Weight gradient of a small conv: a chunk of CH output pixels is staged in
// LDS as dy[CH][Cout] and its im2col rows col[CH][taps*Cin]; each thread owns
// weight entries (co, ci, tap) (+ a bias entry) and sums over the chunk.
// Blocks loop over chunks (grid-stride) and issue their atomics once.
__global__ __launch_bounds__(256) void conv_direct_wgrad_kernel(V x, V dy, int B, int H, int W, int Cin, int Ho,
                                                                int Wo, int Cout, int kh, int kw, int s, int p,
                                                                int d, int CH, float* __restrict__ dw,
                                                                float* __restrict__ dbias) {
  extern __shared__ float sm[];
  const int taps = kh * kw;
  const int KC = taps * Cin;
  float* sdy = sm;              // [CH][Cout]
  float* scol = sm + CH * Cout;  // [CH][KC]
  const long long P = (long long)B * Ho * Wo;
  const int nW = Cout * KC;
  const int nE = nW + (dbias ? Cout : 0);
  constexpr int MAXE = 16;
  float acc[MAXE];
#pragma unroll
  for (int k = 0; k < MAXE; ++k) acc[k] = 0.f;
  for (long long c0 = (long long)blockIdx.x * CH; c0 < P; c0 += (long long)gridDim.x * CH) {
    __syncthreads();
    for (int t = threadIdx.x; t < CH * Cout; t += blockDim.x) {
      const int pp = t / Cout, co = t - pp * Cout;
      const long long pix = c0 + pp;
      float v = 0.f;
      if (pix < P) {
        const int ox = (int)(pix % Wo);
        const long long r = pix / Wo;
        const int oy = (int)(r % Ho), b = (int)(r / Ho);
        v = dy.d[dy.at(b, oy, ox, co)];
      }
      sdy[t] = v;
    }
    for (int t = threadIdx.x; t < CH * KC; t += blockDim.x) {
      const int pp = t / KC, k = t - pp * KC;
      const int tap = k / Cin, ci = k - tap * Cin;
      const int ky = tap / kw, kx = tap - ky * kw;
      const long long pix = c0 + pp;
      float v = 0.f;
      if (pix < P) {
        const int ox = (int)(pix % Wo);
        const long long r = pix / Wo;
        const int oy = (int)(r % Ho), b = (int)(r / Ho);
        const int iy = oy * s - p + ky * d, ix = ox * s - p + kx * d;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) v = x.d[x.at(b, iy, ix, ci)];
      }
      scol[t] = v;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MAXE; ++k) {
      const int e = threadIdx.x + k * 256;
      if (e >= nE) break;
      float a = acc[k];
      if (e < nW) {
        const int co = e / KC, kk = e - co * KC;
        for (int pp = 0; pp < CH; ++pp) a = fmaf(sdy[pp * Cout + co], scol[pp * KC + kk], a);
      } else {
        const int co = e - nW;
        for (int pp = 0; pp < CH; ++pp) a += sdy[pp * Cout + co];
      }
      acc[k] = a;
    }
  }
#pragma unroll
  for (int k = 0; k < MAXE; ++k) {
    const int e = threadIdx.x + k * 256;
    if (e >= nE) break;
    if (e < nW) {
      // e = co*KC + tap*Cin + ci -> PyTorch [co][ci][ky][kx]
      const int co = e / KC, kk = e - co * KC;
      const int tap = kk / Cin, ci = kk - tap * Cin;
      atomicAdd(dw + ((size_t)co * Cin + ci) * taps + tap, acc[k]);
    } else {
      atomicAdd(dbias + (e - nW), acc[k]);
    }
  }
}

// ---------------------------------------------------------------------------
// MFMA weight gradient (C % 32 == 0): block tile 32 co x 32 ci of one tap,
// 4 waves each summing interleaved groups of 4 pixels with
// v_mfma_f32_16x16x4_f32 (A = dy[p][co], B = x[window(p)][ci], k = pixel).
// ---------------------------------------------------------------------------
constexpr int WG_PPB = 1024;  // pixels per block

__global__ __launch_bounds__(256) void conv_wgrad_kernel(const float* __restrict__ x, int B, int H, int W, int Cin,
                                                         int x_cs, int x_coff, const float* __restrict__ dy, int Ho,
                                                         int Wo, int Cout, int dy_cs, int dy_coff, int kh, int kw,
                                                         int s, int p, int d, float* __restrict__ dwp) {
  __shared__ float red[4][32 * 32];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int co0 = blockIdx.y * 32;
  const int cblocks = Cin / 32;
  const int tap = blockIdx.z / cblocks;
  const int ci0 = (blockIdx.z - tap * cblocks) * 32;
  const int ky = tap / kw, kx = tap - ky * kw;
  const long long P = (long long)B * Ho * Wo;
  const long long p0 = (long long)blockIdx.x * WG_PPB;
  const int kk = lane >> 4, r = lane & 15;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int g = wave; g < WG_PPB / 4; g += 4) {
    const long long pix = p0 + g * 4 + kk;
    float a0 = 0.f, a1 = 0.f, b0 = 0.f, b1 = 0.f;
    if (pix < P) {
      const float* dp = dy + pix * dy_cs + dy_coff + co0 + r;
      a0 = dp[0];
      a1 = dp[16];
      const int ox = (int)(pix % Wo);
      const long long rr = pix / Wo;
      const int oy = (int)(rr % Ho), b = (int)(rr / Ho);
      const int iy = oy * s - p + ky * d, ix = ox * s - p + kx * d;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
        const float* xp = x + (((long long)b * H + iy) * W + ix) * x_cs + x_coff + ci0 + r;
        b0 = xp[0];
        b1 = xp[16];
      }
    }
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
  }
  // C[row][col]: lane holds rows 4*(lane>>4)+q, col lane&15 of each 16x16 tile
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = i * 16 + kk * 4 + q, col = j * 16 + r;
        red[wave][row * 32 + col] = acc[i][j][q];
      }
  __syncthreads();
  const int KT = kh * kw * Cin;
  for (int e = threadIdx.x; e < 1024; e += 256) {
    const float v = red[0][e] + red[1][e] + red[2][e] + red[3][e];
    const int row = e >> 5, col = e & 31;
    atomicAdd(dwp + (size_t)(co0 + row) * KT + tap * Cin + ci0 + col, v);
  }
}

// ---------------------------------------------------------------------------
// weight layout transforms
// ---------------------------------------------------------------------------
__global__ void pack_weight_kernel(const float* __restrict__ w, float* __restrict__ o, int Co, int Ci, int kh, int kw,
                                   int mode) {
  const int taps = kh * kw;
  const long long n = (long long)Co * Ci * taps;
  GSTRIDE(i, n) {
    // i enumerates the SOURCE layout
    if (mode == 0 || mode == 1) {
      const int tap = (int)(i % taps);
      const long long r = i / taps;
      const int ci = (int)(r % Ci), co = (int)(r / Ci);
      if (mode == 0) {
        o[((size_t)co * taps + tap) * Ci + ci] = w[i];
      } else {
        const int ft = taps - 1 - tap;  // (kh-1-ky, kw-1-kx)
        o[((size_t)ci * taps + ft) * Co + co] = w[i];
      }
    } else {
      // ConvTranspose weight [Ci][Co][2][2] with Co, Ci as named in the call
      // (Ci = in_channels, Co = out_channels), q = a*2+b
      const int q = (int)(i % 4);
      const long long r = i / 4;
      const int co = (int)(r % Co), ci = (int)(r / Co);
      if (mode == 2) o[((size_t)q * Co + co) * Ci + ci] = w[i];
      else o[((size_t)ci * 4 + q) * Co + co] = w[i];
    }
  }
}

__global__ __launch_bounds__(256) void pack_batch_kernel(const UprPackJob* __restrict__ jobs) {
  const UprPackJob j = jobs[blockIdx.y];
  const int taps = j.kh * j.kw;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < j.n; i += gridDim.x * 256) {
    const float v = j.w[i];
    if (j.mode == 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (j.out32) j.out32[q * j.Co + i] = v;
        if (j.out16) ((half_t*)j.out16)[q * j.Co + i] = (half_t)v;
      }
      continue;
    }
    int dst;
    if (j.mode <= 1) {
      const int tap = i % taps, r = i / taps;
      const int ci = r % j.Ci, co = r / j.Ci;
      dst = j.mode == 0 ? (co * taps + tap) * j.Ci + ci : (ci * taps + (taps - 1 - tap)) * j.Co + co;
    } else {
      const int q = i % 4, r = i / 4;
      const int co = r % j.Co, ci = r / j.Co;
      dst = j.mode == 2 ? (q * j.Co + co) * j.Ci + ci : (ci * 4 + q) * j.Co + co;
    }
    if (j.out32) j.out32[dst] = v;
    if (j.out16) ((half_t*)j.out16)[dst] = (half_t)v;
  }
}

__global__ void unpack_grad_kernel(const float* __restrict__ gp, float* __restrict__ g, int Co, int Ci, int kh, int kw,
                                   int mode, int accum) {
  const int taps = kh * kw;
  const long long n = (long long)Co * Ci * taps;
  GSTRIDE(i, n) {
    float v;
    if (mode == 0) {
      const int tap = (int)(i % taps);
      const long long r = i / taps;
      const int ci = (int)(r % Ci), co = (int)(r / Ci);
      v = gp[((size_t)co * taps + tap) * Ci + ci];
    } else {
      const int q = (int)(i % 4);
      const long long r = i / 4;
      const int co = (int)(r % Co), ci = (int)(r / Co);
      v = gp[((size_t)ci * 4 + q) * Co + co];
    }
    g[i] = accum ? g[i] + v : v;
  }
}

__global__ void zero_upsample_kernel(const float* __restrict__ dy, int B, int Ho, int Wo, int C, int cs, int coff,
                                     float* __restrict__ z) {
  const long long n = (long long)B * 2 * Ho * 2 * Wo * C;
  GSTRIDE(i, n) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int X = (int)(r % (2 * Wo)); r /= 2 * Wo;
    const int Y = (int)(r % (2 * Ho));
    const int b = (int)(r / (2 * Ho));
    float v = 0.f;
    if (!(X & 1) && !(Y & 1)) v = dy[(((long long)b * Ho + (Y >> 1)) * Wo + (X >> 1)) * cs + coff + c];
    z[i] = v;
  }
}

// fp16 form for the autocast stride-2 input gradient: dy (fp32) rounded to
// fp16 as the conv's cast would, zero-upsampled, 8 channels per thread
// from the gradient's compact fp16 copy (dy16 [B][Ho][Wo][C]): 16-byte copies
__global__ __launch_bounds__(256) void zero_upsample16h_kernel(const half_t* __restrict__ dy16, int B, int Ho, int Wo,
                                                               int C, half_t* __restrict__ z, long long n) {
  const int C8 = C / 8;
  GSTRIDE(i, n) {
    const int c = (int)(i % C8) * 8;
    long long r = i / C8;
    const int X = (int)(r % (2 * Wo)); r /= 2 * Wo;
    const int Y = (int)(r % (2 * Ho));
    const int b = (int)(r / (2 * Ho));
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (!(X & 1) && !(Y & 1)) v = *(const uint4*)(dy16 + (((long long)b * Ho + (Y >> 1)) * Wo + (X >> 1)) * C + c);
    *(uint4*)(z + i * 8) = v;
  }
}

__global__ __launch_bounds__(256) void zero_upsample16_kernel(const float* __restrict__ dy, int B, int Ho, int Wo,
                                                              int C, int cs, int coff, half_t* __restrict__ z) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  const int C8 = C / 8;
  const long long n = (long long)B * 2 * Ho * 2 * Wo * C8;
  GSTRIDE(i, n) {
    const int c = (int)(i % C8) * 8;
    long long r = i / C8;
    const int X = (int)(r % (2 * Wo)); r /= 2 * Wo;
    const int Y = (int)(r % (2 * Ho));
    const int b = (int)(r / (2 * Ho));
    h8 v = h8{};
    if (!(X & 1) && !(Y & 1)) {
      const float* src = dy + (((long long)b * Ho + (Y >> 1)) * Wo + (X >> 1)) * cs + coff + c;
      const float4 lo = *(const float4*)src, hi = *(const float4*)(src + 4);
      v = h8{(half_t)lo.x, (half_t)lo.y, (half_t)lo.z, (half_t)lo.w, (half_t)hi.x, (half_t)hi.y, (half_t)hi.z,
             (half_t)hi.w};
    }
    *(h8*)(z + i * 8) = v;
  }
}

// ---------------------------------------------------------------------------
// per-channel reductions over M rows: mode 0 (x, x^2), mode 1 (g, g*xhat),
// mode 2 (g) -> float out via atomics
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void chan_reduce_kernel(const float* __restrict__ a, int a_cs, int a_coff,
                                                          const float* __restrict__ x, int x_cs, int x_coff,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, int M, int C, int mode,
                                                          double* __restrict__ acc, float* __restrict__ fout) {
  __shared__ double s1[256], s2[256];
  const int rows_per_block = (M + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  for (int cb = 0; cb < C; cb += 256) {
    const int cw = min(256, C - cb);
    const int R = 256 / cw;
    const int c = threadIdx.x % cw, rg = threadIdx.x / cw;
    double u = 0.0, v = 0.0;
    if (rg < R) {
      const int cc = cb + c;
      float mu = 0.f, is = 0.f;
      if (mode == 1) { mu = mean[cc]; is = invstd[cc]; }
      for (int r = r0 + rg; r < r1; r += R) {
        const float av = a[(size_t)r * a_cs + a_coff + cc];
        if (mode == 0) { u += av; v += (double)av * av; }
        else if (mode == 1) { u += av; v += (double)av * ((x[(size_t)r * x_cs + x_coff + cc] - mu) * is); }
        else u += av;
      }
    }
    s1[threadIdx.x] = u;
    s2[threadIdx.x] = v;
    __syncthreads();
    if (threadIdx.x < cw) {
      double t1 = 0.0, t2 = 0.0;
      for (int k = 0; k < R; ++k) { t1 += s1[k * cw + threadIdx.x]; t2 += s2[k * cw + threadIdx.x]; }
      const int cc = cb + threadIdx.x;
      if (mode == 2) atomicAdd(fout + cc, (float)t1);
      else { atomicAdd(acc + cc, t1); atomicAdd(acc + C + cc, t2); }
    }
    __syncthreads();
  }
}

static int reduce_grid(int M) { return grid_for(M, 512, 2048); }

// float4 form of chan_reduce_kernel (C % 4 == 0, C <= 1024, 16-byte aligned
// rows): a thread owns 4 consecutive channels, so a wave reads whole 16-byte
// chunks of 64 / (C/4) rows per instruction (same per-channel fp64 sums)
// y = bn(x) of the forward (bn_apply kernels) and of the ReLU-mask recompute
// in the fused backward: ONE expression, so the recomputed sign is the
// forward's bit for bit
__device__ __forceinline__ float bn_affine(float x, float mean, float invstd, float gamma, float beta) {
  return __builtin_fmaf((x - mean) * invstd, gamma, beta);
}

__global__ __launch_bounds__(256) void chan_reduce4_kernel(const float* __restrict__ a, int a_cs, int a_coff,
                                                           const float* __restrict__ x, int x_cs, int x_coff,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd, int M, int C, int mode,
                                                           double* __restrict__ acc, float* __restrict__ fout,
                                                           const float* __restrict__ gamma = nullptr,
                                                           const float* __restrict__ beta = nullptr) {
  // mode 3: mode 1 with the consumer ReLU folded in (g counts where bn(x) > 0)
  __shared__ double s1[256 * 4], s2[256 * 4];
  const int rows_per_block = (M + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  const int C4 = C >> 2;
  const int R = 256 / C4;
  const int q = threadIdx.x % C4, rg = threadIdx.x / C4;
  double u[4] = {0.0, 0.0, 0.0, 0.0}, v[4] = {0.0, 0.0, 0.0, 0.0};
  if (rg < R) {
    float4 mu = make_float4(0.f, 0.f, 0.f, 0.f), is = mu, ga = mu, be = mu;
    if (mode == 1 || mode == 3) { mu = ((const float4*)mean)[q]; is = ((const float4*)invstd)[q]; }
    if (mode == 3) { ga = ((const float4*)gamma)[q]; be = ((const float4*)beta)[q]; }
    auto acc_row = [&](const float4 av, const float4 xv) {
      float ae[4] = {av.x, av.y, av.z, av.w};
      if (mode == 1 || mode == 3) {
        const float xe[4] = {xv.x, xv.y, xv.z, xv.w};
        const float mue[4] = {mu.x, mu.y, mu.z, mu.w}, ise[4] = {is.x, is.y, is.z, is.w};
        const float gae[4] = {ga.x, ga.y, ga.z, ga.w}, bee[4] = {be.x, be.y, be.z, be.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (mode == 3 && !(bn_affine(xe[e], mue[e], ise[e], gae[e], bee[e]) > 0.f)) ae[e] = 0.f;
          const float xh = (xe[e] - mue[e]) * ise[e];
          u[e] += ae[e];
          v[e] += (double)ae[e] * xh;
        }
      } else if (mode == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) { u[e] += ae[e]; v[e] += (double)ae[e] * ae[e]; }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] += ae[e];
      }
    };
    // four rows' loads issued before any is consumed (a single dependent load
    // per iteration left the reduction latency-bound at ~1.2 TB/s)
    const float* ap = a + a_coff + 4 * q;
    const float* xp = x ? x + x_coff + 4 * q : nullptr;
    int r = r0 + rg;
    for (; r + 3 * R < r1; r += 4 * R) {
      float4 av[4], xv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) av[k] = *(const float4*)(ap + (size_t)(r + k * R) * a_cs);
      if (mode == 1 || mode == 3) {
#pragma unroll
        for (int k = 0; k < 4; ++k) xv[k] = *(const float4*)(xp + (size_t)(r + k * R) * x_cs);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) acc_row(av[k], (mode == 1 || mode == 3) ? xv[k] : av[k]);
    }
    for (; r < r1; r += R)
      acc_row(*(const float4*)(ap + (size_t)r * a_cs),
              (mode == 1 || mode == 3) ? *(const float4*)(xp + (size_t)r * x_cs) : make_float4(0.f, 0.f, 0.f, 0.f));
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) { s1[threadIdx.x * 4 + e] = u[e]; s2[threadIdx.x * 4 + e] = v[e]; }
  __syncthreads();
  if (threadIdx.x < C4) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      double t1 = 0.0, t2 = 0.0;
      for (int k = 0; k < R; ++k) { t1 += s1[(k * C4 + threadIdx.x) * 4 + e]; t2 += s2[(k * C4 + threadIdx.x) * 4 + e]; }
      const int cc = 4 * threadIdx.x + e;
      if (mode == 2) atomicAdd(fout + cc, (float)t1);
      else { atomicAdd(acc + cc, t1); atomicAdd(acc + C + cc, t2); }
    }
  }
}

static bool reduce4_ok(int C, int cs, int coff, const void* p) {
  return C % 4 == 0 && C <= 1024 && cs % 4 == 0 && coff % 4 == 0 && ((uintptr_t)p & 15) == 0;
}

// Two-stage per-channel reductions (the float4 path): kRedSlots blocks of 1024
// threads each write their per-channel partial sums to a slot of their own
// (plain stores), then one small kernel adds the slots in slot order.  The
// single-stage form ended every block with 2C same-address fp64 atomics, which
// serialised at the L2 (1.2-1.8 TB/s on the training shapes); this one is also
// deterministic run to run.  Modes as chan_reduce4_kernel (0: x, x^2; 1: g,
// g*xhat; 2: g; 3: mode 1 with the consumer ReLU folded in).
constexpr int kRedSlots = 256;
constexpr int kRedThreads = 1024;

// TA / TX = half_t: the operand is an activation's compact fp16 copy (the
// autocast conv output's exact values: BatchNorm reads half the bytes)
template <typename TA = float, typename TX = float>
__global__ __launch_bounds__(kRedThreads) void chan_part_kernel(const TA* __restrict__ a, int a_cs, int a_coff,
                                                                const TX* __restrict__ x, int x_cs, int x_coff,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ invstd,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, int M, int C, int mode,
                                                                double* __restrict__ part) {
  extern __shared__ double red_sm[];  // [R][2C]: R * C = 4096
  const int C4 = C >> 2;
  const int R = kRedThreads / C4;
  const int q = threadIdx.x % C4, rg = threadIdx.x / C4;
  const int rows_per_block = (M + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  const bool gx = mode == 1 || mode == 3;
  double u[4] = {0.0, 0.0, 0.0, 0.0}, v[4] = {0.0, 0.0, 0.0, 0.0};
  if (rg < R) {
    float mu[4] = {0.f, 0.f, 0.f, 0.f}, is[4] = {0.f, 0.f, 0.f, 0.f}, ga[4] = {0.f, 0.f, 0.f, 0.f},
          be[4] = {0.f, 0.f, 0.f, 0.f};
    if (gx) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { mu[e] = mean[4 * q + e]; is[e] = invstd[4 * q + e]; }
    }
    if (mode == 3) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { ga[e] = gamma[4 * q + e]; be[e] = beta[4 * q + e]; }
    }
    const TA* ap = a + a_coff + 4 * q;
    const TX* xp = x ? x + x_coff + 4 * q : nullptr;
    auto row = [&](const float4 av, const float4 xv) {
      float ae[4] = {av.x, av.y, av.z, av.w};
      const float xe[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (gx) {
          if (mode == 3 && !(bn_affine(xe[e], mu[e], is[e], ga[e], be[e]) > 0.f)) ae[e] = 0.f;
          u[e] += ae[e];
          v[e] += (double)ae[e] * ((xe[e] - mu[e]) * is[e]);
        } else if (mode == 0) {
          u[e] += ae[e];
          v[e] += (double)ae[e] * ae[e];
        } else {
          u[e] += ae[e];
        }
      }
    };
    int r = r0 + rg;
    // one-operand modes (the forward statistics): 8 rows' loads in flight per
    // thread (4 left the 512^2 statistics passes latency-bound at ~3 TB/s),
    // then the 4-row batches, then single rows
    if (!gx) {
      for (; r + 7 * R < r1; r += 8 * R) {
        float4 av[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) av[k] = ld4f(ap + (size_t)(r + k * R) * a_cs);
#pragma unroll
        for (int k = 0; k < 8; ++k) row(av[k], av[k]);
      }
    }
    for (; r + 3 * R < r1; r += 4 * R) {
      float4 av[4], xv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) av[k] = ld4f(ap + (size_t)(r + k * R) * a_cs);
      if (gx) {
#pragma unroll
        for (int k = 0; k < 4; ++k) xv[k] = ld4f(xp + (size_t)(r + k * R) * x_cs);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) row(av[k], gx ? xv[k] : av[k]);
    }
    for (; r < r1; r += R)
      row(ld4f(ap + (size_t)r * a_cs), gx ? ld4f(xp + (size_t)r * x_cs) : make_float4(0.f, 0.f, 0.f, 0.f));
  }
  if (rg < R) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red_sm[rg * 2 * C + 4 * q + e] = u[e];
      red_sm[rg * 2 * C + C + 4 * q + e] = v[e];
    }
  }
  __syncthreads();
  double* dst = part + (size_t)blockIdx.x * 2 * C;
  for (int t = threadIdx.x; t < 2 * C; t += kRedThreads) {
    double s = 0.0;
    for (int k = 0; k < R; ++k) s += red_sm[k * 2 * C + t];
    dst[t] = s;
  }
}

// slot sums -> acc[2C] (modes 0/1/3, overwritten) or out[C] (+)= (mode 2), in
// a fixed order: a block owns 64 outputs (one per lane), wave w adds slots
// w, w + 4, ... in that order, 16 loads issued together per batch (64 slots:
// the former dependent chains waited out ~16 round trips, 5.7 us per call),
// then the 4 wave sums are added in order
__global__ __launch_bounds__(256) void chan_fin_kernel(const double* __restrict__ part, int slots, int C, int mode,
                                                       double* __restrict__ acc, float* __restrict__ out,
                                                       int accumulate) {
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int t = blockIdx.x * 64 + lane;
  const bool ok = t < 2 * C && !(mode == 2 && t >= C);
  double sum = 0.0;
  if (ok) {
    for (int k0 = w; k0 < slots; k0 += 64) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int k = k0 + 4 * u;
        v[u] = k < slots ? part[(size_t)k * 2 * C + t] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) sum += v[u];
    }
  }
  red[w][lane] = sum;
  __syncthreads();
  if (w == 0 && ok) {
    const double v = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    if (mode == 2) out[t] = (accumulate ? out[t] : 0.f) + (float)v;
    else acc[t] = v;
  }
}

template <typename TA = float, typename TX = float>
static int chan_reduce2(const TA* a, int a_cs, int a_coff, const TX* x, int x_cs, int x_coff, const float* mean,
                        const float* invstd, const float* gamma, const float* beta, int M, int C, int mode,
                        double* part, double* acc, float* out, int accumulate, hipStream_t st) {
  const int R = kRedThreads / (C / 4);
  int slots = M / (R * 16);
  slots = slots < 1 ? 1 : (slots > kRedSlots ? kRedSlots : slots);
  hipLaunchKernelGGL((chan_part_kernel<TA, TX>), dim3(slots), dim3(kRedThreads), (size_t)R * 2 * C * sizeof(double), st, a, a_cs,
                     a_coff, x, x_cs, x_coff, mean, invstd, gamma, beta, M, C, mode, part);
  UPR_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(chan_fin_kernel, dim3((2 * C + 63) / 64), dim3(256), 0, st, part, slots, C, mode, acc, out,
                     accumulate);
  return (int)hipGetLastError();
}




__global__ void bn_finalize_kernel(const double* __restrict__ acc, int M, int C, float momentum, float eps,
                                   float* __restrict__ rm, float* __restrict__ rv, long long* nbt,
                                   float* __restrict__ mean, float* __restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt) *nbt += 1;
  if (c >= C) return;
  const double mu = acc[c] / M;
  double var = acc[C + c] / M - mu * mu;
  if (var < 0) var = 0;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rm) rm[c] = (1.f - momentum) * rm[c] + momentum * (float)mu;
  if (rv) {
    const double unb = M > 1 ? var * M / (M - 1) : var;
    rv[c] = (1.f - momentum) * rv[c] + momentum * (float)unb;
  }
}

// eval-mode BatchNorm statistics: mean = running_mean, invstd = 1/sqrt(running_var + eps)
__global__ void bn_eval_stats_kernel(const float* __restrict__ rm, const float* __restrict__ rv, int C, float eps,
                                     float* __restrict__ mean, float* __restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  invstd[c] = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
}

__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ x, int M, int C, int x_cs,
                                                       int x_coff, const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, const float* res, int res_cs,
                                                       int res_coff, int res_post, int relu, float* y, int y_cs,
                                                       int y_coff) {
  const long long n = (long long)M * C;
  GSTRIDE(i, n) {
    const int c = (int)(i % C);
    const long long m = i / C;
    float v = bn_affine(x[m * x_cs + x_coff + c], mean[c], invstd[c], gamma[c], beta[c]);
    const float rv = res ? res[m * res_cs + res_coff + c] : 0.f;
    if (!res_post) v += rv;
    if (relu) v = fmaxf(v, 0.f);
    if (res_post) v += rv;
    y[m * y_cs + y_coff + c] = v;
  }
}

// the same arithmetic, 4 channels per thread (16-byte loads / stores), and
// optionally the compact fp16 copy y16[m][C] the next autocast conv reads
template <typename TX = float>
__global__ __launch_bounds__(256) void bn_apply4_kernel(const TX* __restrict__ x, int M, int C, int x_cs, int x_coff,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, const float* res, int res_cs,
                                                        int res_coff, int res_post, int relu, float* y, int y_cs,
                                                        int y_coff, half_t* __restrict__ y16, int skip32 = 0,
                                                        int y16_cs = 0) {
  const int C4 = C / 4;
  const int ycs16 = y16_cs > 0 ? y16_cs : C;  // y16: compact [M][C], or a channel slice of a wider copy
  if (256 % C4 == 0) {
    // this thread's 4 channels are fixed (the grid stride is a multiple of C4):
    // per-channel parameters once, row index by addition -- no div / mod per
    // element (the 64-bit form ran at ~3 TB/s); 32-bit offsets (host-checked)
    const int c = (threadIdx.x % C4) * 4, rpb = 256 / C4;
    float mu[4], is[4], ga[4], be[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) { mu[e] = mean[c + e]; is[e] = invstd[c + e]; ga[e] = gamma[c + e]; be[e] = beta[c + e]; }
    for (int m = blockIdx.x * rpb + threadIdx.x / C4; m < M; m += gridDim.x * rpb) {
      const float4 xv = ld4f(x + (size_t)m * x_cs + x_coff + c);
      const float4 rv4 = res ? *(const float4*)(res + (size_t)m * res_cs + res_coff + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float xa[4] = {xv.x, xv.y, xv.z, xv.w}, ra[4] = {rv4.x, rv4.y, rv4.z, rv4.w};
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = bn_affine(xa[e], mu[e], is[e], ga[e], be[e]);
        if (!res_post) v += ra[e];
        if (relu) v = fmaxf(v, 0.f);
        if (res_post) v += ra[e];
        o[e] = v;
      }
      if (!skip32) *(float4*)(y + (size_t)m * y_cs + y_coff + c) = make_float4(o[0], o[1], o[2], o[3]);
      if (y16) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        *(h4*)(y16 + (size_t)m * ycs16 + c) = h4{(half_t)o[0], (half_t)o[1], (half_t)o[2], (half_t)o[3]};
      }
    }
    return;
  }
  const long long n = (long long)M * C4;
  GSTRIDE(i, n) {
    const int c = (int)(i % C4) * 4;
    const long long m = i / C4;
    const float4 xv = ld4f(x + m * x_cs + x_coff + c);
    const float4 rv4 = res ? *(const float4*)(res + m * res_cs + res_coff + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float xa[4] = {xv.x, xv.y, xv.z, xv.w}, ra[4] = {rv4.x, rv4.y, rv4.z, rv4.w};
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = bn_affine(xa[e], mean[c + e], invstd[c + e], gamma[c + e], beta[c + e]);
      if (!res_post) v += ra[e];
      if (relu) v = fmaxf(v, 0.f);
      if (res_post) v += ra[e];
      o[e] = v;
    }
    if (!skip32) *(float4*)(y + m * y_cs + y_coff + c) = make_float4(o[0], o[1], o[2], o[3]);
    if (y16) {
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      *(h4*)(y16 + m * ycs16 + c) = h4{(half_t)o[0], (half_t)o[1], (half_t)o[2], (half_t)o[3]};
    }
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ g, int g_cs, int g_coff,
                                                           const float* __restrict__ x, int x_cs, int x_coff,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const double* __restrict__ acc, int M, int C,
                                                           float* dgamma, float* dbeta, float* dx, int dx_cs,
                                                           int dx_coff, int accum, int batch_stats) {
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      if (dgamma) dgamma[c] += (float)acc[C + c];
      if (dbeta) dbeta[c] += (float)acc[c];
    }
  }
  const long long n = (long long)M * C;
  GSTRIDE(i, n) {
    const int c = (int)(i % C);
    const long long m = i / C;
    const float is = invstd[c];
    const float xh = (x[m * x_cs + x_coff + c] - mean[c]) * is;
    // batch statistics: the mean / x-hat terms of the batch-statistics backward;
    // running statistics (an eval-mode BN): the plain affine map g * gamma * invstd
    const float sg = batch_stats ? (float)(acc[c] / M) : 0.f, sgx = batch_stats ? (float)(acc[C + c] / M) : 0.f;
    float v = gamma[c] * is * (g[m * g_cs + g_coff + c] - sg - xh * sgx);
    float* o = dx + m * dx_cs + dx_coff + c;
    if (accum) v += *o;
    *o = v;
  }
}

// the same arithmetic, 4 channels per thread (16-byte loads / stores)
template <typename TX = float, typename TG = float>
__global__ __launch_bounds__(256) void bn_bwd_apply4_kernel(const TG* __restrict__ g, int g_cs, int g_coff,
                                                            const TX* __restrict__ x, int x_cs, int x_coff,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd,
                                                            const float* __restrict__ gamma,
                                                            const double* __restrict__ acc, int M, int C,
                                                            float* dgamma, float* dbeta, float* dx, int dx_cs,
                                                            int dx_coff, int accum, int batch_stats,
                                                            const float* __restrict__ beta = nullptr, int relu = 0,
                                                            half_t* __restrict__ dx16 = nullptr, int skip32 = 0) {
  // relu: the consumer ReLU folded in (g counts where bn(x) > 0, recomputed);
  // dx16: compact [M][C] fp16 copy of dx for the autocast input-gradient conv
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      if (dgamma) dgamma[c] += (float)acc[C + c];
      if (dbeta) dbeta[c] += (float)acc[c];
    }
  }
  const int C4 = C / 4;
  if (256 % C4 == 0) {
    // fixed channels per thread (see bn_apply4_kernel): the per-channel terms,
    // fp64 divides included, once per thread instead of per element
    const int c = (threadIdx.x % C4) * 4, rpb = 256 / C4;
    // every per-channel load unconditional and issued together, the flags applied
    // by selects, 1/M one uniform divide: the conditional-load form (a branch and
    // a full memory wait per term, fp64 divides between) ran at ~2 TB/s on the
    // training shapes, its per-thread prologue dominating a one-row thread
    const float* bp = relu ? beta : gamma;  // beta may be NULL without the fold
    const double invM = batch_stats ? 1.0 / M : 0.0;
    float mu[4], is[4], ga[4], be[4], sg[4], sgx[4], gis[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      mu[e] = mean[c + e];
      is[e] = invstd[c + e];
      ga[e] = gamma[c + e];
      const float bv = bp[c + e];
      be[e] = relu ? bv : 0.f;
      sg[e] = (float)(acc[c + e] * invM);
      sgx[e] = (float)(acc[C + c + e] * invM);
      gis[e] = ga[e] * is[e];
    }
    for (int m = blockIdx.x * rpb + threadIdx.x / C4; m < M; m += gridDim.x * rpb) {
      const float4 gv = ld4f(g + (size_t)m * g_cs + g_coff + c);
      const float4 xv = ld4f(x + (size_t)m * x_cs + x_coff + c);
      const float ga4[4] = {gv.x, gv.y, gv.z, gv.w}, xa[4] = {xv.x, xv.y, xv.z, xv.w};
      float4* o = (float4*)(dx + (size_t)m * dx_cs + dx_coff + c);
      const float4 prev = accum ? *o : make_float4(0.f, 0.f, 0.f, 0.f);
      const float pa[4] = {prev.x, prev.y, prev.z, prev.w};
      float r[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = (xa[e] - mu[e]) * is[e];
        float gg = ga4[e];
        if (relu && !(bn_affine(xa[e], mu[e], is[e], ga[e], be[e]) > 0.f)) gg = 0.f;
        float v = gis[e] * (gg - sg[e] - xh * sgx[e]);
        if (accum) v += pa[e];
        r[e] = v;
      }
      if (!skip32) *o = make_float4(r[0], r[1], r[2], r[3]);
      if (dx16) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        *(h4*)(dx16 + (size_t)m * C + c) = h4{(half_t)r[0], (half_t)r[1], (half_t)r[2], (half_t)r[3]};
      }
    }
    return;
  }
  const long long n = (long long)M * C4;
  GSTRIDE(i, n) {
    const int c = (int)(i % C4) * 4;
    const long long m = i / C4;
    const float4 gv = ld4f(g + m * g_cs + g_coff + c);
    const float4 xv = ld4f(x + m * x_cs + x_coff + c);
    const float ga[4] = {gv.x, gv.y, gv.z, gv.w}, xa[4] = {xv.x, xv.y, xv.z, xv.w};
    float4* o = (float4*)(dx + m * dx_cs + dx_coff + c);
    float4 prev = accum ? *o : make_float4(0.f, 0.f, 0.f, 0.f);
    const float pa[4] = {prev.x, prev.y, prev.z, prev.w};
    float r[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float is = invstd[c + e];
      const float xh = (xa[e] - mean[c + e]) * is;
      const float sg = batch_stats ? (float)(acc[c + e] / M) : 0.f;
      const float sgx = batch_stats ? (float)(acc[C + c + e] / M) : 0.f;
      float gg = ga[e];
      if (relu && !(bn_affine(xa[e], mean[c + e], is, gamma[c + e], beta[c + e]) > 0.f)) gg = 0.f;
      float v = gamma[c + e] * is * (gg - sg - xh * sgx);
      if (accum) v += pa[e];
      r[e] = v;
    }
    if (!skip32) *o = make_float4(r[0], r[1], r[2], r[3]);
    if (dx16) {
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      *(h4*)(dx16 + m * C + c) = h4{(half_t)r[0], (half_t)r[1], (half_t)r[2], (half_t)r[3]};
    }
  }
}

// ---------------------------------------------------------------------------
// elementwise
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void relu_mask4_kernel(float* g, int g_cs, int g_coff, const float* __restrict__ y,
                                                         int y_cs, int y_coff, int M, int C) {
  const int C4 = C / 4;
  if (256 % C4 == 0) {  // fixed channels per thread (see bn_apply4_kernel)
    const int c = (threadIdx.x % C4) * 4, rpb = 256 / C4;
    for (int m = blockIdx.x * rpb + threadIdx.x / C4; m < M; m += gridDim.x * rpb) {
      const float4 yv = *(const float4*)(y + (size_t)m * y_cs + y_coff + c);
      float4* gp = (float4*)(g + (size_t)m * g_cs + g_coff + c);
      float4 gv = *gp;
      if (!(yv.x > 0.f)) gv.x = 0.f;
      if (!(yv.y > 0.f)) gv.y = 0.f;
      if (!(yv.z > 0.f)) gv.z = 0.f;
      if (!(yv.w > 0.f)) gv.w = 0.f;
      *gp = gv;
    }
    return;
  }
  const long long n = (long long)M * C4;
  GSTRIDE(i, n) {
    const int c = (int)(i % C4) * 4;
    const long long m = i / C4;
    const float4 yv = *(const float4*)(y + m * y_cs + y_coff + c);
    float4* gp = (float4*)(g + m * g_cs + g_coff + c);
    float4 gv = *gp;
    if (!(yv.x > 0.f)) gv.x = 0.f;
    if (!(yv.y > 0.f)) gv.y = 0.f;
    if (!(yv.z > 0.f)) gv.z = 0.f;
    if (!(yv.w > 0.f)) gv.w = 0.f;
    *gp = gv;
  }
}

// the mask fused with the fp16 copy of the masked gradient (the autocast
// dgrad operand, trainers/train.py:72): g16[m][c] = half(g masked), g itself
// rewritten only with write32 (a frozen conv's gradient has no fp32 reader)
// TY = half_t: the mask from the activation's fp16 copy (the autocast VGG
// activations are fp16 only; (half)y > 0 <=> y > 0 for their fp16-exact values)
template <typename TY = float>
__global__ __launch_bounds__(256) void relu_mask16_kernel(float* g, int g_cs, int g_coff, const TY* __restrict__ y,
                                                          int y_cs, int y_coff, int M, int C4,
                                                          half_t* __restrict__ g16, int write32) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= M * C4) return;
  const int c = (i % C4) * 4, m = i / C4;
  const float4 yv = ld4f(y + (size_t)m * y_cs + y_coff + c);
  float4* gp = (float4*)(g + (size_t)m * g_cs + g_coff + c);
  float4 gv = *gp;
  if (!(yv.x > 0.f)) gv.x = 0.f;
  if (!(yv.y > 0.f)) gv.y = 0.f;
  if (!(yv.z > 0.f)) gv.z = 0.f;
  if (!(yv.w > 0.f)) gv.w = 0.f;
  if (write32) *gp = gv;
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  *(h4*)(g16 + (size_t)i * 4) = h4{(half_t)gv.x, (half_t)gv.y, (half_t)gv.z, (half_t)gv.w};
}

__global__ void relu_mask_kernel(float* g, int g_cs, int g_coff, const float* __restrict__ y, int y_cs, int y_coff,
                                 int M, int C) {
  const long long n = (long long)M * C;
  GSTRIDE(i, n) {
    const int c = (int)(i % C);
    const long long m = i / C;
    if (!(y[m * y_cs + y_coff + c] > 0.f)) g[m * g_cs + g_coff + c] = 0.f;
  }
}

__global__ void copy_kernel(V s, V d, int B, int H, int W, int C, int accum) {
  const long long n = (long long)B * H * W * C;
  GSTRIDE(i, n) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int x = (int)(r % W); r /= W;
    const int y = (int)(r % H);
    const int b = (int)(r / H);
    const float v = s.d[s.at(b, y, x, c)];
    float* o = d.d + d.at(b, y, x, c);
    *o = accum ? *o + v : v;
  }
}

__device__ __forceinline__ float hash_uniform(unsigned long long seed, unsigned long long i) {
  // splitmix64 of (seed, index) -> [0, 1)
  unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

__global__ void pointwise_kernel(const float* a, const float* b, float* out, long long n, int op,
                                 const uint8_t* __restrict__ mask_in, uint8_t* __restrict__ mask_out, float p,
                                 unsigned long long seed) {
  GSTRIDE(i, n) {
    const float av = a[i];
    float v;
    switch (op) {
      case 0: v = 1.f / (1.f + expf(-av)); break;
      case 1: { const float s = b[i]; v = av * s * (1.f - s); } break;
      case 2: {
        const uint8_t m = hash_uniform(seed, (unsigned long long)i) >= p ? 1 : 0;
        mask_out[i] = m;
        v = m ? av * (1.f / (1.f - p)) : 0.f;
      } break;
      case 3: v = mask_in[i] ? av * (1.f / (1.f - p)) : 0.f; break;
      case 4: v = av + b[i]; break;
      default: v = av * b[0]; break;
    }
    out[i] = v;
  }
}

// ---------------------------------------------------------------------------
// pooling / resampling
// ---------------------------------------------------------------------------
__global__ void maxpool_kernel(V x, int B, int H, int W, int C, int k, int s, int p, V y, int Ho, int Wo) {
  const long long n = (long long)B * Ho * Wo * C;
  GSTRIDE(i, n) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int ox = (int)(r % Wo); r /= Wo;
    const int oy = (int)(r % Ho);
    const int b = (int)(r / Ho);
    float m = -INFINITY;
    for (int ky = 0; ky < k; ++ky) {
      const int iy = oy * s - p + ky;
      if (iy < 0 || iy >= H) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int ix = ox * s - p + kx;
        if (ix < 0 || ix >= W) continue;
        const float v = x.d[x.at(b, iy, ix, c)];
        if (v > m || isnan(v)) m = v;
      }
    }
    y.d[y.at(b, oy, ox, c)] = m;
  }
}

__device__ __forceinline__ void bilin_src(int o, int in, float scale, int& i0, int& i1, float& l) {
  float sr = ((float)o + 0.5f) * scale - 0.5f;
  if (sr < 0.f) sr = 0.f;
  i0 = (int)sr;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l = sr - (float)i0;
}

__global__ void bilinear_kernel(V x, int B, int H, int W, int C, V y, int Ho, int Wo, float sh, float sw, int accum) {
  const long long n = (long long)B * Ho * Wo * C;
  GSTRIDE(i, n) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int ox = (int)(r % Wo); r /= Wo;
    const int oy = (int)(r % Ho);
    const int b = (int)(r / Ho);
    int y0, y1, x0, x1;
    float ly, lx;
    bilin_src(oy, H, sh, y0, y1, ly);
    bilin_src(ox, W, sw, x0, x1, lx);
    const float v = (1.f - ly) * ((1.f - lx) * x.d[x.at(b, y0, x0, c)] + lx * x.d[x.at(b, y0, x1, c)]) +
                    ly * ((1.f - lx) * x.d[x.at(b, y1, x0, c)] + lx * x.d[x.at(b, y1, x1, c)]);
    float* o = y.d + y.at(b, oy, ox, c);
    *o = accum ? *o + v : v;
  }
}

// gather form of the bilinear backward: one thread per SOURCE element sums the
// output gradients whose forward taps (bilin_src, the forward's own arithmetic)
// land on it -- no atomics (the scatter form contends 16-256 ways on the 4x /
// 16x head upsamplings).  Candidate outputs: those whose source coordinate lies
// in [i-1, i+1]; the last row / column also collects the clamped tail.
__device__ __forceinline__ void bilin_range(int i, int in, int out, float scale, int& lo, int& hi) {
  lo = (int)floorf(((float)i - 0.5f) / scale - 0.5f) - 1;
  hi = (int)ceilf(((float)i + 1.5f) / scale - 0.5f) + 1;
  if (lo < 0) lo = 0;
  if (i == in - 1 || hi > out - 1) hi = out - 1;
}

__device__ __forceinline__ float bilin_w(int o, int i, int in, float scale) {
  int i0, i1;
  float l;
  bilin_src(o, in, scale, i0, i1, l);
  return (i0 == i ? 1.f - l : 0.f) + (i1 == i ? l : 0.f);
}

__global__ void bilinear_bwd_gather_kernel(V dy, int B, int H, int W, int C, int Ho, int Wo, float sh, float sw, V dx) {
  const long long n = (long long)B * H * W * C;
  GSTRIDE(i, n) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int ix = (int)(r % W); r /= W;
    const int iy = (int)(r % H);
    const int b = (int)(r / H);
    int ylo, yhi, xlo, xhi;
    bilin_range(iy, H, Ho, sh, ylo, yhi);
    bilin_range(ix, W, Wo, sw, xlo, xhi);
    float acc = 0.f;
    for (int oy = ylo; oy <= yhi; ++oy) {
      const float wy = bilin_w(oy, iy, H, sh);
      if (wy == 0.f) continue;
      float row = 0.f;
      for (int ox = xlo; ox <= xhi; ++ox) {
        const float wx = bilin_w(ox, ix, W, sw);
        if (wx != 0.f) row += wx * dy.d[dy.at(b, oy, ox, c)];
      }
      acc += wy * row;
    }
    dx.d[dx.at(b, iy, ix, c)] += acc;
  }
}

// 4-channel forms (V4 views, one thread per pixel and 4 channels)
__device__ __forceinline__ void dec4(int i, int CV, int W, int H, int& b, int& y, int& x, int& c) {
  c = (i % CV) * 4;
  int r = i / CV;
  x = r % W;
  r /= W;
  y = r % H;
  b = r / H;
}

// d16 (nullable): fp16 copy of the result at d16[pixel * cs16 + c] (pixel = (b*H + y)*W + x)
__device__ __forceinline__ void store16(half_t* d16, int cs16, int pix, int c, float4 v) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  *(h4*)(d16 + (size_t)pix * cs16 + c) = h4{(half_t)v.x, (half_t)v.y, (half_t)v.z, (half_t)v.w};
}

__global__ __launch_bounds__(256) void copy4_kernel(V4 s, V4 d, int H, int W, int CV, int n, int accum,
                                                    half_t* __restrict__ d16, int cs16) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int b, y, x, c;
  dec4(i, CV, W, H, b, y, x, c);
  float4 v = *(const float4*)s.at(b, y, x, c);
  float4* o = (float4*)d.at(b, y, x, c);
  if (accum == 1) {
    const float4 u = *o;
    v = make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w);
  }
  if (accum != 2) *o = v;  // 2: the fp16 copy only
  if (d16) store16(d16, cs16, i / CV, c, v);
}

__global__ __launch_bounds__(256) void bilinear4_kernel(V4 x, int H, int W, int CV, V4 y, int Ho, int Wo, float sh,
                                                        float sw, int n, int accum, half_t* __restrict__ y16,
                                                        int cs16) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int b, oy, ox, c;
  dec4(i, CV, Wo, Ho, b, oy, ox, c);
  int y0, y1, x0, x1;
  float ly, lx;
  bilin_src(oy, H, sh, y0, y1, ly);
  bilin_src(ox, W, sw, x0, x1, lx);
  const float4 a = *(const float4*)x.at(b, y0, x0, c), bq = *(const float4*)x.at(b, y0, x1, c);
  const float4 cq = *(const float4*)x.at(b, y1, x0, c), d = *(const float4*)x.at(b, y1, x1, c);
  // the scalar kernel's expression per channel
  float4 v;
  v.x = (1.f - ly) * ((1.f - lx) * a.x + lx * bq.x) + ly * ((1.f - lx) * cq.x + lx * d.x);
  v.y = (1.f - ly) * ((1.f - lx) * a.y + lx * bq.y) + ly * ((1.f - lx) * cq.y + lx * d.y);
  v.z = (1.f - ly) * ((1.f - lx) * a.z + lx * bq.z) + ly * ((1.f - lx) * cq.z + lx * d.z);
  v.w = (1.f - ly) * ((1.f - lx) * a.w + lx * bq.w) + ly * ((1.f - lx) * cq.w + lx * d.w);
  float4* o = (float4*)y.at(b, oy, ox, c);
  if (accum == 1) {
    const float4 u = *o;
    v = make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w);
  }
  if (accum != 2) *o = v;  // 2: the fp16 copy only
  if (y16) store16(y16, cs16, i / CV, c, v);
}

// bilinear backward, separable and in the gather kernel's summation order:
// pass 1 row[b][oy][ix] = sum over ox (ascending, nonzero weights) of
// wx * dy[b][oy][ox]; pass 2 dx[b][iy][ix] += sum over oy (ascending, nonzero
// weights) of wy * row[b][oy][ix].  Each pass scans ~3/scale candidates
// instead of the product of both axes.
__global__ __launch_bounds__(256) void bilinear_bwd_rows4_kernel(V4 dy, int Ho, int Wo, int W, int CV, float sw,
                                                                 float* __restrict__ row, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int b, oy, ix, c;
  dec4(i, CV, W, Ho, b, oy, ix, c);
  int xlo, xhi;
  bilin_range(ix, W, Wo, sw, xlo, xhi);
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  // four taps' loads issued together per pass (the tap loop of one load per
  // dependent step ran the 4x / 16x upsample backward at ~3 TB/s); zero-weight
  // taps are skipped as before, so the sums are unchanged
  for (int ox0 = xlo; ox0 <= xhi; ox0 += 4) {
    float wx[4];
    float4 g[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int ox = ox0 + k;
      wx[k] = ox <= xhi ? bilin_w(ox, ix, W, sw) : 0.f;
      g[k] = wx[k] != 0.f ? *(const float4*)dy.at(b, oy, ox, c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (wx[k] == 0.f) continue;
      r.x += wx[k] * g[k].x;
      r.y += wx[k] * g[k].y;
      r.z += wx[k] * g[k].z;
      r.w += wx[k] * g[k].w;
    }
  }
  *(float4*)(row + (size_t)i * 4) = r;
}

__global__ __launch_bounds__(256) void bilinear_bwd_cols4_kernel(const float* __restrict__ row, int Ho, int H, int W,
                                                                 int CV, float sh, V4 dx, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int b, iy, ix, c;
  dec4(i, CV, W, H, b, iy, ix, c);
  int ylo, yhi;
  bilin_range(iy, H, Ho, sh, ylo, yhi);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int C = CV * 4;
  for (int oy = ylo; oy <= yhi; ++oy) {
    const float wy = bilin_w(oy, iy, H, sh);
    if (wy == 0.f) continue;
    const float4 r = *(const float4*)(row + (((size_t)b * Ho + oy) * W + ix) * C + c);
    acc.x += wy * r.x;
    acc.y += wy * r.y;
    acc.z += wy * r.z;
    acc.w += wy * r.w;
  }
  float4* o = (float4*)dx.at(b, iy, ix, c);
  const float4 u = *o;
  *o = make_float4(u.x + acc.x, u.y + acc.y, u.z + acc.z, u.w + acc.w);
}

// per-(image, channel) pixel sums: grid (chunks, B)
__global__ __launch_bounds__(256) void pixel_sum_kernel(const float* __restrict__ x, int HW, int C, int cs, int coff,
                                                        float scale, float* __restrict__ out) {
  __shared__ float sm[256];
  const int b = blockIdx.y;
  const int per = (HW + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * per, p1 = min(HW, p0 + per);
  for (int cb = 0; cb < C; cb += 256) {
    const int cw = min(256, C - cb);
    const int R = 256 / cw;
    const int c = threadIdx.x % cw, rg = threadIdx.x / cw;
    float u = 0.f;
    if (rg < R)
      for (int q = p0 + rg; q < p1; q += R) u += x[((size_t)b * HW + q) * cs + coff + cb + c];
    sm[threadIdx.x] = u;
    __syncthreads();
    if (threadIdx.x < cw) {
      float t = 0.f;
      for (int k = 0; k < R; ++k) t += sm[k * cw + threadIdx.x];
      atomicAdd(out + (size_t)b * C + cb + threadIdx.x, t * scale);
    }
    __syncthreads();
  }
}

// The same with 4 channels per lane (C % 4 == 0, 16-byte rows; C <= 1024) and
// 4 rows of loads in flight per lane, each block's sums stored to its own
// partial slot and added in chunk order by pixel_sum_fin_kernel (the FAM
// pool's 32-channel sum at 512^2 ran at 1.3 TB/s as one float per lane per
// dependent step, and its per-block atomics made the order run-dependent)
__global__ __launch_bounds__(256) void pixel_sum4_kernel(const float* __restrict__ x, int HW, int C, int cs, int coff,
                                                         float* __restrict__ part) {
  __shared__ float4 sm[256];
  const int b = blockIdx.y;
  const int C4 = C >> 2, R = 256 / C4;
  const int per = (HW + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * per, p1 = min(HW, p0 + per);
  const int c4 = threadIdx.x % C4, rg = threadIdx.x / C4;
  float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
  if (rg < R) {
    const float* base = x + (size_t)b * HW * cs + coff + 4 * c4;
    int q = p0 + rg;
    for (; q + 3 * R < p1; q += 4 * R) {
      float4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = *(const float4*)(base + (size_t)(q + k * R) * cs);
#pragma unroll
      for (int k = 0; k < 4; ++k) { u.x += v[k].x; u.y += v[k].y; u.z += v[k].z; u.w += v[k].w; }
    }
    for (; q < p1; q += R) {
      const float4 v = *(const float4*)(base + (size_t)q * cs);
      u.x += v.x; u.y += v.y; u.z += v.z; u.w += v.w;
    }
  }
  sm[threadIdx.x] = u;
  __syncthreads();
  if (threadIdx.x < C4) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < R; ++k) {
      const float4 w = sm[k * C4 + threadIdx.x];
      t.x += w.x; t.y += w.y; t.z += w.z; t.w += w.w;
    }
    *(float4*)(part + ((size_t)b * gridDim.x + blockIdx.x) * C + 4 * threadIdx.x) = t;
  }
}

// out[b][c] (+)= scale * (partials of chunks 0, 1, ... in order)
__global__ __launch_bounds__(256) void pixel_sum_fin_kernel(const float* __restrict__ part, int chunks, int BC, int C,
                                                            float scale, float* __restrict__ out, int accumulate) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= BC) return;
  const int b = j / C, c = j - b * C;
  const float* p = part + (size_t)b * chunks * C + c;
  float t = 0.f;
  int k = 0;
  for (; k + 3 < chunks; k += 4) {
    const float v0 = p[(size_t)k * C], v1 = p[(size_t)(k + 1) * C], v2 = p[(size_t)(k + 2) * C], v3 = p[(size_t)(k + 3) * C];
    t += v0; t += v1; t += v2; t += v3;
  }
  for (; k < chunks; ++k) t += p[(size_t)k * C];
  out[j] = (accumulate ? out[j] : 0.f) + t * scale;
}

// the fp16 form: y16[b][p][coff + c] = (half)(v[b][c] * scale), 4 channels per thread
__global__ void broadcast16_kernel(const float* __restrict__ v, int B, int HW, int C, float scale,
                                   half_t* __restrict__ y16, int y_cs, int y_coff) {
  const int C4 = C / 4;
  const long long n = (long long)B * HW * C4;
  GSTRIDE(i, n) {
    const int c = (int)(i % C4) * 4;
    const long long m = i / C4;
    const int b = (int)(m / HW);
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const float* s = v + (size_t)b * C + c;
    *(h4*)(y16 + m * y_cs + y_coff + c) =
        h4{(half_t)(s[0] * scale), (half_t)(s[1] * scale), (half_t)(s[2] * scale), (half_t)(s[3] * scale)};
  }
}

__global__ void broadcast_kernel(const float* __restrict__ v, int B, int HW, int C, float scale, float* y, int y_cs,
                                 int y_coff, int accum) {
  const long long n = (long long)B * HW * C;
  GSTRIDE(i, n) {
    const int c = (int)(i % C);
    const long long m = i / C;
    const int b = (int)(m / HW);
    float* o = y + m * y_cs + y_coff + c;
    const float val = v[(size_t)b * C + c] * scale;
    *o = accum ? *o + val : val;
  }
}

// ---------------------------------------------------------------------------
// EnhancedFAM attention (one thread per pixel, C channels contiguous)
// ---------------------------------------------------------------------------
__global__ void fam_ca_apply_kernel(const float* __restrict__ o, const float* __restrict__ ca, int B, int HW, int C,
                                    float* __restrict__ o2, float* __restrict__ m) {
  const long long n = (long long)B * HW;
  GSTRIDE(i, n) {
    const int b = (int)(i / HW);
    const float* op = o + i * C;
    float* q = o2 + i * C;
    float s = 0.f, mx = -INFINITY;
    for (int c = 0; c < C; ++c) {
      const float v = op[c] * ca[(size_t)b * C + c];
      q[c] = v;
      s += v;
      if (v > mx || isnan(v)) mx = v;
    }
    m[i * 2] = s / (float)C;
    m[i * 2 + 1] = mx;
  }
}

__global__ void fam_sa_apply_kernel(const float* __restrict__ o2, const float* __restrict__ s_pre, int B, int HW, int C,
                                    float* __restrict__ sa, float* __restrict__ out) {
  const long long n = (long long)B * HW;
  GSTRIDE(i, n) {
    const float a = 1.f / (1.f + expf(-s_pre[i]));
    sa[i] = a;
    for (int c = 0; c < C; ++c) out[i * C + c] = o2[i * C + c] * a;
  }
}

__global__ void fam_sa_bwd_kernel(const float* __restrict__ g, int g_cs, const float* __restrict__ o2,
                                  const float* __restrict__ sa, int B, int HW, int C, float* __restrict__ g_o2,
                                  float* __restrict__ g_spre) {
  const long long n = (long long)B * HW;
  GSTRIDE(i, n) {
    const float a = sa[i];
    float t = 0.f;
    for (int c = 0; c < C; ++c) {
      const float gv = g[i * g_cs + c];
      t += gv * o2[i * C + c];
      g_o2[i * C + c] = gv * a;
    }
    g_spre[i] = t * a * (1.f - a);
  }
}

// C == 32 forms of the three per-pixel attention kernels above: 8 lanes per
// pixel, one float4 per lane (a wave reads 8 whole 128-byte pixel rows per
// instruction instead of 64 lanes striding 128 B apart), the channel mean / max /
// dot reduced over the 8-lane group by xor shuffles.  Groups of 8 are aligned
// (n and blockDim multiples of 8), so a whole group leaves the loop together.
__device__ __forceinline__ float nanmax(float a, float b) { return (b > a || isnan(b)) ? b : a; }

__global__ void fam_ca_apply32_kernel(const float* __restrict__ o, const float* __restrict__ ca, int B, int HW,
                                      float* __restrict__ o2, float* __restrict__ m) {
  const long long n = (long long)B * HW * 8;
  GSTRIDE(i, n) {
    const long long pix = i >> 3;
    const int q = (int)(i & 7);
    const int b = (int)(pix / HW);
    float4 v = ((const float4*)(o + pix * 32))[q];
    const float4 w = ((const float4*)(ca + (size_t)b * 32))[q];
    v.x *= w.x; v.y *= w.y; v.z *= w.z; v.w *= w.w;
    ((float4*)(o2 + pix * 32))[q] = v;
    float sm = (v.x + v.y) + (v.z + v.w);
    float mx = nanmax(nanmax(v.x, v.y), nanmax(v.z, v.w));
    for (int off = 1; off < 8; off <<= 1) {
      sm += __shfl_xor(sm, off);
      mx = nanmax(mx, __shfl_xor(mx, off));
    }
    if (q == 0) {
      m[pix * 2] = sm / 32.f;
      m[pix * 2 + 1] = mx;
    }
  }
}

__global__ void fam_sa_apply32_kernel(const float* __restrict__ o2, const float* __restrict__ s_pre, int B, int HW,
                                      float* __restrict__ sa, float* __restrict__ out) {
  const long long n = (long long)B * HW * 8;
  GSTRIDE(i, n) {
    const long long pix = i >> 3;
    const int q = (int)(i & 7);
    const float a = 1.f / (1.f + expf(-s_pre[pix]));
    if (q == 0) sa[pix] = a;
    float4 v = ((const float4*)(o2 + pix * 32))[q];
    v.x *= a; v.y *= a; v.z *= a; v.w *= a;
    ((float4*)(out + pix * 32))[q] = v;
  }
}

__global__ void fam_sa_bwd32_kernel(const float* __restrict__ g, int g_cs, const float* __restrict__ o2,
                                    const float* __restrict__ sa, int B, int HW, float* __restrict__ g_o2,
                                    float* __restrict__ g_spre) {
  const long long n = (long long)B * HW * 8;
  GSTRIDE(i, n) {
    const long long pix = i >> 3;
    const int q = (int)(i & 7);
    const float a = sa[pix];
    const float4 gv = ((const float4*)(g + pix * g_cs))[q];
    const float4 ov = ((const float4*)(o2 + pix * 32))[q];
    float t = (gv.x * ov.x + gv.y * ov.y) + (gv.z * ov.z + gv.w * ov.w);
    ((float4*)(g_o2 + pix * 32))[q] = make_float4(gv.x * a, gv.y * a, gv.z * a, gv.w * a);
    for (int off = 1; off < 8; off <<= 1) t += __shfl_xor(t, off);
    if (q == 0) g_spre[pix] = t * a * (1.f - a);
  }
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// g_ca[b][c] partials go through LDS: a block covers a pixel range of one image
__global__ __launch_bounds__(256) void fam_ca_bwd_kernel(const float* __restrict__ g_o2, const float* __restrict__ g_m,
                                                         const float* __restrict__ o, const float* __restrict__ o2,
                                                         const float* __restrict__ ca, int HW, int C,
                                                         float* __restrict__ g_o, float* __restrict__ g_ca) {
  __shared__ float sm[256][33];
  const int b = blockIdx.y;
  const int per = (HW + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * per, p1 = min(HW, p0 + per);
  float part[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) part[c] = 0.f;
  for (int q = p0 + threadIdx.x; q < p1; q += 256) {
    const size_t i = (size_t)b * HW + q;
    const float gm0 = g_m[i * 2] / (float)C, gm1 = g_m[i * 2 + 1];
    // argmax over channels of o2 (first maximum, torch.max semantics)
    int am = 0;
    float mx = o2[i * C];
    for (int c = 1; c < C; ++c) {
      const float v = o2[i * C + c];
      if (v > mx || (isnan(v) && !isnan(mx))) { mx = v; am = c; }
    }
#pragma unroll
    for (int c = 0; c < 32; ++c) {
      if (c >= C) break;
      const float gt = g_o2[i * C + c] + gm0 + (c == am ? gm1 : 0.f);
      g_o[i * C + c] = gt * ca[(size_t)b * C + c];
      part[c] += gt * o[i * C + c];
    }
  }
#pragma unroll
  for (int c = 0; c < 32; ++c) sm[threadIdx.x][c] = part[c];
  __syncthreads();
  if (threadIdx.x < C) {
    float t = 0.f;
    for (int k = 0; k < 256; ++k) t += sm[k][threadIdx.x];
    atomicAdd(g_ca + (size_t)b * C + threadIdx.x, t);
  }
}

// C = 32 form: 8 lanes per pixel (a float4 of channels each, coalesced rows),
// the channel argmax reduced across the 8 lanes with the scan's rule (first
// NaN, else first maximum), per-block partial sums of gt * o in a fixed order
// to part[b][chunk][c] (summed in chunk order by fam_ca_fin_kernel: no atomics)
__device__ __forceinline__ void argmax_pick(float& v, int& i, float v2, int i2) {
  const bool second_is_later = i2 > i;
  const float fv = second_is_later ? v : v2, sv = second_is_later ? v2 : v;
  const int fi = second_is_later ? i : i2, si = second_is_later ? i2 : i;
  const bool take_second = sv > fv || (isnan(sv) && !isnan(fv));
  v = take_second ? sv : fv;
  i = take_second ? si : fi;
}

__global__ __launch_bounds__(256) void fam_ca_bwd32_kernel(const float* __restrict__ g_o2,
                                                           const float* __restrict__ g_m, const float* __restrict__ o,
                                                           const float* __restrict__ o2, const float* __restrict__ ca,
                                                           int HW, float* __restrict__ g_o, float* __restrict__ part) {
  __shared__ float sm[32][33];
  const int b = blockIdx.y, q = threadIdx.x & 7, pl = threadIdx.x >> 3;
  const int per = (HW + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * per, p1 = min(HW, p0 + per);
  const float4 cav = *(const float4*)(ca + (size_t)b * 32 + q * 4);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  // (each pixel's four operand loads are issued together, before its argmax
  // shuffles: 99.9 -> 93.7 us per call on the training step)
  for (int p = p0 + pl; p < p1; p += 32) {
    const size_t i = (size_t)b * HW + p;
    const float4 v = *(const float4*)(o2 + i * 32 + q * 4);
    const float4 gv = *(const float4*)(g_o2 + i * 32 + q * 4);
    const float4 ov = *(const float4*)(o + i * 32 + q * 4);
    const float gm0 = g_m[i * 2] / 32.f, gm1 = g_m[i * 2 + 1];
    float mv = v.x;
    int mi = q * 4;
    argmax_pick(mv, mi, v.y, q * 4 + 1);
    argmax_pick(mv, mi, v.z, q * 4 + 2);
    argmax_pick(mv, mi, v.w, q * 4 + 3);
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) {
      const float v2 = __shfl_xor(mv, off);
      const int i2 = __shfl_xor(mi, off);
      argmax_pick(mv, mi, v2, i2);
    }
    const int c0 = q * 4;
    const float t0 = gv.x + gm0 + (mi == c0 ? gm1 : 0.f), t1 = gv.y + gm0 + (mi == c0 + 1 ? gm1 : 0.f);
    const float t2 = gv.z + gm0 + (mi == c0 + 2 ? gm1 : 0.f), t3 = gv.w + gm0 + (mi == c0 + 3 ? gm1 : 0.f);
    *(float4*)(g_o + i * 32 + q * 4) = make_float4(t0 * cav.x, t1 * cav.y, t2 * cav.z, t3 * cav.w);
    acc.x += t0 * ov.x;
    acc.y += t1 * ov.y;
    acc.z += t2 * ov.z;
    acc.w += t3 * ov.w;
  }
  sm[pl][q * 4] = acc.x;
  sm[pl][q * 4 + 1] = acc.y;
  sm[pl][q * 4 + 2] = acc.z;
  sm[pl][q * 4 + 3] = acc.w;
  __syncthreads();
  if (threadIdx.x < 32) {
    float t = 0.f;
    for (int k = 0; k < 32; ++k) t += sm[k][threadIdx.x];
    part[((size_t)b * gridDim.x + blockIdx.x) * 32 + threadIdx.x] = t;
  }
}

__global__ __launch_bounds__(256) void fam_ca_fin_kernel(const float* __restrict__ part, int chunks, int n,
                                                         float* __restrict__ g_ca) {
  __shared__ float red[256];
  const int j = blockIdx.x;  // j = b * 32 + c: one block per output, fixed-order tree
  const int b = j >> 5, c = j & 31;
  float t = 0.f;
  for (int k = threadIdx.x; k < chunks; k += 256) t += part[((size_t)b * chunks + k) * 32 + c];
  red[threadIdx.x] = t;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) g_ca[j] = red[0];
}

__global__ void fam_pool_bwd_kernel(float* g_o, const float* __restrict__ g_pool, const float* __restrict__ o, int B,
                                    int HW, int C) {
  const long long n = (long long)B * HW * C;
  GSTRIDE(i, n) {
    const int c = (int)(i % C);
    const int b = (int)(i / ((long long)HW * C));
    const float v = g_o[i] + g_pool[(size_t)b * C + c] / (float)HW;
    g_o[i] = o[i] > 0.f ? v : 0.f;
  }
}

// the same, 4 channels per thread (the channels of a thread fixed: C / 4
// divides 256), 32-bit offsets (host-checked), and optionally the compact fp16
// copy g16 of the result (the fusion conv's autocast gradient operand)
__global__ __launch_bounds__(256) void fam_pool_bwd4_kernel(float* g_o, const float* __restrict__ g_pool,
                                                            const float* __restrict__ o, int M, int HW, int C,
                                                            half_t* __restrict__ g16) {
  const int C4 = C / 4, c = (threadIdx.x % C4) * 4, rpb = 256 / C4;
  for (int m = blockIdx.x * rpb + threadIdx.x / C4; m < M; m += gridDim.x * rpb) {
    const int b = m / HW;
    const int off = m * C + c;
    const float4 gv = *(const float4*)(g_o + off), ov = *(const float4*)(o + off);
    const float4 pv = *(const float4*)(g_pool + b * C + c);
    float4 r;
    // g_pool / HW as the scalar kernel: a division per element
    r.x = ov.x > 0.f ? gv.x + pv.x / (float)HW : 0.f;
    r.y = ov.y > 0.f ? gv.y + pv.y / (float)HW : 0.f;
    r.z = ov.z > 0.f ? gv.z + pv.z / (float)HW : 0.f;
    r.w = ov.w > 0.f ? gv.w + pv.w / (float)HW : 0.f;
    *(float4*)(g_o + off) = r;
    if (g16) {
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      *(h4*)(g16 + off) = h4{(half_t)r.x, (half_t)r.y, (half_t)r.z, (half_t)r.w};
    }
  }
}

// ---------------------------------------------------------------------------
// network tail
// ---------------------------------------------------------------------------
__global__ void head_fwd_kernel(const float* __restrict__ x, const float* __restrict__ r, float* __restrict__ illu,
                                int B, int HW) {
  const long long n = (long long)B * HW;
  GSTRIDE(i, n) {
    const int b = (int)(i / HW), p = (int)(i - (long long)b * HW);
    const float* xb = x + (size_t)b * 3 * HW + p;
    const float z = (xb[0] + xb[HW] + xb[2 * HW]) / 3.f + r[i];
    illu[i] = 1.f / (1.f + expf(-z));
  }
}

__global__ void retinex_fwd_kernel(const float* __restrict__ x, const float* __restrict__ illu,
                                   const float* __restrict__ o, float* __restrict__ e, float* __restrict__ refl,
                                   float* __restrict__ enh, int B, int HW) {
  const long long n = (long long)B * HW;
  GSTRIDE(i, n) {
    const int b = (int)(i / HW), p = (int)(i - (long long)b * HW);
    const float den = illu[i] + 1e-6f;
    for (int c = 0; c < 3; ++c) {
      const size_t k = ((size_t)b * 3 + c) * HW + p;
      const float ev = 1.f / (1.f + expf(-o[i * 3 + c]));
      const float rv = x[k] / den;
      e[i * 3 + c] = ev;
      refl[k] = rv;
      enh[k] = rv * ev + (1.f - rv) * (ev * ev);
    }
  }
}

__global__ void retinex_bwd_kernel(const float* __restrict__ x, const float* __restrict__ illu,
                                   const float* __restrict__ e, const float* __restrict__ refl,
                                   const float* __restrict__ g_enh, const float* __restrict__ g_refl,
                                   const float* __restrict__ g_illu, float* __restrict__ g_o, float* __restrict__ g_r,
                                   int B, int HW) {
  const long long n = (long long)B * HW;
  GSTRIDE(i, n) {
    const int b = (int)(i / HW), p = (int)(i - (long long)b * HW);
    const float il = illu[i];
    const float den = il + 1e-6f;
    float gi = g_illu ? g_illu[i] : 0.f;
    for (int c = 0; c < 3; ++c) {
      const size_t k = ((size_t)b * 3 + c) * HW + p;
      const float ev = e[i * 3 + c], rv = refl[k], ge = g_enh[k];
      // enh = r*e + (1-r)*e^2
      const float gev = ge * (rv + 2.f * ev * (1.f - rv));
      const float grv = ge * (ev - ev * ev) + (g_refl ? g_refl[k] : 0.f);
      g_o[i * 3 + c] = gev * ev * (1.f - ev);
      // r = x / (illu + 1e-6)
      gi -= grv * x[k] / (den * den);
    }
    g_r[i] = gi * il * (1.f - il);
  }
}

// multi_scale_enhance's combine with a caller-given reflectance
// (models/model.py:439-443): e = sigmoid(o), enh = refl*e + (1-refl)*e^2; the
// backward writes dL/do (NHWC, through the sigmoid) and dL/drefl (NCHW)
__global__ void enhance_fwd_kernel(const float* __restrict__ refl, const float* __restrict__ o, float* __restrict__ e,
                                   float* __restrict__ enh, int B, int HW) {
  const long long n = (long long)B * HW;
  GSTRIDE(i, n) {
    const int b = (int)(i / HW), p = (int)(i - (long long)b * HW);
    for (int c = 0; c < 3; ++c) {
      const size_t k = ((size_t)b * 3 + c) * HW + p;
      const float ev = 1.f / (1.f + expf(-o[i * 3 + c]));
      const float rv = refl[k];
      e[i * 3 + c] = ev;
      enh[k] = rv * ev + (1.f - rv) * (ev * ev);
    }
  }
}

__global__ void enhance_bwd_kernel(const float* __restrict__ e, const float* __restrict__ refl,
                                   const float* __restrict__ g_enh, float* __restrict__ g_o,
                                   float* __restrict__ g_refl, int B, int HW) {
  const long long n = (long long)B * HW;
  GSTRIDE(i, n) {
    const int b = (int)(i / HW), p = (int)(i - (long long)b * HW);
    for (int c = 0; c < 3; ++c) {
      const size_t k = ((size_t)b * 3 + c) * HW + p;
      const float ev = e[i * 3 + c], rv = refl[k], ge = g_enh[k];
      g_o[i * 3 + c] = ge * (rv + 2.f * ev * (1.f - rv)) * ev * (1.f - ev);
      if (g_refl) g_refl[k] = ge * (ev - ev * ev);
    }
  }
}

// ---------------------------------------------------------------------------
// TotalLoss pixel terms (loss.py): workspace of fp64 accumulators
// ---------------------------------------------------------------------------
enum {
  LA_COL = 0,      // 3: sum enh_c
  LA_SPA_H = 3, LA_SPA_V = 4,
  LA_SM_H = 5, LA_SM_V = 6,
  LA_TV_H = 7, LA_TV_V = 8,
  LA_GLOW = 9,
  LA_FIXED = 16,   // then per image LA_IMG: [sum illu_c (3), sum r_j (3), sum illu_c*r_j (3x3)]
  LA_IMG = 16,     // (one illumination channel: c = 0 only)
};

struct LossWS {
  double* acc;     // LA_FIXED + LA_IMG * B
  double* patch;   // B * (H/ps) * (W/ps) sums of gray(enh) (ps = exposure patch size)
  double* rowsum;  // B*H   sum_{x<W-1} edge
  double* colsum;  // B*W   sum_{y<H-1} edge
  double* ed;      // 2B    texture 'edge_density': per image sum of |Sobel|, count above threshold
  float* scal;     // finalised scalars for the gradient pass
  // loss module arguments (UprLossParams)
  int ps;          // AdaptiveExposureLoss patch_size
  float base_exp;  // base_target_exposure
  float lam_s, alpha;  // EdgeAwareSmoothnessLoss lambda_val, alpha
  float lam_d;     // IlluminationReflectanceDecouplingLoss lambda_val
  int dynamic;     // TotalLoss use_dynamic_smooth_weight
};

// finalised scalars: 64 + per image LS_IMG
static size_t loss_scal_bytes(int B) { return align_up(sizeof(float) * (64 + 16 * B), 256); }

static LossWS loss_ws(void* ws, int B, int H, int W, int ps) {
  LossWS l;
  char* p = (char*)ws;
  l.acc = (double*)p; p += align_up(sizeof(double) * (LA_FIXED + LA_IMG * B), 256);
  l.patch = (double*)p; p += align_up(sizeof(double) * B * (H / ps) * (W / ps), 256);
  l.rowsum = (double*)p; p += align_up(sizeof(double) * B * H, 256);
  l.colsum = (double*)p; p += align_up(sizeof(double) * B * W, 256);
  l.ed = (double*)p; p += align_up(sizeof(double) * 2 * B, 256);
  l.scal = (float*)p;
  return l;
}
static size_t loss_ws_bytes(int B, int H, int W, int ps) {
  return align_up(sizeof(double) * (LA_FIXED + LA_IMG * B), 256) +
         align_up(sizeof(double) * B * (H / ps) * (W / ps), 256) + align_up(sizeof(double) * B * H, 256) +
         align_up(sizeof(double) * B * W, 256) + align_up(sizeof(double) * 2 * B, 256) + loss_scal_bytes(B);
}

// scalar slots
// per image LS_IMG: covariance [c][j] (9; one illumination channel: [j] = row 0),
// mean differences (3 at +9; one channel: +9 = mean I - mean of the R means),
// illumination means (3 at +12)
enum { LS_T = 0, LS_NPATCH = 1, LS_WS = 2, LS_MU = 3 /*3*/, LS_NH = 6, LS_NV = 7, LS_DEC = 8, LS_IMG = 16 };

__device__ __forceinline__ float gray_at(const float* img, size_t base, int HW, int p) {
  return (img[base + p] + img[base + HW + p] + img[base + 2 * HW + p]) / 3.f;
}

// Sobel edge magnitude of gray(low) with reflect padding (loss.py:110-136)
__device__ float edge_at(const float* low, size_t base, int H, int W, int y, int x) {
  const int HW = H * W;
  float g[3][3];
  for (int dy = -1; dy <= 1; ++dy) {
    int yy = y + dy;
    yy = yy < 0 ? -yy : (yy >= H ? 2 * H - 2 - yy : yy);
    for (int dx = -1; dx <= 1; ++dx) {
      int xx = x + dx;
      xx = xx < 0 ? -xx : (xx >= W ? 2 * W - 2 - xx : xx);
      g[dy + 1][dx + 1] = gray_at(low, base, HW, yy * W + xx);
    }
  }
  const float gx = -g[0][0] + g[0][2] - 2.f * g[1][0] + 2.f * g[1][2] - g[2][0] + g[2][2];
  const float gy = -g[0][0] - 2.f * g[0][1] - g[0][2] + g[2][0] + 2.f * g[2][1] + g[2][2];
  return sqrtf(gx * gx + gy * gy);
}

template <int NV>
__device__ __forceinline__ void block_sum_atomic(double (&v)[NV], double* dst[NV]) {
  __shared__ double sm[NV][256];
#pragma unroll
  for (int k = 0; k < NV; ++k) sm[k][threadIdx.x] = v[k];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
#pragma unroll
      for (int k = 0; k < NV; ++k) sm[k][threadIdx.x] += sm[k][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k)
      if (dst[k]) atomicAdd(dst[k], sm[k][0]);
  }
  __syncthreads();
}

template <int CI>
constexpr int loss_nv() { return 10 + CI + 3 + 3 * CI; }  // fixed sums, then sum I_c, sum R_j, sum I_c R_j

// one pixel's pass-1 terms into v; ge = gray(enh), ed = Sobel magnitude of gray(low)
template <int CI>
__device__ __forceinline__ void loss_pixel1(const float* __restrict__ low, const float* __restrict__ enh,
                                            const float* __restrict__ illu, const float* __restrict__ refl, int b,
                                            size_t base, int H, int W, int q, int y, int x,
                                            double (&v)[loss_nv<CI>()], float& ge, float& ed) {
  const int HW = H * W;
  float le[3], ll[3];
  for (int c = 0; c < 3; ++c) { le[c] = enh[base + c * HW + q]; ll[c] = low[base + c * HW + q]; }
  for (int c = 0; c < 3; ++c) v[c] += le[c];
  v[9] += (ll[0] + ll[1] + ll[2]) / 3.f;
  if (x < W - 1) {
    for (int c = 0; c < 3; ++c) {
      const float de = le[c] - enh[base + c * HW + q + 1], dl = ll[c] - low[base + c * HW + q + 1];
      v[3] += (double)(de - dl) * (de - dl);
      v[7] += fabsf(dl);
    }
  }
  if (y < H - 1) {
    for (int c = 0; c < 3; ++c) {
      const float de = le[c] - enh[base + c * HW + q + W], dl = ll[c] - low[base + c * HW + q + W];
      v[4] += (double)(de - dl) * (de - dl);
      v[8] += fabsf(dl);
    }
  }
  float il[CI];
#pragma unroll
  for (int c = 0; c < CI; ++c) {
    il[c] = illu[((size_t)b * CI + c) * HW + q];
    v[10 + c] += il[c];
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float r = refl[base + j * HW + q];
    v[10 + CI + j] += r;
#pragma unroll
    for (int c = 0; c < CI; ++c) v[13 + CI + c * 3 + j] += (double)il[c] * r;
  }
  ge = (le[0] + le[1] + le[2]) / 3.f;
  ed = edge_at(low, base, H, W, y, x);
}

template <int CI>
__device__ __forceinline__ void loss_pass1_flush(double (&v)[loss_nv<CI>()], const LossWS& ws, int b) {
  constexpr int NV = loss_nv<CI>();
  double* dst[NV];
  for (int k = 0; k < 10; ++k) dst[k] = ws.acc + k;
  double* img = ws.acc + LA_FIXED + b * LA_IMG;
  for (int c = 0; c < CI; ++c) dst[10 + c] = img + c;
  for (int j = 0; j < 3; ++j) dst[10 + CI + j] = img + 3 + j;
  for (int k = 0; k < 3 * CI; ++k) dst[13 + CI + k] = img + 6 + k;
  block_sum_atomic<NV>(v, dst);
}

// pass 1, any shape: grid (chunks, B); CI = illumination channels (1 or 3)
template <int CI>
__global__ __launch_bounds__(256) void loss_pass1_kernel(const float* __restrict__ low, const float* __restrict__ enh,
                                                         const float* __restrict__ illu,
                                                         const float* __restrict__ refl, int H, int W, LossWS ws) {
  const int b = blockIdx.y;
  const int HW = H * W;
  const size_t base = (size_t)b * 3 * HW;
  const int per = (HW + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * per, p1 = min(HW, p0 + per);
  double v[loss_nv<CI>()] = {};
  const int ps = ws.ps, PH = H / ps, PW = W / ps;
  for (int q = p0 + threadIdx.x; q < p1; q += 256) {
    const int y = q / W, x = q - y * W;
    float ge, ed;
    loss_pixel1<CI>(low, enh, illu, refl, b, base, H, W, q, y, x, v, ge, ed);
    // exposure patches, edge row / column sums (per-pixel atomics on small arrays)
    // F.avg_pool2d(kernel = stride = ps): floor(H/ps) x floor(W/ps) patches, the remainder ignored
    if (y < PH * ps && x < PW * ps) atomicAdd(ws.patch + ((size_t)b * PH + y / ps) * PW + x / ps, (double)ge);
    if (x < W - 1) atomicAdd(ws.rowsum + (size_t)b * H + y, (double)ed);
    if (y < H - 1) atomicAdd(ws.colsum + (size_t)b * W + x, (double)ed);
  }
  loss_pass1_flush<CI>(v, ws, b);
}

// pass 1 on patch-row bands (H, W multiples of ps, ps a power of two <= 64):
// grid (ceil(W / 256), H / ps, B), one column per thread over the band's ps
// rows.  A patch is ps adjacent lanes of one wave (a shuffle sum, stored: each
// patch has one owner), a row's edge sum is a block sum (one atomic per row per
// 256 columns), a column's one atomic per band -- instead of the three fp64
// atomics per pixel of the generic pass (contended 256 / W / H ways; ~0.3 ms
// at 8 x 512 x 512)
template <int CI>
__global__ __launch_bounds__(256) void loss_pass1_band_kernel(const float* __restrict__ low,
                                                              const float* __restrict__ enh,
                                                              const float* __restrict__ illu,
                                                              const float* __restrict__ refl, int H, int W,
                                                              LossWS ws) {
  __shared__ double rowred[64][4];
  const int b = blockIdx.z, band = blockIdx.y, ps = ws.ps;
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t base = (size_t)b * 3 * H * W;
  const bool in = x < W;
  double v[loss_nv<CI>()] = {};
  double cpatch = 0.0, ccol = 0.0;
  for (int r = 0; r < ps; ++r) {
    const int y = band * ps + r;
    double red = 0.0;
    if (in) {
      float ge, ed;
      loss_pixel1<CI>(low, enh, illu, refl, b, base, H, W, y * W + x, y, x, v, ge, ed);
      cpatch += (double)ge;
      if (y < H - 1) ccol += (double)ed;
      if (x < W - 1) red = (double)ed;
    }
    for (int o = 32; o > 0; o >>= 1) red += __shfl_xor(red, o);
    if (lane == 0) rowred[r][wave] = red;
  }
  for (int o = ps / 2; o > 0; o >>= 1) cpatch += __shfl_xor(cpatch, o);
  if (in) {
    if ((x & (ps - 1)) == 0) ws.patch[((size_t)b * (H / ps) + band) * (W / ps) + x / ps] = cpatch;
    atomicAdd(ws.colsum + (size_t)b * W + x, ccol);
  }
  __syncthreads();
  if (threadIdx.x < ps) {
    const int t = threadIdx.x;
    atomicAdd(ws.rowsum + (size_t)b * H + band * ps + t, ((rowred[t][0] + rowred[t][1]) + rowred[t][2]) + rowred[t][3]);
  }
  loss_pass1_flush<CI>(v, ws, b);
}

// pass 2: edge-aware smoothness sums (needs the row / column edge means),
// summed over the CI illumination planes (the finaliser divides by CI)
template <int CI>
__global__ __launch_bounds__(256) void loss_pass2_kernel(const float* __restrict__ low, const float* __restrict__ illu,
                                                         int H, int W, LossWS ws) {
  const int b = blockIdx.y;
  const int HW = H * W;
  const size_t base = (size_t)b * 3 * HW;
  const int per = (HW + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * per, p1 = min(HW, p0 + per);
  double v[2] = {0.0, 0.0};
  for (int q = p0 + threadIdx.x; q < p1; q += 256) {
    const int y = q / W, x = q - y * W;
    const float* ip = illu + (size_t)b * CI * HW + q;
    if (x < W - 1) {
      float s = 0.f;
      for (int c = 0; c < 3; ++c) s += fabsf(low[base + c * HW + q] - low[base + c * HW + q + 1]);
      const float wh = expf(-ws.lam_s * (s / 3.f));
      const float ef = 1.f + ws.alpha * (float)(ws.rowsum[(size_t)b * H + y] / (W - 1));
#pragma unroll
      for (int c = 0; c < CI; ++c) v[0] += wh * ef * fabsf(ip[c * HW] - ip[c * HW + 1]);
    }
    if (y < H - 1) {
      float s = 0.f;
      for (int c = 0; c < 3; ++c) s += fabsf(low[base + c * HW + q] - low[base + c * HW + q + W]);
      const float wv = expf(-ws.lam_s * (s / 3.f));
      const float ef = 1.f + ws.alpha * (float)(ws.colsum[(size_t)b * W + x] / (H - 1));
#pragma unroll
      for (int c = 0; c < CI; ++c) v[1] += wv * ef * fabsf(ip[c * HW] - ip[c * HW + W]);
    }
  }
  double* dst[2] = {ws.acc + LA_SM_H, ws.acc + LA_SM_V};
  block_sum_atomic<2>(v, dst);
}

// texture complexity 'edge_density' (loss.py:549-577): per image, the share of
// pixels whose Sobel magnitude of gray(low) exceeds 1.5x the image mean.
// mode 0: per-image sum of magnitudes; mode 1: per-image count above threshold
__global__ __launch_bounds__(256) void edge_density_kernel(const float* __restrict__ low, int H, int W, LossWS ws,
                                                           int mode) {
  const int b = blockIdx.y;
  const int HW = H * W;
  const size_t base = (size_t)b * 3 * HW;
  const int per = (HW + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * per, p1 = min(HW, p0 + per);
  const float thr = mode ? (float)(ws.ed[b] / HW) * 1.5f : 0.f;
  double v[1] = {0.0};
  for (int q = p0 + threadIdx.x; q < p1; q += 256) {
    const int y = q / W, x = q - y * W;
    const float e = edge_at(low, base, H, W, y, x);
    v[0] += mode ? (e > thr ? 1.0 : 0.0) : (double)e;
  }
  double* dst[1] = {ws.ed + mode * gridDim.y + b};
  block_sum_atomic<1>(v, dst);
}

// calculate_texture_complexity (losses/loss.py:523-583) called on its own, for
// any channel count: img [B][C][H][W] fp32.  grid (chunks, B).
//   method 0 'tv':  acc[b] += sum |x[..,w] - x[..,w+1]|, acc[B+b] += sum |x[h] - x[h+1]|
//   method 1 'edge_density': gray = channel mean (torch.mean dim 1), reflect-
//     padded Sobel magnitude; mode 0 acc[b] += sum of magnitudes, mode 1
//     acc[B+b] += count of magnitudes > 1.5 * fp32 mean
__device__ __forceinline__ float gray_mean_c(const float* img, size_t base, int C, int HW, int q) {
  float s = img[base + q];
  for (int c = 1; c < C; ++c) s += img[base + (size_t)c * HW + q];
  return C > 1 ? s / (float)C : s;
}

__global__ __launch_bounds__(256) void texture_kernel(const float* __restrict__ img, int C, int H, int W, int method,
                                                      int mode, double* __restrict__ acc) {
  const int b = blockIdx.y, B = gridDim.y;
  const int HW = H * W;
  const size_t base = (size_t)b * C * HW;
  const int per = (HW + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * per, p1 = min(HW, p0 + per);
  double v[2] = {0.0, 0.0};
  const float thr = (method == 1 && mode == 1) ? (float)(acc[b] / HW) * 1.5f : 0.f;
  for (int q = p0 + threadIdx.x; q < p1; q += 256) {
    const int y = q / W, x = q - y * W;
    if (method == 0) {
      for (int c = 0; c < C; ++c) {
        const float* pl = img + base + (size_t)c * HW;
        const float a = pl[q];
        if (x + 1 < W) v[0] += fabsf(a - pl[q + 1]);
        if (y + 1 < H) v[1] += fabsf(a - pl[q + W]);
      }
    } else {
      float g[3][3];
      for (int dy = -1; dy <= 1; ++dy) {
        int yy = y + dy;
        yy = yy < 0 ? -yy : (yy >= H ? 2 * H - 2 - yy : yy);
        for (int dx = -1; dx <= 1; ++dx) {
          int xx = x + dx;
          xx = xx < 0 ? -xx : (xx >= W ? 2 * W - 2 - xx : xx);
          g[dy + 1][dx + 1] = gray_mean_c(img, base, C, HW, yy * W + xx);
        }
      }
      const float gx = -g[0][0] + g[0][2] - 2.f * g[1][0] + 2.f * g[1][2] - g[2][0] + g[2][2];
      const float gy = -g[0][0] - 2.f * g[0][1] - g[0][2] + g[2][0] + 2.f * g[2][1] + g[2][2];
      const float e = sqrtf(gx * gx + gy * gy);
      if (mode == 0) v[0] += (double)e;
      else v[1] += e > thr ? 1.0 : 0.0;
    }
  }
  double* dst[2] = {(method == 0 || mode == 0) ? acc + b : nullptr, (method == 0 || mode == 1) ? acc + B + b : nullptr};
  block_sum_atomic<2>(v, dst);
}

__global__ void texture_final_kernel(const double* __restrict__ acc, int B, int C, int H, int W, int method,
                                     float* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  if (method == 0) {
    // torch.mean per direction (fp32 results), then their fp32 sum
    const float th = (float)(acc[b] / ((double)C * H * (W - 1)));
    const float tv = (float)(acc[B + b] / ((double)C * (H - 1) * W));
    out[b] = th + tv;
  } else {
    out[b] = (float)(acc[B + b] / ((double)H * W));
  }
}

// finalise: one block
__global__ void loss_final_kernel(int B, int H, int W, LossWS ws, float* __restrict__ terms, int texture,
                                  float w_smooth, int CI) {
  __shared__ double ex[256];
  const int HW = H * W;
  const double N = (double)B * HW;
  // adaptive target base + (0.8 - base) * (1 - mean gray(low)) (loss.py:49)
  const double T = ws.base_exp + (0.8 - (double)ws.base_exp) * (1.0 - ws.acc[LA_GLOW] / N);
  const int NP = B * (H / ws.ps) * (W / ws.ps);
  const double parea = (double)ws.ps * ws.ps;
  double e = 0.0;
  for (int k = threadIdx.x; k < NP; k += blockDim.x) e += fabs(ws.patch[k] / parea - T);
  ex[threadIdx.x] = e;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) ex[threadIdx.x] += ex[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const double nh = (double)B * 3 * H * (W - 1), nv = (double)B * 3 * (H - 1) * W;
  const double nh1 = (double)B * H * (W - 1), nv1 = (double)B * (H - 1) * W;
  const double mu0 = ws.acc[0] / N, mu1 = ws.acc[1] / N, mu2 = ws.acc[2] / N;
  const double col = (mu0 - mu1) * (mu0 - mu1) + (mu0 - mu2) * (mu0 - mu2) + (mu1 - mu2) * (mu1 - mu2);
  const double spa = ws.acc[LA_SPA_H] / nh + ws.acc[LA_SPA_V] / nv;
  // smoothness: torch.mean over B x CI x H x (W-1) (loss.py:171-172)
  const double smo = (ws.acc[LA_SM_H] / nh1 + ws.acc[LA_SM_V] / nv1) / CI;
  double tc = ws.acc[LA_TV_H] / nh + ws.acc[LA_TV_V] / nv;
  if (texture == 1) {
    tc = 0.0;
    for (int b = 0; b < B; ++b) tc += ws.ed[B + b] / HW;
    tc /= B;
  }
  double wsm = (double)w_smooth;
  if (ws.dynamic) {  // loss.py:705-720
    wsm = (double)w_smooth * (1.0 - tc * 0.8);
    wsm = wsm < 0.1 ? 0.1 : (wsm > 5.0 ? 5.0 : wsm);
  }
  double frob = 0.0, md = 0.0;
  for (int b = 0; b < B; ++b) {
    const double* a = ws.acc + LA_FIXED + b * LA_IMG;  // [sI_c (3), sR_j (3), sIR_cj (9)]
    float* sc = ws.scal + LS_DEC + b * LS_IMG;
    if (CI == 1) {
      // loss.py:308-312: illumination expanded to 3 rows, NOT centred; each
      // row of the 3x3 covariance is the same cov_j -> Frobenius^2 = 3 sum_j cov_j^2;
      // mean term: mse of the channel means' means (:326-329)
      const double im = a[0] / HW;
      double rmm = 0.0;
      for (int j = 0; j < 3; ++j) {
        const double cov = (a[6 + j] - a[3 + j] * a[0] / HW) / (HW - 1);
        frob += 3.0 * cov * cov;
        sc[j] = (float)cov;
        rmm += a[3 + j] / HW / 3.0;
      }
      md += (im - rmm) * (im - rmm) / B;
      sc[9] = (float)(im - rmm);
      sc[12] = (float)im;
    } else {
      // loss.py:302-304: both centred, cov[c][j] over the 3x3 channel pairs;
      // mean term: F.mse_loss of the [B,3,1] means (:323-324)
      for (int c = 0; c < 3; ++c) {
        for (int j = 0; j < 3; ++j) {
          const double cov = (a[6 + c * 3 + j] - a[c] * a[3 + j] / HW) / (HW - 1);
          frob += cov * cov;
          sc[c * 3 + j] = (float)cov;
        }
        const double d = a[c] / HW - a[3 + c] / HW;
        md += d * d / (3.0 * B);
        sc[9 + c] = (float)d;
        sc[12 + c] = (float)(a[c] / HW);
      }
    }
  }
  const double dec = frob + (double)ws.lam_d * md;
  terms[0] = (float)(ex[0] / NP);
  terms[1] = (float)smo;
  terms[2] = (float)col;
  terms[3] = (float)spa;
  terms[4] = (float)dec;
  terms[8] = (float)wsm;
  ws.scal[LS_T] = (float)T;
  ws.scal[LS_NPATCH] = (float)NP;
  ws.scal[LS_WS] = (float)wsm;
  ws.scal[LS_MU + 0] = (float)mu0;
  ws.scal[LS_MU + 1] = (float)mu1;
  ws.scal[LS_MU + 2] = (float)mu2;
}

// gradient pass: one thread per pixel, overwrites g_enh / g_illu / g_refl
template <int CI>
__global__ __launch_bounds__(256) void loss_grad_kernel(const float* __restrict__ low, const float* __restrict__ enh,
                                                        const float* __restrict__ illu,
                                                        const float* __restrict__ refl, int B, int H, int W,
                                                        LossWS ws, float* __restrict__ g_enh,
                                                        float* __restrict__ g_illu, float* __restrict__ g_refl,
                                                        float w_exp, float w_col, float w_spa, float w_dec) {
  const int HW = H * W;
  const long long n = (long long)B * HW;
  const float T = ws.scal[LS_T];
  const float NP = ws.scal[LS_NPATCH];
  const float wsm = ws.scal[LS_WS];
  const float mu0 = ws.scal[LS_MU], mu1 = ws.scal[LS_MU + 1], mu2 = ws.scal[LS_MU + 2];
  const float N = (float)n;
  const float dcol[3] = {2.f * (mu0 - mu1) + 2.f * (mu0 - mu2), -2.f * (mu0 - mu1) + 2.f * (mu1 - mu2),
                         -2.f * (mu0 - mu2) - 2.f * (mu1 - mu2)};
  const float nh = (float)B * 3 * H * (W - 1), nv = (float)B * 3 * (H - 1) * W;
  const float nh1 = (float)B * H * (W - 1), nv1 = (float)B * (H - 1) * W;
  const int ps = ws.ps, PH = H / ps, PW = W / ps;
  const float parea = (float)(ps * ps);
  GSTRIDE(i, n) {
    const int b = (int)(i / HW), q = (int)(i - (long long)b * HW);
    const int y = q / W, x = q - y * W;
    const size_t base = (size_t)b * 3 * HW;
    // exposure: sign(P - T) / NP / ps^2 / 3 (pixels outside the pooled area: 0)
    float gexp = 0.f;
    if (y < PH * ps && x < PW * ps) {
      const float P = (float)(ws.patch[((size_t)b * PH + y / ps) * PW + x / ps] / parea);
      const float dp = P - T;
      gexp = w_exp * (dp > 0.f ? 1.f : (dp < 0.f ? -1.f : 0.f)) / NP / parea / 3.f;
    }
    for (int c = 0; c < 3; ++c) {
      const size_t k = base + c * HW + q;
      float g = gexp + w_col * dcol[c] / N;
      // spatial: d/de of mean((De - Dl)^2), horizontal and vertical
      const float e0 = enh[k], l0 = low[k];
      if (x < W - 1) g += w_spa * 2.f * ((e0 - enh[k + 1]) - (l0 - low[k + 1])) / nh;
      if (x > 0) g -= w_spa * 2.f * ((enh[k - 1] - e0) - (low[k - 1] - l0)) / nh;
      if (y < H - 1) g += w_spa * 2.f * ((e0 - enh[k + W]) - (l0 - low[k + W])) / nv;
      if (y > 0) g -= w_spa * 2.f * ((enh[k - W] - e0) - (low[k - W] - l0)) / nv;
      g_enh[k] = g;
    }
    // smoothness on each illumination plane (weight wsm; mean over CI planes)
    auto sgn = [](float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); };
    auto wgt = [&](int qa, int qb) {
      float s = 0.f;
      for (int c = 0; c < 3; ++c) s += fabsf(low[base + c * HW + qa] - low[base + c * HW + qb]);
      return expf(-ws.lam_s * (s / 3.f));
    };
    const float efh = 1.f + ws.alpha * (float)(ws.rowsum[(size_t)b * H + y] / (W - 1));
    const float efv = 1.f + ws.alpha * (float)(ws.colsum[(size_t)b * W + x] / (H - 1));
    const float wr = x < W - 1 ? wgt(q, q + 1) * efh : 0.f, wl = x > 0 ? wgt(q - 1, q) * efh : 0.f;
    const float wd = y < H - 1 ? wgt(q, q + W) * efv : 0.f, wu = y > 0 ? wgt(q - W, q) * efv : 0.f;
    const float* sc = ws.scal + LS_DEC + b * LS_IMG;
    const double* a = ws.acc + LA_FIXED + b * LA_IMG;
    const float inv = 1.f / (float)(HW - 1);
    float il[CI], r[3], rm[3];
#pragma unroll
    for (int c = 0; c < CI; ++c) il[c] = illu[((size_t)b * CI + c) * HW + q];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      r[j] = refl[base + j * HW + q];
      rm[j] = (float)(a[3 + j] / HW);
    }
#pragma unroll
    for (int c = 0; c < CI; ++c) {
      const size_t ii = ((size_t)b * CI + c) * HW + q;
      float gi = 0.f;
      if (x < W - 1) gi += wr * sgn(il[c] - illu[ii + 1]) / nh1;
      if (x > 0) gi -= wl * sgn(illu[ii - 1] - il[c]) / nh1;
      if (y < H - 1) gi += wd * sgn(il[c] - illu[ii + W]) / nv1;
      if (y > 0) gi -= wu * sgn(illu[ii - W] - il[c]) / nv1;
      gi *= wsm / CI;
      float gd = 0.f;
      if (CI == 1) {
        // 3 * sum_j cov_j^2 (uncentred I) + lam_d (imean - mean_j rmean_j)^2 / B
#pragma unroll
        for (int j = 0; j < 3; ++j) gd += 6.f * sc[j] * (r[j] - rm[j]) * inv;
        gd += ws.lam_d * 2.f * sc[9] / ((float)B * HW);
      } else {
        // sum_cj cov_cj^2 (centred) + lam_d sum_c (imean_c - rmean_c)^2 / (3B)
#pragma unroll
        for (int j = 0; j < 3; ++j) gd += 2.f * sc[c * 3 + j] * (r[j] - rm[j]) * inv;
        gd += ws.lam_d * 2.f * sc[9 + c] / (3.f * B * HW);
      }
      g_illu[ii] = gi + w_dec * gd;
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float g;
      if (CI == 1) {
        g = 6.f * sc[j] * (il[0] - sc[12]) * inv - ws.lam_d * 2.f * sc[9] / (B * 3.f * HW);
      } else {
        g = 0.f;
#pragma unroll
        for (int c = 0; c < CI; ++c) g += 2.f * sc[c * 3 + j] * (il[c] - sc[12 + c]) * inv;
        g -= ws.lam_d * 2.f * sc[9 + j] / (3.f * B * HW);
      }
      g_refl[base + j * HW + q] = w_dec * g;
    }
  }
}

__global__ void loss_total_kernel(float* t, float we, float wc, float wsp, float wd, float wp, float wf) {
  if (threadIdx.x == 0)
    t[7] = we * t[0] + t[8] * t[1] + wc * t[2] + wsp * t[3] + wd * t[4] + wp * t[5] + wf * t[6];
}

__global__ __launch_bounds__(256) void mse_kernel(const float* __restrict__ a, const float* __restrict__ b, long long n,
                                                  double* acc, float* g, float scale) {
  double v[1] = {0.0};
  GSTRIDE(i, n) {
    const float d = a[i] - b[i];
    v[0] += (double)d * d;
    if (g) g[i] = scale * 2.f * d;
  }
  v[0] /= (double)n;
  double* dst[1] = {acc};
  block_sum_atomic<1>(v, dst);
}

__constant__ float kVggMean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kVggStd[3] = {0.229f, 0.224f, 0.225f};

__global__ void vgg_norm_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int HW) {
  const long long n = (long long)B * HW;
  GSTRIDE(i, n) {
    const int b = (int)(i / HW), p = (int)(i - (long long)b * HW);
    for (int c = 0; c < 3; ++c) y[i * 3 + c] = (x[((size_t)b * 3 + c) * HW + p] - kVggMean[c]) / kVggStd[c];
  }
}

__global__ void vgg_norm_bwd_kernel(const float* __restrict__ gy, float* __restrict__ gx, int B, int HW) {
  const long long n = (long long)B * HW;
  GSTRIDE(i, n) {
    const int b = (int)(i / HW), p = (int)(i - (long long)b * HW);
    for (int c = 0; c < 3; ++c) gx[((size_t)b * 3 + c) * HW + p] += gy[i * 3 + c] / kVggStd[c];
  }
}

__global__ __launch_bounds__(256) void freq_kernel(const float2* __restrict__ ze, const float2* __restrict__ zl, int BC,
                                                   int H, int W, double* acc, float2* G, float scale, float w_high,
                                                   float w_low) {
  const long long n = (long long)BC * H * W;
  const int ch = H / 2, cw = W / 2, rad = min(H, W) / 4;
  double v[1] = {0.0};
  GSTRIDE(i, n) {
    const int q = (int)(i % ((long long)H * W));
    const int y = q / W, x = q - y * W;
    const float dist = sqrtf((float)((x - cw) * (x - cw)) + (float)((y - ch) * (y - ch)));
    const float w = dist <= (float)rad ? w_low : w_high;
    const float2 a = ze[i], c = zl[i];
    const float me = sqrtf(a.x * a.x + a.y * a.y), ml = sqrtf(c.x * c.x + c.y * c.y);
    const float d = me - ml;
    v[0] += (double)w * d * d;
    if (G) {
      const float k = me > 0.f ? scale * 2.f * w * d / me : 0.f;
      G[i] = make_float2(k * a.x, k * a.y);
    }
  }
  double* dst[1] = {acc};
  block_sum_atomic<1>(v, dst);
}

__global__ void add_real_kernel(const float2* __restrict__ z, float* g, long long n, float scale) {
  GSTRIDE(i, n) g[i] += scale * z[i].x;
}

__global__ void scale_acc_kernel(const double* __restrict__ acc, int n, float scale, float* out) {
  const int i = threadIdx.x;
  if (i < n) out[i] = (float)(acc[i] * scale);
}

// ---------------------------------------------------------------------------
// optimiser
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sqsum_kernel(const float* __restrict__ g, long long n, double* acc) {
  double v[1] = {0.0};
  GSTRIDE(i, n) v[0] += (double)g[i] * g[i];
  double* dst[1] = {acc};
  block_sum_atomic<1>(v, dst);
}

// GradScaler.unscale_ (torch.amp.GradScaler, train.py:84-86): g *= 1/scale and
// found_inf = 1 if any unscaled value is inf/nan (a benign same-value race)
__global__ __launch_bounds__(256) void unscale_kernel(float* __restrict__ g, long long n,
                                                      const float* __restrict__ scale, float* __restrict__ found_inf) {
  const float inv = 1.f / *scale;
  bool bad = false;
  GSTRIDE(i, n) {
    const float v = g[i] * inv;
    g[i] = v;
    bad |= !isfinite(v);
  }
  if (bad) *found_inf = 1.f;
}

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long long n, const double* __restrict__ sq, float max_norm,
                            float lr, float b1, float b2, float eps, float wd, float bc1, float bc2s,
                            float* norm_out) {
  const float norm = (float)sqrt(*sq);
  float coef = 1.f;
  if (max_norm > 0.f) coef = fminf(max_norm / (norm + 1e-6f), 1.f);
  if (norm_out && blockIdx.x == 0 && threadIdx.x == 0) *norm_out = norm;
  const float step = lr / bc1;
  GSTRIDE(i, n) {
    const float pv = p[i];
    const float gv = g[i] * coef + wd * pv;
    const float mv = b1 * m[i] + (1.f - b1) * gv;
    const float vv = b2 * v[i] + (1.f - b2) * gv * gv;
    m[i] = mv;
    v[i] = vv;
    p[i] = pv - step * mv / (sqrtf(vv) / bc2s + eps);
  }
}

}  // namespace upr

using namespace upr;

#define ST(s) ((hipStream_t)(s))

extern "C" {

int upr_t_zero(void* p, size_t bytes, void* stream) {
  if (!p && bytes) return UPR_ERR_ARG;
  if (!bytes) return UPR_OK;
  return (int)hipMemsetAsync(p, 0, bytes, ST(stream));
}

int upr_t_conv_direct(const UprView* x, int B, int H, int W, int Cin, const float* w, const float* bias, int Cout,
                      int kh, int kw, int stride, int pad, int dil, const UprView* y, int Ho, int Wo, int relu,
                      int accumulate, void* stream) {
  if (!x || !y || !x->data || !y->data || !w || B <= 0 || Cin <= 0 || Cout <= 0 || stride <= 0 || dil <= 0)
    return UPR_ERR_ARG;
  if (Ho != (H + 2 * pad - dil * (kh - 1) - 1) / stride + 1 || Wo != (W + 2 * pad - dil * (kw - 1) - 1) / stride + 1)
    return UPR_ERR_SHAPE;
  {
    const int rc = small_conv_fwd(x, B, H, W, Cin, w, bias, Cout, kh, kw, stride, pad, dil, y, Ho, Wo, relu,
                                  accumulate, ST(stream));
    if (rc != kErrUnsupported) return rc;
  }
  const long long n = (long long)B * Ho * Wo * Cout;
  if (Cin == 3 && kh == 3 && kw == 3 && stride == 1 && dil == 1) {
    hipLaunchKernelGGL(conv_direct_c3k3_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), mkv(x), B, H, W, w, bias,
                       Cout, pad, mkv(y), Ho, Wo, relu, accumulate);
    LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(conv_direct_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), mkv(x), B, H, W, Cin, w, bias,
                     Cout, kh, kw, stride, pad, dil, mkv(y), Ho, Wo, relu, accumulate);
  LAUNCH_CHECK();
}

int upr_t_conv_dgrad_c3_16(const void* dy16, int B, int H, int W, const float* w, int Cout, const UprView* dx,
                           int accumulate, void* stream) {
  if (!dy16 || !w || !dx || !dx->data || B <= 0 || H <= 0 || W <= 0) return UPR_ERR_ARG;
  const int rc = small_conv_dgrad_c3_16(dy16, B, H, W, w, Cout, dx, accumulate, ST(stream));
  return rc == kErrUnsupported ? UPR_ERR_UNSUPPORTED : rc;
}

int upr_t_conv_direct16(const UprView* x, int B, int H, int W, int Cin, const float* w, const float* bias, int Cout,
                        int kh, int kw, int stride, int pad, int dil, const UprView* y, int Ho, int Wo, int relu,
                        int accumulate, void* y16, int skip32, void* stream) {
  if (!x || !y || !x->data || !y->data || !w || !y16 || B <= 0 || Cin <= 0 || Cout <= 0 || stride <= 0 || dil <= 0)
    return UPR_ERR_ARG;
  if (Ho != (H + 2 * pad - dil * (kh - 1) - 1) / stride + 1 || Wo != (W + 2 * pad - dil * (kw - 1) - 1) / stride + 1)
    return UPR_ERR_SHAPE;
  if (skip32 && accumulate) return UPR_ERR_ARG;
  const int rc = small_conv_fwd(x, B, H, W, Cin, w, bias, Cout, kh, kw, stride, pad, dil, y, Ho, Wo, relu, accumulate,
                                ST(stream), y16, skip32);
  return rc == kErrUnsupported ? UPR_ERR_UNSUPPORTED : rc;
}

int upr_t_conv_direct_dgrad(const UprView* dy, int Ho, int Wo, const float* w, int B, int H, int W, int Cin, int Cout,
                            int kh, int kw, int stride, int pad, int dil, const UprView* dx, int accumulate,
                            void* stream) {
  if (!dy || !dx || !dy->data || !dx->data || !w || B <= 0 || stride <= 0 || dil <= 0) return UPR_ERR_ARG;
  {
    const int rc = small_conv_dgrad(dy, Ho, Wo, w, B, H, W, Cin, Cout, kh, kw, stride, pad, dil, dx, accumulate,
                                    ST(stream));
    if (rc != kErrUnsupported) return rc;
  }
  const long long n = (long long)B * H * W * Cin;
  hipLaunchKernelGGL(conv_direct_dgrad_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), mkv(dy), Ho, Wo, w, B, H,
                     W, Cin, Cout, kh, kw, stride, pad, dil, mkv(dx), accumulate);
  LAUNCH_CHECK();
}

int upr_t_conv_stem_wgrad_relu16(const UprView* x, const float* dy, const void* y16, int B, int H, int W, float* dw,
                                 float* dbias, void* stream) {
  if (!x || !dy || !y16 || !dw || !dbias || B <= 0 || H <= 0 || W <= 0) return UPR_ERR_ARG;
  const int rc = small_stem_wgrad_relu16(x, dy, y16, B, H, W, dw, dbias, ST(stream));
  return rc == kErrUnsupported ? UPR_ERR_UNSUPPORTED : rc;
}

int upr_t_conv_direct_wgrad_relu(const UprView* x, const UprView* dy, const UprView* y, int B, int H, int W, int Cin,
                                 int Ho, int Wo, int Cout, int kh, int kw, int stride, int pad, int dil, float* dw,
                                 float* dbias, void* stream) {
  if (!x || !dy || !y || !dw || B <= 0) return UPR_ERR_ARG;
  const int rc = small_conv_wgrad(x, dy, B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pad, dil, dw, dbias, ST(stream),
                                  y);
  return rc == kErrUnsupported ? UPR_ERR_UNSUPPORTED : rc;
}

int upr_t_conv_direct_wgrad(const UprView* x, const UprView* dy, int B, int H, int W, int Cin, int Ho, int Wo,
                            int Cout, int kh, int kw, int stride, int pad, int dil, float* dw, float* dbias,
                            void* stream) {
  if (!x || !dy || !dw || B <= 0) return UPR_ERR_ARG;
  {
    const int rc = small_conv_wgrad(x, dy, B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pad, dil, dw, dbias, ST(stream));
    if (rc != kErrUnsupported) return rc;
  }
  const int KC = kh * kw * Cin;
  const int nE = Cout * KC + (dbias ? Cout : 0);
  if (nE > 16 * 256) return UPR_ERR_UNSUPPORTED;
  int CH = 12288 / (Cout + KC);
  if (CH > 64) CH = 64;
  if (CH < 1) return UPR_ERR_UNSUPPORTED;
  const long long P = (long long)B * Ho * Wo;
  const int grid = grid_for(P, CH, 1024);
  const size_t lds = sizeof(float) * CH * (Cout + KC);
  hipLaunchKernelGGL(conv_direct_wgrad_kernel, dim3(grid), dim3(256), lds, ST(stream), mkv(x), mkv(dy), B, H, W, Cin,
                     Ho, Wo, Cout, kh, kw, stride, pad, dil, CH, dw, dbias);
  LAUNCH_CHECK();
}

int upr_t_conv_mfma(const float* x, int B, int H, int W, int Cin, int x_cs, int x_coff, const float* wp,
                    const float* bias, int N, int kh, int kw, int stride, int pad, int dil, const float* res,
                    int res_cs, int relu, float* y, int y_cs, int y_coff, int store, void* stream) {
  if (!x || !wp || !y || B <= 0 || Cin % 32 || N % 32 || Cin <= 0 || N <= 0) return UPR_ERR_ARG;
  if (kh <= 0 || kw <= 0 || stride <= 0 || dil <= 0 || pad < 0) return UPR_ERR_ARG;
  if (x_cs % 4 || x_coff % 4 || y_cs % 4 || y_coff % 4 || (res && res_cs % 4)) return UPR_ERR_ARG;
  if (store == 1 && ((N / 4) % 32)) return UPR_ERR_SHAPE;
  const int Ho = (H + 2 * pad - dil * (kh - 1) - 1) / stride + 1;
  const int Wo = (W + 2 * pad - dil * (kw - 1) - 1) / stride + 1;
  if (Ho <= 0 || Wo <= 0) return UPR_ERR_SHAPE;
  ConvOp c;
  memset(&c, 0, sizeof(c));
  c.nseg = 1;
  ConvSeg& s = c.seg[0];
  s.src = x; s.C = Cin; s.cs = x_cs; s.coff = x_coff; s.Hin = H; s.Win = W;
  s.kh = kh; s.kw = kw; s.stride = stride; s.pad = pad; s.dil = dil; s.pre = kPreNone; s.kbase = 0;
  c.B = B; c.Ho = Ho; c.Wo = Wo; c.N = N; c.Kpad = kh * kw * Cin;
  c.W = wp; c.bias = bias; c.res1 = res; c.res1_cs = res_cs; c.relu = relu;
  c.out = y; c.out_cs = y_cs; c.out_coff = y_coff; c.store = store == 1 ? kStoreConvT2x2 : kStoreNHWC;
  return launch_conv(c, kF32, ST(stream));
}

// ---- autocast (AMP) convs: fp16 operands, fp32 accumulate, fp32 activations ----
// x[m][coff + c] (fp32, pixel stride cs) -> dense fp16 [m][C], 8 channels per thread
__global__ __launch_bounds__(256) void cast_act_f16_kernel(const float* __restrict__ x, long long M, int C, int cs,
                                                           int coff, half_t* __restrict__ y) {
  const int C8 = C / 8;
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  if (256 % C8 == 0) {  // fixed channels per thread, rows by addition (no 64-bit div per element)
    const int c = (threadIdx.x % C8) * 8, rpb = 256 / C8;
    for (long long m = (long long)blockIdx.x * rpb + threadIdx.x / C8; m < M; m += (long long)gridDim.x * rpb) {
      const float4* src = (const float4*)(x + m * cs + coff + c);
      const float4 a = src[0], b = src[1];
      *(h8*)(y + m * C + c) =
          h8{(half_t)a.x, (half_t)a.y, (half_t)a.z, (half_t)a.w, (half_t)b.x, (half_t)b.y, (half_t)b.z, (half_t)b.w};
    }
    return;
  }
  GSTRIDE(i, M * C8) {
    const long long m = i / C8;
    const int c = (int)(i - m * C8) * 8;
    const float4* src = (const float4*)(x + m * cs + coff + c);
    const float4 a = src[0], b = src[1];
    h8 o = {(half_t)a.x, (half_t)a.y, (half_t)a.z, (half_t)a.w, (half_t)b.x, (half_t)b.y, (half_t)b.z, (half_t)b.w};
    *(h8*)(y + m * C + c) = o;
  }
}
// dense fp16 [m][C] -> y[m][coff + c] (fp32) (+ res[m * res_cs + c], fp32; res may alias y)
__global__ __launch_bounds__(256) void cast_act_f32_kernel(const half_t* __restrict__ x, long long M, int C,
                                                           const float* res, int res_cs, float* y, int cs, int coff,
                                                           int xcs) {
  const int C4 = C / 4;
  GSTRIDE(i, M * C4) {
    const long long m = i / C4;
    const int c = (int)(i - m * C4) * 4;
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const h4 v = *(const h4*)(x + m * xcs + c);
    float4 o = make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
    if (res) {
      const float4 r = *(const float4*)(res + m * res_cs + c);
      o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
    }
    *(float4*)(y + m * cs + coff + c) = o;
  }
}
__global__ __launch_bounds__(256) void cast_f16_kernel(const float* __restrict__ x, long long n, half_t* __restrict__ y) {
  GSTRIDE(i, n) y[i] = (half_t)x[i];
}

int upr_t_cast_f16(const float* x, void* y, size_t n, void* stream) {
  if (!x || !y) return UPR_ERR_ARG;
  hipLaunchKernelGGL(cast_f16_kernel, dim3(grid_for((long long)n)), dim3(256), 0, ST(stream), x, (long long)n,
                     (half_t*)y);
  LAUNCH_CHECK();
}

// UPR_T_OUT32=0: fp16 conv output + separate fp32 cast pass (A/B timing)

int upr_t_conv_mfma16(const float* x, int B, int H, int W, int Cin, int x_cs, int x_coff, const void* wp16,
                      const float* bias, int N, int kh, int kw, int stride, int pad, int dil, const float* res,
                      int res_cs, int relu, float* y, int y_cs, int y_coff, int store, void* x16, int x16_ready,
                      void* y16, int y16_cs, void* stream) {
  if (!x16 || !wp16 || !y || !y16 || B <= 0 || Cin % 32 || N % 32 || Cin <= 0 || N <= 0) return UPR_ERR_ARG;
  if (!x16_ready && !x) return UPR_ERR_ARG;
  const bool want16 = (store & 2) != 0;  // y16 must end up holding (half)y
  const bool only16 = want16 && (store & 4) != 0;  // y itself not needed (written only on the fallback path)
  // the 1x1 stride-2 conv's input gradient (y = 2H x 2W, accumulated into at the even pixels)
  const bool s2 = (store & 8) != 0;
  // the 3x3 stride-2 pad-1 conv's input gradient from dy itself (x16 = dy over H x W, wp16 the
  // flipped filter, y = 2H x 2W); UPR_ERR_UNSUPPORTED when the kernel does not take the shape
  const bool s2dg = (store & 16) != 0;
  // the ready x16 keeps x's channel stride (a slice of a concat's fp16 copy)
  const bool x16_strided = (store & 32) != 0;
  store &= 1;
  if (x16_strided && (!x16_ready || x_cs % 8 || x_cs < Cin || (uintptr_t)x16 % 16)) return UPR_ERR_ARG;
  if (s2 && (kh != 1 || kw != 1 || stride != 1 || pad != 0 || dil != 1 || store != 0 || !res || relu)) return UPR_ERR_ARG;
  if (s2dg && (s2 || kh != 3 || kw != 3 || stride != 1 || dil != 1 || store != 0 || relu || bias)) return UPR_ERR_ARG;
  const int ycs16 = y16_cs > 0 ? y16_cs : (store == 1 ? N / 4 : N);  // y16's channel stride
  if (ycs16 % 8 || ((uintptr_t)y16 & 15)) return UPR_ERR_ARG;
  if (kh <= 0 || kw <= 0 || stride <= 0 || dil <= 0 || pad < 0) return UPR_ERR_ARG;
  if (x_cs % 4 || x_coff % 4 || y_cs % 4 || y_coff % 4 || (res && res_cs % 4)) return UPR_ERR_ARG;
  if (res && relu) return UPR_ERR_ARG;  // the residual is added in fp32 after the fp16 GEMM
  if (store == 1 && ((N / 4) % 32)) return UPR_ERR_SHAPE;
  const int Ho = (H + 2 * pad - dil * (kh - 1) - 1) / stride + 1;
  const int Wo = (W + 2 * pad - dil * (kw - 1) - 1) / stride + 1;
  if (Ho <= 0 || Wo <= 0) return UPR_ERR_SHAPE;
  hipStream_t st = ST(stream);
  const long long Mi = (long long)B * H * W;
  ConvOp c;
  memset(&c, 0, sizeof(c));
  c.nseg = 1;
  ConvSeg& s = c.seg[0];
  s.src = x16; s.C = Cin; s.cs = x16_strided ? x_cs : Cin; s.coff = 0; s.Hin = H; s.Win = W;
  s.kh = kh; s.kw = kw; s.stride = stride; s.pad = pad; s.dil = dil; s.pre = kPreNone; s.kbase = 0;
  c.B = B; c.Ho = Ho; c.Wo = Wo; c.N = N; c.Kpad = kh * kw * Cin;
  c.W = wp16; c.bias = bias; c.relu = relu;
  c.store = store == 1 ? kStoreConvT2x2 : kStoreNHWC;
  // the fp32 output (+ fp32 residual / accumulated gradient) straight from the conv epilogue
  ConvOp c32 = c;
  c32.out32 = y; c32.out32_cs = y_cs; c32.out32_coff = y_coff;
  c32.res32 = res; c32.res32_cs = res_cs;
  if (want16) { c32.out32_h16 = y16; c32.out32_h16_cs = ycs16; }
  c32.skip32 = only16 ? 1 : 0;
  c32.out_s2 = s2 ? 1 : 0;
  ConvOp cdg = c;
  if (s2dg) {
    cdg.Ho = 2 * H; cdg.Wo = 2 * W;
    cdg.out32 = y; cdg.out32_cs = y_cs; cdg.out32_coff = y_coff;
    cdg.res32 = res; cdg.res32_cs = res_cs;
    if (want16) { cdg.out32_h16 = y16; cdg.out32_h16_cs = ycs16; }
    cdg.skip32 = only16 ? 1 : 0;
  }
  // the forms only one kernel implements decline BEFORE the operand cast is queued
  if (s2dg && launch_conv_s2dg(cdg, st, true) == kErrUnsupported) return UPR_ERR_UNSUPPORTED;
  if (s2 && launch_conv_pw(c32, st, true) == kErrUnsupported) return UPR_ERR_UNSUPPORTED;
  if (!x16_ready) {
    if ((uintptr_t)x % 16 || x_cs % 8 || x_coff % 8) return UPR_ERR_ARG;
    hipLaunchKernelGGL(cast_act_f16_kernel, dim3(grid_for(Mi * (Cin / 8))), dim3(256), 0, st, x, Mi, Cin, x_cs, x_coff,
                       (half_t*)x16);
    UPR_CHECK_HIP(hipGetLastError());
  }
  if (s2dg) {
    const int rc = launch_conv_s2dg(cdg, st);
    if (rc == kErrUnsupported) return UPR_ERR_UNSUPPORTED;
    if (rc != 0) return rc;
    LAUNCH_CHECK();
  }
  {
    const int rc = launch_conv_out32(c32, st);
    if (rc != kErrUnsupported) {
      if (rc != 0) return rc;
      LAUNCH_CHECK();
    }
    if (s2) return UPR_ERR_UNSUPPORTED;  // no other kernel scatters at stride 2
  }
  c.out = y16; c.out_cs = ycs16; c.out_coff = 0;
  const int rc = launch_conv(c, kF16, st);
  if (rc != 0) return rc;
  const long long Mo = store == 1 ? (long long)B * 4 * Ho * Wo : (long long)B * Ho * Wo;
  const int Co = store == 1 ? N / 4 : N;
  hipLaunchKernelGGL(cast_act_f32_kernel, dim3(grid_for(Mo * (Co / 4))), dim3(256), 0, st, (const half_t*)y16, Mo, Co,
                     res, res_cs, y, y_cs, y_coff, ycs16);
  LAUNCH_CHECK();
}

int upr_t_conv_mfma16_relu_bwd(const void* x16, int B, int H, int W, int Cin, const void* wp16, int N, int kh, int kw,
                               int pad, int dil, float* y, int y_cs, int y_coff, void* y16, int y16_cs,
                               const void* mask16, int mask16_cs, int skip32, void* stream) {
  return upr_t_conv_mfma16_relu_bwd_cs(x16, Cin, B, H, W, Cin, wp16, N, kh, kw, pad, dil, y, y_cs, y_coff, y16, y16_cs,
                                       mask16, mask16_cs, skip32, stream);
}

int upr_t_conv_mfma16_relu_bwd_cs(const void* x16, int x16_cs, int B, int H, int W, int Cin, const void* wp16, int N,
                                  int kh, int kw, int pad, int dil, float* y, int y_cs, int y_coff, void* y16,
                                  int y16_cs, const void* mask16, int mask16_cs, int skip32, void* stream) {
  if (!x16 || !wp16 || !y || !y16 || !mask16 || B <= 0 || Cin % 32 || N % 32 || Cin <= 0 || N <= 0) return UPR_ERR_ARG;
  if (kh <= 0 || kw <= 0 || dil <= 0 || pad < 0 || x16_cs < Cin) return UPR_ERR_ARG;
  if (((uintptr_t)x16 | (uintptr_t)y16 | (uintptr_t)mask16) % 16 || y16_cs % 8 || mask16_cs % 8 || y_cs % 4 ||
      y_coff % 4 || (uintptr_t)y % 16 || x16_cs % 8)
    return UPR_ERR_UNSUPPORTED;
  const int Ho = H + 2 * pad - dil * (kh - 1), Wo = W + 2 * pad - dil * (kw - 1);
  if (Ho <= 0 || Wo <= 0) return UPR_ERR_SHAPE;
  ConvOp c;
  memset(&c, 0, sizeof(c));
  c.nseg = 1;
  ConvSeg& sg = c.seg[0];
  sg.src = x16; sg.C = Cin; sg.cs = x16_cs; sg.coff = 0; sg.Hin = H; sg.Win = W;
  sg.kh = kh; sg.kw = kw; sg.stride = 1; sg.pad = pad; sg.dil = dil; sg.pre = kPreNone; sg.kbase = 0;
  c.B = B; c.Ho = Ho; c.Wo = Wo; c.N = N; c.Kpad = kh * kw * Cin;
  c.W = wp16; c.bias = nullptr; c.relu = 0;
  c.store = kStoreNHWC;
  c.out32 = y; c.out32_cs = y_cs; c.out32_coff = y_coff;
  c.out32_h16 = y16; c.out32_h16_cs = y16_cs;
  c.mask16 = mask16; c.mask16_cs = mask16_cs; c.skip32 = skip32 ? 1 : 0;
  const int rc = launch_conv_out32(c, ST(stream));
  if (rc == kErrUnsupported) return UPR_ERR_UNSUPPORTED;
  if (rc != 0) return rc;
  LAUNCH_CHECK();
}

int upr_t_conv_wgrad(const float* x, int B, int H, int W, int Cin, int x_cs, int x_coff, const float* dy, int Ho,
                     int Wo, int Cout, int dy_cs, int dy_coff, int kh, int kw, int stride, int pad, int dil,
                     float* dwp, void* stream) {
  if (!x || !dy || !dwp || B <= 0 || Cin % 32 || Cout % 32 || Cin <= 0 || Cout <= 0) return UPR_ERR_ARG;
  {
    const int rc = wgrad_gemm(x, B, H, W, Cin, x_cs, x_coff, dy, Ho, Wo, Cout, dy_cs, dy_coff, kh, kw, stride, pad, dil,
                              dwp, ST(stream));
    if (rc != kErrUnsupported) return rc;
  }
  const long long P = (long long)B * Ho * Wo;
  const long long chunks = (P + WG_PPB - 1) / WG_PPB;
  if (chunks > 0x7fffffff) return UPR_ERR_SHAPE;
  dim3 grid((unsigned)chunks, Cout / 32, kh * kw * (Cin / 32));
  hipLaunchKernelGGL(conv_wgrad_kernel, grid, dim3(256), 0, ST(stream), x, B, H, W, Cin, x_cs, x_coff, dy, Ho, Wo,
                     Cout, dy_cs, dy_coff, kh, kw, stride, pad, dil, dwp);
  LAUNCH_CHECK();
}

int upr_t_conv_wgrad16(const float* x, const void* x16, int B, int H, int W, int Cin, int x_cs, int x_coff,
                       const float* dy, int Ho, int Wo, int Cout, int dy_cs, int dy_coff, int kh, int kw, int stride,
                       int pad, int dil, float* dwp, void* stream) {
  if ((!x && !x16) || !dy || !dwp || B <= 0 || Cin % 32 || Cout % 32 || Cin <= 0 || Cout <= 0) return UPR_ERR_ARG;
  hipStream_t st = ST(stream);
  const bool fits = Wo % 64 == 0 && dy_cs % 4 == 0 && dy_coff % 4 == 0 && (uintptr_t)dy % 16 == 0 &&
                    (uintptr_t)dwp % 16 == 0 && (x16 || (x && x_cs % 8 == 0 && x_coff % 8 == 0 && (uintptr_t)x % 16 == 0));
  if (fits) {
    void* tmp = nullptr;
    const void* src = x16;
    if (!src) {
      const long long Mi = (long long)B * H * W;
      tmp = scratch(kSlotCast, (size_t)Mi * Cin * sizeof(half_t), st);
      if (!tmp) return (int)hipErrorOutOfMemory;
      hipLaunchKernelGGL(cast_act_f16_kernel, dim3(grid_for(Mi * (Cin / 8))), dim3(256), 0, st, x, Mi, Cin, x_cs, x_coff,
                         (half_t*)tmp);
      src = tmp;
    }
    const int rc = wgrad16_gemm(src, B, H, W, Cin, dy, Ho, Wo, Cout, dy_cs, dy_coff, kh, kw, stride, pad, dil, dwp, st);
    if (rc != kErrUnsupported) return rc;
  }
  if (!x) return UPR_ERR_ARG;
  return upr_t_conv_wgrad(x, B, H, W, Cin, x_cs, x_coff, dy, Ho, Wo, Cout, dy_cs, dy_coff, kh, kw, stride, pad, dil, dwp,
                          stream);
}

int upr_t_conv_wgrad_into(const float* x, const void* x16, int B, int H, int W, int Cin, int x_cs, int x_coff,
                          const float* dy, const void* dy16, int Ho, int Wo, int Cout, int dy_cs, int dy_coff, int kh,
                          int kw, int stride, int pad, int dil, float* dw, void* stream) {
  if ((!x && !x16) || !dy || !dw || B <= 0 || Cin % 32 || Cout % 32 || Cin <= 0 || Cout <= 0) return UPR_ERR_ARG;
  hipStream_t st = ST(stream);
  if (x16) {
    const int rc = wgrad16_gemm(x16, B, H, W, Cin, dy, Ho, Wo, Cout, dy_cs, dy_coff, kh, kw, stride, pad, dil, dw, st,
                                Cin, dy16);
    if (rc != kErrUnsupported) return rc;
  }
  if (!x) return UPR_ERR_ARG;
  {
    const int rc = wgrad_gemm(x, B, H, W, Cin, x_cs, x_coff, dy, Ho, Wo, Cout, dy_cs, dy_coff, kh, kw, stride, pad, dil,
                              dw, st, Cin);
    if (rc != kErrUnsupported) return rc;
  }
  // any other shape: the packed form into scratch, then added in PyTorch's layout
  const size_t n = (size_t)Cout * Cin * kh * kw;
  float* tmp = nullptr;
  tmp = (float*)scratch(kSlotTmp, n * sizeof(float), st);
  if (!tmp) return (int)hipErrorOutOfMemory;
  UPR_CHECK_HIP(hipMemsetAsync(tmp, 0, n * sizeof(float), st));
  int rc = x16 ? upr_t_conv_wgrad16(x, x16, B, H, W, Cin, x_cs, x_coff, dy, Ho, Wo, Cout, dy_cs, dy_coff, kh, kw, stride,
                                    pad, dil, tmp, stream)
               : upr_t_conv_wgrad(x, B, H, W, Cin, x_cs, x_coff, dy, Ho, Wo, Cout, dy_cs, dy_coff, kh, kw, stride, pad,
                                  dil, tmp, stream);
  if (rc == UPR_OK) rc = upr_t_unpack_grad(tmp, dw, Cout, Cin, kh, kw, 0, 1, stream);
  return rc;
}

int upr_t_pack_weight(const float* w, float* out, int Co, int Ci, int kh, int kw, int mode, void* stream) {
  if (!w || !out || Co <= 0 || Ci <= 0 || mode < 0 || mode > 3) return UPR_ERR_ARG;
  if (mode >= 2 && (kh != 2 || kw != 2)) return UPR_ERR_SHAPE;
  const long long n = (long long)Co * Ci * kh * kw;
  hipLaunchKernelGGL(pack_weight_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), w, out, Co, Ci, kh, kw, mode);
  LAUNCH_CHECK();
}

int upr_t_pack_weights(const UprPackJob* jobs, int njobs, int max_n, void* stream) {
  if (!jobs || njobs < 0 || max_n < 0 || njobs > 65535) return UPR_ERR_ARG;
  if (njobs == 0 || max_n == 0) return UPR_OK;
  const int gx = (max_n + 255) / 256 < 64 ? (max_n + 255) / 256 : 64;
  hipLaunchKernelGGL(pack_batch_kernel, dim3(gx, njobs), dim3(256), 0, ST(stream), jobs);
  LAUNCH_CHECK();
}

int upr_t_unpack_grad(const float* gp, float* g, int Co, int Ci, int kh, int kw, int mode, int accumulate,
                      void* stream) {
  if (!gp || !g || (mode != 0 && mode != 3)) return UPR_ERR_ARG;
  const long long n = (long long)Co * Ci * kh * kw;
  hipLaunchKernelGGL(unpack_grad_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), gp, g, Co, Ci, kh, kw, mode,
                     accumulate);
  LAUNCH_CHECK();
}

int upr_t_zero_upsample(const float* dy, int B, int Ho, int Wo, int C, int dy_cs, int dy_coff, float* z,
                        void* stream) {
  if (!dy || !z) return UPR_ERR_ARG;
  const long long n = (long long)B * 4 * Ho * Wo * C;
  hipLaunchKernelGGL(zero_upsample_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), dy, B, Ho, Wo, C, dy_cs,
                     dy_coff, z);
  LAUNCH_CHECK();
}

int upr_t_bn_stats(const float* x, int M, int C, int cs, int coff, double* acc, void* stream) {
  if (!x || !acc || M <= 0 || C <= 0) return UPR_ERR_ARG;
  if (reduce4_ok(C, cs, coff, x))
    return chan_reduce2(x, cs, coff, (const float*)nullptr, 0, 0, nullptr, nullptr, nullptr, nullptr, M, C, 0,
                        acc + 2 * C, acc, nullptr, 0, ST(stream));
  // the atomic fallback adds into acc: cleared here, so every path overwrites
  UPR_CHECK_HIP(hipMemsetAsync(acc, 0, sizeof(double) * 2 * C, ST(stream)));
  hipLaunchKernelGGL(chan_reduce_kernel, dim3(reduce_grid(M)), dim3(256), 0, ST(stream), x, cs, coff, nullptr, 0, 0,
                     nullptr, nullptr, M, C, 0, acc, nullptr);
  LAUNCH_CHECK();
}

int upr_t_bn_finalize(const double* acc, int M, int C, float momentum, float eps, float* running_mean,
                      float* running_var, int64_t* nbt, float* mean, float* invstd, void* stream) {
  if (!acc || !mean || !invstd || M <= 0) return UPR_ERR_ARG;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, ST(stream), acc, M, C, momentum, eps,
                     running_mean, running_var, (long long*)nbt, mean, invstd);
  LAUNCH_CHECK();
}

int upr_t_bn_eval_stats(const float* running_mean, const float* running_var, int C, float eps, float* mean,
                        float* invstd, void* stream) {
  if (!running_mean || !running_var || !mean || !invstd || C <= 0) return UPR_ERR_ARG;
  hipLaunchKernelGGL(bn_eval_stats_kernel, dim3((C + 255) / 256), dim3(256), 0, ST(stream), running_mean, running_var, C,
                     eps, mean, invstd);
  LAUNCH_CHECK();
}

int upr_t_bn_apply16(const float* x, int M, int C, int x_cs, int x_coff, const float* mean, const float* invstd,
                     const float* gamma, const float* beta, const float* res, int res_cs, int res_coff, int res_post,
                     int relu, float* y, int y_cs, int y_coff, void* y16, void* stream) {
  if (!x || !y || !mean || !invstd || !gamma || !beta) return UPR_ERR_ARG;
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  const bool v4 = C % 4 == 0 && x_cs % 4 == 0 && x_coff % 4 == 0 && y_cs % 4 == 0 && y_coff % 4 == 0 && a16(x) &&
                  a16(y) && (!res || (res_cs % 4 == 0 && res_coff % 4 == 0 && a16(res))) &&
                  (!y16 || ((uintptr_t)y16 & 7) == 0);
  if (v4) {
    const long long n4 = (long long)M * (C / 4);
    hipLaunchKernelGGL(bn_apply4_kernel<float>, dim3(grid_for(n4)), dim3(256), 0, ST(stream), x, M, C, x_cs, x_coff, mean,
                       invstd, gamma, beta, res, res_cs, res_coff, res_post, relu, y, y_cs, y_coff, (half_t*)y16);
    LAUNCH_CHECK();
  }
  if (y16) return UPR_ERR_ARG;  // the fp16 copy needs the vectorised layout
  const long long n = (long long)M * C;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), x, M, C, x_cs, x_coff, mean,
                     invstd, gamma, beta, res, res_cs, res_coff, res_post, relu, y, y_cs, y_coff);
  LAUNCH_CHECK();
}

int upr_t_bn_apply(const float* x, int M, int C, int x_cs, int x_coff, const float* mean, const float* invstd,
                   const float* gamma, const float* beta, const float* res, int res_cs, int res_coff, int res_post,
                   int relu, float* y, int y_cs, int y_coff, void* stream) {
  return upr_t_bn_apply16(x, M, C, x_cs, x_coff, mean, invstd, gamma, beta, res, res_cs, res_coff, res_post, relu, y,
                          y_cs, y_coff, nullptr, stream);
}

int upr_t_bn_bwd_reduce(const float* g, int g_cs, int g_coff, const float* x, int x_cs, int x_coff, const float* mean,
                        const float* invstd, int M, int C, double* acc, void* stream) {
  if (!g || !x || !acc) return UPR_ERR_ARG;
  if (reduce4_ok(C, g_cs, g_coff, g) && reduce4_ok(C, x_cs, x_coff, x))
    return chan_reduce2(g, g_cs, g_coff, x, x_cs, x_coff, mean, invstd, nullptr, nullptr, M, C, 1, acc + 2 * C, acc,
                        nullptr, 0, ST(stream));
  else
    hipLaunchKernelGGL(chan_reduce_kernel, dim3(reduce_grid(M)), dim3(256), 0, ST(stream), g, g_cs, g_coff, x, x_cs,
                       x_coff, mean, invstd, M, C, 1, acc, nullptr);
  LAUNCH_CHECK();
}

int upr_t_bn_bwd_apply(const float* g, int g_cs, int g_coff, const float* x, int x_cs, int x_coff, const float* mean,
                       const float* invstd, const float* gamma, const double* acc, int M, int C, float* dgamma,
                       float* dbeta, float* dx, int dx_cs, int dx_coff, int accumulate, int batch_stats,
                       void* stream) {
  if (!g || !x || !acc || !dx || !gamma) return UPR_ERR_ARG;
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (C % 4 == 0 && g_cs % 4 == 0 && g_coff % 4 == 0 && x_cs % 4 == 0 && x_coff % 4 == 0 && dx_cs % 4 == 0 &&
      dx_coff % 4 == 0 && a16(g) && a16(x) && a16(dx)) {
    const long long n4 = (long long)M * (C / 4);
    hipLaunchKernelGGL((bn_bwd_apply4_kernel<float, float>), dim3(grid_for(n4)), dim3(256), 0, ST(stream), g, g_cs, g_coff, x, x_cs,
                       x_coff, mean, invstd, gamma, acc, M, C, dgamma, dbeta, dx, dx_cs, dx_coff, accumulate,
                       batch_stats);
    LAUNCH_CHECK();
  }
  const long long n = (long long)M * C;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), g, g_cs, g_coff, x, x_cs,
                     x_coff, mean, invstd, gamma, acc, M, C, dgamma, dbeta, dx, dx_cs, dx_coff, accumulate,
                       batch_stats);
  LAUNCH_CHECK();
}

int upr_t_bn_bwd_fused(const float* g, int g_cs, int g_coff, const float* x, int x_cs, const float* mean,
                       const float* invstd, const float* gamma, const float* beta, int relu, int M, int C,
                       double* acc, float* dgamma, float* dbeta, float* dx, int dx_cs, int dx_coff, int accumulate,
                       int batch_stats, void* dx16, void* stream) {
  if (!g || !x || !acc || !dx || !gamma || !beta || !mean || !invstd || M <= 0 || C <= 0) return UPR_ERR_ARG;
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (C % 4 || C > 1024 || g_cs % 4 || g_coff % 4 || x_cs % 4 || dx_cs % 4 || dx_coff % 4 || !a16(g) || !a16(x) ||
      !a16(dx) || !a16(mean) || !a16(invstd) || !a16(gamma) || !a16(beta) || ((uintptr_t)dx16 & 7))
    return UPR_ERR_UNSUPPORTED;
  hipStream_t st = ST(stream);
  const int rc = chan_reduce2(g, g_cs, g_coff, x, x_cs, 0, mean, invstd, gamma, beta, M, C, relu ? 3 : 1, acc + 2 * C,
                              acc, nullptr, 0, st);
  if (rc) return rc;
  const long long n4 = (long long)M * (C / 4);
  hipLaunchKernelGGL((bn_bwd_apply4_kernel<float, float>), dim3(grid_for(n4)), dim3(256), 0, st, g, g_cs, g_coff, x, x_cs, 0, mean,
                     invstd, gamma, acc, M, C, dgamma, dbeta, dx, dx_cs, dx_coff, accumulate, batch_stats, beta, relu,
                     (half_t*)dx16);
  LAUNCH_CHECK();
}

// x read from its compact fp16 copy x16 ([M][C]; under autocast the BN input
// is an fp16 conv's output, whose fp32 form holds the same values)
int upr_t_bn_stats16(const void* x16, int M, int C, double* acc, void* stream) {
  if (!x16 || !acc || M <= 0 || C <= 0) return UPR_ERR_ARG;
  if (C % 4 || C > 1024 || (uintptr_t)x16 % 8) return UPR_ERR_UNSUPPORTED;
  return chan_reduce2((const half_t*)x16, C, 0, (const float*)nullptr, 0, 0, nullptr, nullptr, nullptr, nullptr, M, C,
                      0, acc + 2 * C, acc, nullptr, 0, ST(stream));
}

// chan_fin (mode 0) and bn_finalize in one launch: a block owns 32 channels,
// lanes 0-31 their sums and 32-63 their sums of squares (the same slot order
// and partial-sum tree as chan_fin: bit-identical acc), then lanes 0-31
// finalise their channel as bn_finalize_kernel does
__global__ __launch_bounds__(256) void chan_fin_bn_kernel(const double* __restrict__ part, int slots, int C,
                                                          double* __restrict__ acc, int M, float momentum, float eps,
                                                          float* __restrict__ rm, float* __restrict__ rv,
                                                          long long* nbt, float* __restrict__ mean,
                                                          float* __restrict__ invstd) {
  __shared__ double red[4][64];
  __shared__ double fin[64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 32 + (lane & 31);
  const bool ok = c < C;
  const int t = lane < 32 ? c : C + c;
  double sum = 0.0;  // (chan_fin_kernel's order and batching)
  if (ok) {
    for (int k0 = w; k0 < slots; k0 += 64) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int k = k0 + 4 * u;
        v[u] = k < slots ? part[(size_t)k * 2 * C + t] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) sum += v[u];
    }
  }
  red[w][lane] = sum;
  __syncthreads();
  if (w == 0) {
    const double v = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    fin[lane] = v;
    if (ok) acc[t] = v;
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  if (w != 0 || lane >= 32 || !ok) return;
  const double mu = fin[lane] / M;
  double var = fin[lane + 32] / M - mu * mu;
  if (var < 0) var = 0;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rm) rm[c] = (1.f - momentum) * rm[c] + momentum * (float)mu;
  if (rv) {
    const double unb = M > 1 ? var * M / (M - 1) : var;
    rv[c] = (1.f - momentum) * rv[c] + momentum * (float)unb;
  }
}

int upr_t_bn_stats16_fin(const void* x16, int M, int C, double* acc, float momentum, float eps, float* running_mean,
                         float* running_var, int64_t* nbt, float* mean, float* invstd, void* stream) {
  if (!x16 || !acc || !mean || !invstd || M <= 0 || C <= 0) return UPR_ERR_ARG;
  if (C % 4 || C > 1024 || (uintptr_t)x16 % 8) return UPR_ERR_UNSUPPORTED;
  hipStream_t st = ST(stream);
  const int R = kRedThreads / (C / 4);
  int slots = M / (R * 16);
  slots = slots < 1 ? 1 : (slots > kRedSlots ? kRedSlots : slots);
  double* part = acc + 2 * C;
  hipLaunchKernelGGL((chan_part_kernel<half_t, float>), dim3(slots), dim3(kRedThreads),
                     (size_t)R * 2 * C * sizeof(double), st, (const half_t*)x16, C, 0, (const float*)nullptr, 0, 0,
                     nullptr, nullptr, nullptr, nullptr, M, C, 0, part);
  UPR_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(chan_fin_bn_kernel, dim3((C + 31) / 32), dim3(256), 0, st, (const double*)part, slots, C, acc, M,
                     momentum, eps, running_mean, running_var, (long long*)nbt, mean, invstd);
  LAUNCH_CHECK();
}

int upr_t_bn_apply16h_cs(const void* x16, int M, int C, const float* mean, const float* invstd, const float* gamma,
                         const float* beta, const float* res, int res_cs, int res_coff, int res_post, int relu,
                         float* y, int y_cs, int y_coff, void* y16, int y16_cs, int skip32, void* stream) {
  if (!x16 || !y || !mean || !invstd || !gamma || !beta || M <= 0 || C <= 0) return UPR_ERR_ARG;
  if (skip32 && !y16) return UPR_ERR_ARG;
  if (y16_cs < 0 || (y16_cs > 0 && y16_cs < C)) return UPR_ERR_ARG;
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (C % 4 || (uintptr_t)x16 % 8 || y_cs % 4 || y_coff % 4 || !a16(y) ||
      (res && (res_cs % 4 || res_coff % 4 || !a16(res))) || ((uintptr_t)y16 & 7) || y16_cs % 4)
    return UPR_ERR_UNSUPPORTED;
  const long long n4 = (long long)M * (C / 4);
  hipLaunchKernelGGL(bn_apply4_kernel<half_t>, dim3(grid_for(n4)), dim3(256), 0, ST(stream), (const half_t*)x16, M, C,
                     C, 0, mean, invstd, gamma, beta, res, res_cs, res_coff, res_post, relu, y, y_cs, y_coff,
                     (half_t*)y16, skip32, y16_cs);
  LAUNCH_CHECK();
}

int upr_t_bn_apply16h(const void* x16, int M, int C, const float* mean, const float* invstd, const float* gamma,
                      const float* beta, const float* res, int res_cs, int res_coff, int res_post, int relu, float* y,
                      int y_cs, int y_coff, void* y16, int skip32, void* stream) {
  return upr_t_bn_apply16h_cs(x16, M, C, mean, invstd, gamma, beta, res, res_cs, res_coff, res_post, relu, y, y_cs,
                              y_coff, y16, 0, skip32, stream);
}

int upr_t_bn_bwd_fused16(const float* g, const void* g16, int g_cs, int g_coff, const void* x16, const float* mean,
                         const float* invstd, const float* gamma, const float* beta, int relu, int M, int C,
                         double* acc, float* dgamma, float* dbeta, float* dx, int dx_cs, int dx_coff, int accumulate,
                         int batch_stats, void* dx16, int skip32, void* stream) {
  if ((!g && !g16) || !x16 || !acc || !dx || !gamma || !beta || !mean || !invstd || M <= 0 || C <= 0)
    return UPR_ERR_ARG;
  if (skip32 && (accumulate || !dx16)) return UPR_ERR_ARG;
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (C % 4 || C > 1024 || dx_cs % 4 || dx_coff % 4 || (uintptr_t)x16 % 8 || !a16(dx) || !a16(mean) ||
      !a16(invstd) || !a16(gamma) || !a16(beta) || ((uintptr_t)dx16 & 7))
    return UPR_ERR_UNSUPPORTED;
  if (g16 ? (uintptr_t)g16 % 8 != 0 : (g_cs % 4 || g_coff % 4 || !a16(g))) return UPR_ERR_UNSUPPORTED;
  hipStream_t st = ST(stream);
  const long long n4 = (long long)M * (C / 4);
  if (g16) {  // g = the input-gradient conv's fp16 output (compact [M][C])
    const int rc = chan_reduce2((const half_t*)g16, C, 0, (const half_t*)x16, C, 0, mean, invstd, gamma, beta, M, C,
                                relu ? 3 : 1, acc + 2 * C, acc, nullptr, 0, st);
    if (rc) return rc;
    hipLaunchKernelGGL((bn_bwd_apply4_kernel<half_t, half_t>), dim3(grid_for(n4)), dim3(256), 0, st,
                       (const half_t*)g16, C, 0, (const half_t*)x16, C, 0, mean, invstd, gamma, acc, M, C, dgamma,
                       dbeta, dx, dx_cs, dx_coff, accumulate, batch_stats, beta, relu, (half_t*)dx16, skip32);
    LAUNCH_CHECK();
  }
  const int rc = chan_reduce2(g, g_cs, g_coff, (const half_t*)x16, C, 0, mean, invstd, gamma, beta, M, C,
                              relu ? 3 : 1, acc + 2 * C, acc, nullptr, 0, st);
  if (rc) return rc;
  hipLaunchKernelGGL((bn_bwd_apply4_kernel<half_t, float>), dim3(grid_for(n4)), dim3(256), 0, st, g, g_cs, g_coff,
                     (const half_t*)x16, C, 0, mean, invstd, gamma, acc, M, C, dgamma, dbeta, dx, dx_cs, dx_coff,
                     accumulate, batch_stats, beta, relu, (half_t*)dx16, skip32);
  LAUNCH_CHECK();
}

int upr_t_zero_upsample16(const float* dy, int B, int Ho, int Wo, int C, int dy_cs, int dy_coff, void* z16,
                          void* stream) {
  if (!dy || !z16 || C % 8 || dy_cs % 4 || dy_coff % 4 || ((uintptr_t)dy & 15) || ((uintptr_t)z16 & 15))
    return UPR_ERR_ARG;
  const long long n = (long long)B * 4 * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(zero_upsample16_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), dy, B, Ho, Wo, C, dy_cs,
                     dy_coff, (half_t*)z16);
  LAUNCH_CHECK();
}

int upr_t_zero_upsample16h(const void* dy16, int B, int Ho, int Wo, int C, void* z16, void* stream) {
  if (!dy16 || !z16 || C % 8 || ((uintptr_t)dy16 & 15) || ((uintptr_t)z16 & 15)) return UPR_ERR_ARG;
  const long long n = (long long)B * 4 * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(zero_upsample16h_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), (const half_t*)dy16, B, Ho,
                     Wo, C, (half_t*)z16, n);
  LAUNCH_CHECK();
}

int upr_t_chan_sum(const float* g, int M, int C, int cs, int coff, float* out, int accumulate, void* stream) {
  if (!g || !out) return UPR_ERR_ARG;
  if (!accumulate) UPR_CHECK_HIP(hipMemsetAsync(out, 0, sizeof(float) * C, ST(stream)));
  if (reduce4_ok(C, cs, coff, g)) {
    hipLaunchKernelGGL(chan_reduce4_kernel, dim3(reduce_grid(M)), dim3(256), 0, ST(stream), g, cs, coff, nullptr, 0, 0,
                       nullptr, nullptr, M, C, 2, nullptr, out);
    LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(chan_reduce_kernel, dim3(reduce_grid(M)), dim3(256), 0, ST(stream), g, cs, coff, nullptr, 0, 0,
                     nullptr, nullptr, M, C, 2, nullptr, out);
  LAUNCH_CHECK();
}

int upr_t_chan_sum_ws(const float* g, int M, int C, int cs, int coff, float* out, int accumulate, double* ws,
                      void* stream) {
  if (!g || !out || !ws || M <= 0 || C <= 0) return UPR_ERR_ARG;
  if (!reduce4_ok(C, cs, coff, g)) return upr_t_chan_sum(g, M, C, cs, coff, out, accumulate, stream);
  return chan_reduce2(g, cs, coff, (const float*)nullptr, 0, 0, nullptr, nullptr, nullptr, nullptr, M, C, 2, ws, nullptr, out,
                      accumulate, ST(stream));
}

int upr_t_chan_sum16(const void* g16, int M, int C, float* out, int accumulate, double* ws, void* stream) {
  if (!g16 || !out || !ws || M <= 0 || C <= 0) return UPR_ERR_ARG;
  if (C % 4 || C > 1024 || (uintptr_t)g16 % 8) return UPR_ERR_UNSUPPORTED;
  return chan_reduce2((const half_t*)g16, C, 0, (const float*)nullptr, 0, 0, nullptr, nullptr, nullptr, nullptr, M, C,
                      2, ws, nullptr, out, accumulate, ST(stream));
}

int upr_t_chan_sum16s(const void* g16, int M, int C, int cs, float* out, int accumulate, double* ws, void* stream) {
  if (!g16 || !out || !ws || M <= 0 || C <= 0 || cs < C) return UPR_ERR_ARG;
  if (C % 4 || C > 1024 || cs % 4 || (uintptr_t)g16 % 8) return UPR_ERR_UNSUPPORTED;
  return chan_reduce2((const half_t*)g16, cs, 0, (const float*)nullptr, 0, 0, nullptr, nullptr, nullptr, nullptr, M, C,
                      2, ws, nullptr, out, accumulate, ST(stream));
}

int upr_t_reduce_acc_doubles(int C) { return 2 * C * (1 + kRedSlots); }

int upr_t_relu_mask(float* g, int g_cs, int g_coff, const float* y, int y_cs, int y_coff, int M, int C,
                    void* stream) {
  if (!g || !y) return UPR_ERR_ARG;
  if (C % 4 == 0 && g_cs % 4 == 0 && g_coff % 4 == 0 && y_cs % 4 == 0 && y_coff % 4 == 0 && ((uintptr_t)g & 15) == 0 &&
      ((uintptr_t)y & 15) == 0) {
    const long long n4 = (long long)M * (C / 4);
    hipLaunchKernelGGL(relu_mask4_kernel, dim3(grid_for(n4)), dim3(256), 0, ST(stream), g, g_cs, g_coff, y, y_cs,
                       y_coff, M, C);
    LAUNCH_CHECK();
  }
  const long long n = (long long)M * C;
  hipLaunchKernelGGL(relu_mask_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), g, g_cs, g_coff, y, y_cs, y_coff,
                     M, C);
  LAUNCH_CHECK();
}

int upr_t_relu_mask16(float* g, int g_cs, int g_coff, const float* y, int y_cs, int y_coff, int M, int C, void* g16,
                      int write32, void* stream) {
  if (!g || !y || !g16) return UPR_ERR_ARG;
  if (C % 4 || g_cs % 4 || g_coff % 4 || y_cs % 4 || y_coff % 4 || ((uintptr_t)g & 15) || ((uintptr_t)y & 15) ||
      ((uintptr_t)g16 & 7) || (long long)M * C >= (1LL << 31))
    return UPR_ERR_UNSUPPORTED;
  const int n = M * (C / 4);
  if (n == 0) return UPR_OK;
  hipLaunchKernelGGL(relu_mask16_kernel<float>, dim3((n + 255) / 256), dim3(256), 0, ST(stream), g, g_cs, g_coff, y,
                     y_cs, y_coff, M, C / 4, (half_t*)g16, write32);
  LAUNCH_CHECK();
}

int upr_t_relu_mask16h(float* g, int g_cs, int g_coff, const void* y16, int y16_cs, int M, int C, void* g16,
                       int write32, void* stream) {
  if (!g || !y16 || !g16) return UPR_ERR_ARG;
  if (C % 4 || g_cs % 4 || g_coff % 4 || y16_cs % 4 || ((uintptr_t)g & 15) || ((uintptr_t)y16 & 7) ||
      ((uintptr_t)g16 & 7) || (long long)M * C >= (1LL << 31))
    return UPR_ERR_UNSUPPORTED;
  const int n = M * (C / 4);
  if (n == 0) return UPR_OK;
  hipLaunchKernelGGL(relu_mask16_kernel<half_t>, dim3((n + 255) / 256), dim3(256), 0, ST(stream), g, g_cs, g_coff,
                     (const half_t*)y16, y16_cs, 0, M, C / 4, (half_t*)g16, write32);
  LAUNCH_CHECK();
}

int upr_t_copy(const UprView* src, const UprView* dst, int B, int H, int W, int C, int accumulate, void* stream) {
  if (!src || !dst || !src->data || !dst->data) return UPR_ERR_ARG;
  const long long n = (long long)B * H * W * C;
  if (n == 0) return UPR_OK;
  if (vec4_view_ok(src, B, H, W, C) && vec4_view_ok(dst, B, H, W, C)) {
    const int nv = (int)(n / 4);
    hipLaunchKernelGGL(copy4_kernel, dim3((nv + 255) / 256), dim3(256), 0, ST(stream), mkv4(src), mkv4(dst), H, W,
                       C / 4, nv, accumulate, (half_t*)nullptr, 0);
    LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(copy_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), mkv(src), mkv(dst), B, H, W, C,
                     accumulate);
  LAUNCH_CHECK();
}

int upr_t_pointwise(const float* a, const float* b, float* out, size_t n, int op, const uint8_t* mask_in,
                    uint8_t* mask_out, float p, uint64_t seed, void* stream) {
  if (!a || !out || op < 0 || op > 5) return UPR_ERR_ARG;
  if ((op == 1 || op == 4 || op == 5) && !b) return UPR_ERR_ARG;
  if ((op == 2 && !mask_out) || (op == 3 && !mask_in)) return UPR_ERR_ARG;
  if (n == 0) return UPR_OK;
  hipLaunchKernelGGL(pointwise_kernel, dim3(grid_for((long long)n)), dim3(256), 0, ST(stream), a, b, out,
                     (long long)n, op, mask_in, mask_out, p, (unsigned long long)seed);
  LAUNCH_CHECK();
}

int upr_t_maxpool(const UprView* x, int B, int H, int W, int C, int k, int s, int p, const UprView* y, int Ho, int Wo,
                  void* stream) {
  return upr_t_maxpool_code(x, B, H, W, C, k, s, p, y, Ho, Wo, nullptr, nullptr, stream);
}

// Max-pool backward as two deterministic passes (the atomic scatter above --
// up to k*k fp32 atomics per input element in arbitrary order -- stays behind
// UPR_MAXPOOL_BWD_SCATTER=1 for A/B timing):
//  1. per output element the window position of its max, PyTorch's rule
//     (max_pool2d CPU kernel: the first in-bounds tap, then every tap with
//     v > max or v NaN), as a byte code ky * k + kx;
//  2. per input element, in output order, the dy of every window whose code
//     points at it, added to dx.
extern "C++" {
template <int VEC>
__global__ void maxpool_arg_kernel(V x, int B, int H, int W, int C, int k, int s, int p, int Ho, int Wo,
                                   unsigned char* __restrict__ code) {
  const int CV = C / VEC;
  const long long n = (long long)B * Ho * Wo * CV;
  GSTRIDE(i, n) {
    const int c = (int)(i % CV) * VEC;
    long long r = i / CV;
    const int ox = (int)(r % Wo); r /= Wo;
    const int oy = (int)(r % Ho);
    const int b = (int)(r / Ho);
    float m[VEC];
    int best[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) { m[v] = -INFINITY; best[v] = -1; }
    for (int ky = 0; ky < k; ++ky) {
      const int iy = oy * s - p + ky;
      if (iy < 0 || iy >= H) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int ix = ox * s - p + kx;
        if (ix < 0 || ix >= W) continue;
        float val[VEC];
        if constexpr (VEC == 4) {
          const float4 q = *(const float4*)(x.d + x.at(b, iy, ix, c));
          val[0] = q.x; val[1] = q.y; val[2] = q.z; val[3] = q.w;
        } else {
          val[0] = x.d[x.at(b, iy, ix, c)];
        }
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          if (best[v] < 0) best[v] = ky * k + kx;  // the first in-bounds tap is the default index
          if (val[v] > m[v] || isnan(val[v])) {
            m[v] = val[v];
            best[v] = ky * k + kx;
          }
        }
      }
    }
    unsigned char* o = code + (((long long)b * Ho + oy) * Wo + ox) * C + c;
#pragma unroll
    for (int v = 0; v < VEC; ++v) o[v] = (unsigned char)(best[v] < 0 ? 255 : best[v]);
  }
}

template <int VEC>
__global__ void maxpool_bwd_gather_kernel(const unsigned char* __restrict__ code, V dy, int B, int H, int W, int C, int k,
                                          int s, int p, int Ho, int Wo, V dx) {
  const int CV = C / VEC;
  const long long n = (long long)B * H * W * CV;
  GSTRIDE(i, n) {
    const int c = (int)(i % CV) * VEC;
    long long r = i / CV;
    const int ix = (int)(r % W); r /= W;
    const int iy = (int)(r % H);
    const int b = (int)(r / H);
    float* dp = dx.d + dx.at(b, iy, ix, c);
    float acc[VEC];
    if constexpr (VEC == 4) {
      const float4 q = *(const float4*)dp;
      acc[0] = q.x; acc[1] = q.y; acc[2] = q.z; acc[3] = q.w;
    } else {
      acc[0] = *dp;
    }
    // windows containing (iy, ix): oy*s - p <= iy <= oy*s - p + k - 1
    const int oy0 = max(0, (iy + p - k + 1 + s - 1 + s * k) / s - k), oy1 = min(Ho - 1, (iy + p) / s);
    const int ox0 = max(0, (ix + p - k + 1 + s - 1 + s * k) / s - k), ox1 = min(Wo - 1, (ix + p) / s);
    for (int oy = oy0; oy <= oy1; ++oy) {
      const int ty = iy - (oy * s - p);
      if (ty < 0 || ty >= k) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int tx = ix - (ox * s - p);
        if (tx < 0 || tx >= k) continue;
        const unsigned char want = (unsigned char)(ty * k + tx);
        const unsigned char* cd = code + (((long long)b * Ho + oy) * Wo + ox) * C + c;
        const float* g = dy.d + dy.at(b, oy, ox, c);
#pragma unroll
        for (int v = 0; v < VEC; ++v)
          if (cd[v] == want) acc[v] += g[v * dy.sc];
      }
    }
    if constexpr (VEC == 4) {
      *(float4*)dp = make_float4(acc[0], acc[1], acc[2], acc[3]);
    } else {
      *dp = acc[0];
    }
  }
}

// Fast paths for the two pools of the training step -- EnhancedFAM's 3x3/1/1
// (models/model.py:32) and the VGG 2x2/2 (losses/loss.py perceptual
// features[4], [9], [18]) -- on channel-contiguous views: 4 channels per
// thread, 32-bit index math (the generic kernels' 64-bit div/mod per element
// ran at <1 TB/s), compile-time windows.  The forward optionally writes the
// argmax byte codes (PyTorch's rule, as maxpool_arg_kernel) so the backward
// is the gather alone.
// TI = half_t: the input is an activation's compact fp16 copy (the autocast
// VGG activations live in fp16 only, as the reference's under autocast)
template <int K, int S, int P, typename TI = float>
__global__ __launch_bounds__(256) void maxpool4_kernel(const TI* __restrict__ x, int xsb, int xsh, int xsw, int H,
                                                       int W, int CV, int Ho, int Wo, int n, float* __restrict__ y,
                                                       int ysb, int ysh, int ysw, unsigned* __restrict__ code,
                                                       half_t* __restrict__ y16) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int c = (i % CV) * 4;
  int r = i / CV;
  const int ox = r % Wo;
  r /= Wo;
  const int oy = r % Ho, b = r / Ho;
  float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int best[4] = {-1, -1, -1, -1};
  const TI* xb = x + b * xsb + c;
#pragma unroll
  for (int ky = 0; ky < K; ++ky) {
    const int iy = oy * S - P + ky;
    if ((unsigned)iy >= (unsigned)H) continue;
#pragma unroll
    for (int kx = 0; kx < K; ++kx) {
      const int ix = ox * S - P + kx;
      if ((unsigned)ix >= (unsigned)W) continue;
      const float4 q = ld4f(xb + iy * xsh + ix * xsw);
      const float val[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if (best[v] < 0) best[v] = ky * K + kx;
        if (val[v] > m[v] || isnan(val[v])) {
          m[v] = val[v];
          best[v] = ky * K + kx;
        }
      }
    }
  }
  if (y) *(float4*)(y + b * ysb + oy * ysh + ox * ysw + c) = make_float4(m[0], m[1], m[2], m[3]);
  if (y16) {  // compact [b][oy][ox][C] fp16 copy: element index 4 i
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    *(h4*)(y16 + (size_t)i * 4) = h4{(half_t)m[0], (half_t)m[1], (half_t)m[2], (half_t)m[3]};
  }
  if (code) {
    unsigned w = 0;
#pragma unroll
    for (int v = 0; v < 4; ++v) w |= (unsigned)(best[v] < 0 ? 255 : best[v]) << (8 * v);
    code[i] = w;
  }
}

// dx[b][iy][ix][c..c+3] += dy of every window (ascending oy, then ox: the
// generic gather's order) whose code points at (iy, ix).  O16: the result
// goes to the compact fp16 g16 instead (element 4 i), masked by the producing
// ReLU's fp16 output y16 when given -- the frozen VGG's pool backward, whose
// only reader is the masked fp16 dgrad operand (relu_mask16h fused away)
template <int K, int S, int P, int O16 = 0>
__global__ __launch_bounds__(256) void maxpool_gather4_kernel(const unsigned* __restrict__ code,
                                                              const float* __restrict__ dy, int dsb, int dsh, int dsw,
                                                              int H, int W, int CV, int Ho, int Wo, int n,
                                                              float* __restrict__ dx, int xsb, int xsh, int xsw,
                                                              int accumulate, const half_t* __restrict__ y16 = nullptr,
                                                              half_t* __restrict__ g16 = nullptr) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int cv = i % CV, c = cv * 4;
  int r = i / CV;
  const int ix = r % W;
  r /= W;
  const int iy = r % H, b = r / H;
  float* dp = O16 ? nullptr : dx + b * xsb + iy * xsh + ix * xsw + c;
  float4 acc = !O16 && accumulate ? *(const float4*)dp : make_float4(0.f, 0.f, 0.f, 0.f);
  // every window's code word and gradient run is loaded first (independent
  // loads, one round trip each; a window outside the output reads nothing and
  // gets the no-hit code 0xffffffff), then the hits are added in the same
  // window order as before (the 3x3 pool's code -> dy -> next window chain
  // was 18 dependent round trips per thread: 1.6 TB/s at 512^2)
  unsigned wv[K * K];
  float4 gv[K * K];
#pragma unroll
  for (int t = 0; t < K; ++t) {
    const int ky = K - 1 - t, ny = iy + P - ky;  // oy * S
    const bool oky = ny >= 0 && ny % S == 0 && ny / S < Ho;
    const int oy = oky ? ny / S : 0;
#pragma unroll
    for (int u = 0; u < K; ++u) {
      const int kx = K - 1 - u, nx = ix + P - kx;
      const bool ok = oky && nx >= 0 && nx % S == 0 && nx / S < Wo;
      const int ox = ok ? nx / S : 0;
      wv[t * K + u] = ok ? code[((b * Ho + oy) * Wo + ox) * CV + cv] : 0xffffffffu;
      gv[t * K + u] = ok ? *(const float4*)(dy + b * dsb + oy * dsh + ox * dsw + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
#pragma unroll
  for (int t = 0; t < K; ++t) {
    const int ky = K - 1 - t;
#pragma unroll
    for (int u = 0; u < K; ++u) {
      const int kx = K - 1 - u;
      const unsigned want = (unsigned)(ky * K + kx) * 0x01010101u;
      const unsigned hit = wv[t * K + u] ^ want;  // a zero byte marks a window whose max sits here
      const float4 g = gv[t * K + u];
      if ((hit & 0xffu) == 0) acc.x += g.x;
      if ((hit & 0xff00u) == 0) acc.y += g.y;
      if ((hit & 0xff0000u) == 0) acc.z += g.z;
      if ((hit & 0xff000000u) == 0) acc.w += g.w;
    }
  }
  if (O16) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    if (y16) {
      const h4 y = *(const h4*)(y16 + (size_t)i * 4);
      if (!(y[0] > (half_t)0)) acc.x = 0.f;
      if (!(y[1] > (half_t)0)) acc.y = 0.f;
      if (!(y[2] > (half_t)0)) acc.z = 0.f;
      if (!(y[3] > (half_t)0)) acc.w = 0.f;
    }
    *(h4*)(g16 + (size_t)i * 4) = h4{(half_t)acc.x, (half_t)acc.y, (half_t)acc.z, (half_t)acc.w};
    return;
  }
  *(float4*)dp = acc;
}

}  // extern "C++"

int upr_t_maxpool_bwd(const UprView* x, const UprView* dy, int B, int H, int W, int C, int k, int s, int p, int Ho,
                      int Wo, const UprView* dx, void* stream) {
  if (!x || !dy || !dx || k <= 0 || s <= 0 || k * k > 255) return UPR_ERR_ARG;
  hipStream_t st = ST(stream);
  const long long n = (long long)B * Ho * Wo * C;
  void* code = nullptr;
  code = scratch(kSlotCode, (size_t)n, st);
  if (!code) return (int)hipErrorOutOfMemory;
  const bool v4 = C % 4 == 0 && x->sc == 1 && dx->sc == 1 && (uintptr_t)x->data % 16 == 0 &&
                  (uintptr_t)dx->data % 16 == 0 && x->sw % 4 == 0 && x->sh % 4 == 0 && x->sb % 4 == 0 &&
                  dx->sw % 4 == 0 && dx->sh % 4 == 0 && dx->sb % 4 == 0;
  const long long ni = (long long)B * H * W * C;
  if (v4) {
    hipLaunchKernelGGL(maxpool_arg_kernel<4>, dim3(grid_for(n / 4)), dim3(256), 0, st, mkv(x), B, H, W, C, k, s, p, Ho,
                       Wo, (unsigned char*)code);
    hipLaunchKernelGGL(maxpool_bwd_gather_kernel<4>, dim3(grid_for(ni / 4)), dim3(256), 0, st,
                       (const unsigned char*)code, mkv(dy), B, H, W, C, k, s, p, Ho, Wo, mkv(dx));
  } else {
    hipLaunchKernelGGL(maxpool_arg_kernel<1>, dim3(grid_for(n)), dim3(256), 0, st, mkv(x), B, H, W, C, k, s, p, Ho, Wo,
                       (unsigned char*)code);
    hipLaunchKernelGGL(maxpool_bwd_gather_kernel<1>, dim3(grid_for(ni)), dim3(256), 0, st, (const unsigned char*)code,
                       mkv(dy), B, H, W, C, k, s, p, Ho, Wo, mkv(dx));
  }
  UPR_CHECK_HIP(hipGetLastError());
  return UPR_OK;
}

__global__ void zero_view_kernel(V v, int B, int H, int W, int C) {
  const long long n = (long long)B * H * W * C;
  GSTRIDE(i, n) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int x = (int)(r % W);
    r /= W;
    v.d[v.at((int)(r / H), (int)(r % H), x, c)] = 0.f;
  }
}

// shape of a fast-path pool: (k, s, p) one of the two instantiated windows,
// channel-contiguous 16-byte aligned views whose extents fit 32-bit offsets
static int pool_fast_kind(int k, int s, int p) {
  if (k == 3 && s == 1 && p == 1) return 1;
  if (k == 2 && s == 2 && p == 0) return 2;
  return 0;
}

int upr_t_maxpool_code(const UprView* x, int B, int H, int W, int C, int k, int s, int p, const UprView* y, int Ho,
                       int Wo, unsigned char* code, void* y16, void* stream) {
  if (!x || !y || k <= 0 || s <= 0 || k * k > 255) return UPR_ERR_ARG;
  hipStream_t st = ST(stream);
  const long long n = (long long)B * Ho * Wo * C;
  if (n == 0) return UPR_OK;
  const int kind = pool_fast_kind(k, s, p);
  if (kind && vec4_view_ok(x, B, H, W, C) && vec4_view_ok(y, B, Ho, Wo, C) && (uintptr_t)code % 4 == 0 &&
      (uintptr_t)y16 % 8 == 0 && n < (1LL << 31)) {
    const int nv = (int)(n / 4), CV = C / 4;
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((nv + 255) / 256), dim3(256), 0, st, (const float*)x->data, (int)x->sb,
                         (int)x->sh, (int)x->sw, H, W, CV, Ho, Wo, nv, (float*)y->data, (int)y->sb, (int)y->sh,
                         (int)y->sw, (unsigned*)code, (half_t*)y16);
    };
    if (kind == 1) go(maxpool4_kernel<3, 1, 1>);
    else go(maxpool4_kernel<2, 2, 0>);
    LAUNCH_CHECK();
  }
  if (y16) return UPR_ERR_UNSUPPORTED;  // the fp16 copy comes with the 4-channel path only
  hipLaunchKernelGGL(maxpool_kernel, dim3(grid_for(n)), dim3(256), 0, st, mkv(x), B, H, W, C, k, s, p, mkv(y), Ho, Wo);
  if (code)
    hipLaunchKernelGGL(maxpool_arg_kernel<1>, dim3(grid_for(n)), dim3(256), 0, st, mkv(x), B, H, W, C, k, s, p, Ho,
                       Wo, code);
  LAUNCH_CHECK();
}

int upr_t_maxpool16_code(const void* x16, int B, int H, int W, int C, int k, int s, int p, const UprView* y, int Ho,
                         int Wo, unsigned char* code, void* y16, void* stream) {
  if (!x16 || !y || k <= 0 || s <= 0 || k * k > 255) return UPR_ERR_ARG;
  if (!y->data && !y16) return UPR_ERR_ARG;  // y->data NULL: the fp16 copy only (its values are exact)
  const long long n = (long long)B * Ho * Wo * C;
  if (n == 0) return UPR_OK;
  const int kind = pool_fast_kind(k, s, p);
  if (!kind || C % 4 || (uintptr_t)x16 % 8 || !vec4_view_ok(y, B, Ho, Wo, C) || (uintptr_t)code % 4 ||
      (uintptr_t)y16 % 8 || (long long)B * H * W * C >= (1LL << 31))
    return UPR_ERR_UNSUPPORTED;
  const int nv = (int)(n / 4), CV = C / 4;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((nv + 255) / 256), dim3(256), 0, ST(stream), (const half_t*)x16, H * W * C, W * C,
                       C, H, W, CV, Ho, Wo, nv, (float*)y->data, (int)y->sb, (int)y->sh, (int)y->sw, (unsigned*)code,
                       (half_t*)y16);
  };
  if (kind == 1) go(maxpool4_kernel<3, 1, 1, half_t>);
  else go(maxpool4_kernel<2, 2, 0, half_t>);
  LAUNCH_CHECK();
}

int upr_t_maxpool_bwd_code(const unsigned char* code, const UprView* dy, int B, int H, int W, int C, int k, int s,
                           int p, int Ho, int Wo, const UprView* dx, int accumulate, void* stream) {
  if (!code || !dy || !dx || k <= 0 || s <= 0 || k * k > 255) return UPR_ERR_ARG;
  hipStream_t st = ST(stream);
  const long long ni = (long long)B * H * W * C;
  if (ni == 0) return UPR_OK;
  const int kind = pool_fast_kind(k, s, p);
  if (kind && vec4_view_ok(dy, B, Ho, Wo, C) && vec4_view_ok(dx, B, H, W, C) && (uintptr_t)code % 4 == 0 &&
      ni < (1LL << 31)) {
    const int nv = (int)(ni / 4), CV = C / 4;
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((nv + 255) / 256), dim3(256), 0, st, (const unsigned*)code,
                         (const float*)dy->data, (int)dy->sb, (int)dy->sh, (int)dy->sw, H, W, CV, Ho, Wo, nv,
                         (float*)dx->data, (int)dx->sb, (int)dx->sh, (int)dx->sw, accumulate, (const half_t*)nullptr,
                         (half_t*)nullptr);
    };
    if (kind == 1) go(maxpool_gather4_kernel<3, 1, 1>);
    else go(maxpool_gather4_kernel<2, 2, 0>);
    LAUNCH_CHECK();
  }
  if (!accumulate) {
    // the generic gather adds into dx: clear the view first
    hipLaunchKernelGGL(zero_view_kernel, dim3(grid_for(ni)), dim3(256), 0, st, mkv(dx), B, H, W, C);
  }
  hipLaunchKernelGGL(maxpool_bwd_gather_kernel<1>, dim3(grid_for(ni)), dim3(256), 0, st, code, mkv(dy), B, H, W, C,
                     k, s, p, Ho, Wo, mkv(dx));
  LAUNCH_CHECK();
}

int upr_t_maxpool_bwd_code16(const unsigned char* code, const UprView* dy, int B, int H, int W, int C, int k, int s,
                             int p, int Ho, int Wo, const void* y16, void* g16, void* stream) {
  if (!code || !dy || !g16 || k <= 0 || s <= 0 || k * k > 255) return UPR_ERR_ARG;
  const long long ni = (long long)B * H * W * C;
  if (ni == 0) return UPR_OK;
  const int kind = pool_fast_kind(k, s, p);
  if (!kind || !vec4_view_ok(dy, B, Ho, Wo, C) || (uintptr_t)code % 4 || (uintptr_t)g16 % 8 || (uintptr_t)y16 % 8 ||
      ni >= (1LL << 31))
    return UPR_ERR_UNSUPPORTED;
  const int nv = (int)(ni / 4), CV = C / 4;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((nv + 255) / 256), dim3(256), 0, ST(stream), (const unsigned*)code,
                       (const float*)dy->data, (int)dy->sb, (int)dy->sh, (int)dy->sw, H, W, CV, Ho, Wo, nv,
                       (float*)nullptr, 0, 0, 0, 0, (const half_t*)y16, (half_t*)g16);
  };
  if (kind == 1) go(maxpool_gather4_kernel<3, 1, 1, 1>);
  else go(maxpool_gather4_kernel<2, 2, 0, 1>);
  LAUNCH_CHECK();
}

int upr_t_bilinear(const UprView* x, int B, int H, int W, int C, const UprView* y, int Ho, int Wo, int accumulate,
                   void* stream) {
  if (!x || !y || Ho <= 0 || Wo <= 0) return UPR_ERR_ARG;
  const long long n = (long long)B * Ho * Wo * C;
  if (n == 0) return UPR_OK;
  if (vec4_view_ok(x, B, H, W, C) && vec4_view_ok(y, B, Ho, Wo, C)) {
    const int nv = (int)(n / 4);
    hipLaunchKernelGGL(bilinear4_kernel, dim3((nv + 255) / 256), dim3(256), 0, ST(stream), mkv4(x), H, W, C / 4,
                       mkv4(y), Ho, Wo, (float)H / Ho, (float)W / Wo, nv, accumulate, (half_t*)nullptr, 0);
    LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(bilinear_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), mkv(x), B, H, W, C, mkv(y), Ho, Wo,
                     (float)H / Ho, (float)W / Wo, accumulate);
  LAUNCH_CHECK();
}

int upr_t_bilinear_bwd(const UprView* dy, int B, int H, int W, int C, int Ho, int Wo, const UprView* dx,
                       void* stream) {
  if (!dy || !dx) return UPR_ERR_ARG;
  const long long n = (long long)B * Ho * Wo * C;
  if (n > 0 && vec4_view_ok(dy, B, Ho, Wo, C) && vec4_view_ok(dx, B, H, W, C) &&
             (long long)B * Ho * W * C < (1LL << 31)) {
    hipStream_t st = ST(stream);
    const int nr = B * Ho * W * C / 4, ns = B * H * W * C / 4;
    float* row = nullptr;
    row = (float*)scratch(kSlotRows, sizeof(float) * 4 * (size_t)nr, st);
    if (!row) return (int)hipErrorOutOfMemory;
    hipLaunchKernelGGL(bilinear_bwd_rows4_kernel, dim3((nr + 255) / 256), dim3(256), 0, st, mkv4(dy), Ho, Wo, W, C / 4,
                       (float)W / Wo, row, nr);
    hipLaunchKernelGGL(bilinear_bwd_cols4_kernel, dim3((ns + 255) / 256), dim3(256), 0, st, (const float*)row, Ho, H,
                       W, C / 4, (float)H / Ho, mkv4(dx), ns);
    UPR_CHECK_HIP(hipGetLastError());
    return UPR_OK;
  } else {
    const long long ns = (long long)B * H * W * C;
    hipLaunchKernelGGL(bilinear_bwd_gather_kernel, dim3(grid_for(ns)), dim3(256), 0, ST(stream), mkv(dy), B, H, W, C,
                       Ho, Wo, (float)H / Ho, (float)W / Wo, mkv(dx));
  }
  LAUNCH_CHECK();
}

int upr_t_copy16(const UprView* src, const UprView* dst, int B, int H, int W, int C, int accumulate, void* dst16,
                 int dst16_cs, void* stream) {
  if (!src || !dst || !src->data || !dst->data || !dst16 || accumulate < 0 || accumulate > 2) return UPR_ERR_ARG;
  const long long n = (long long)B * H * W * C;
  if (n == 0) return UPR_OK;
  if (!vec4_view_ok(src, B, H, W, C) || !vec4_view_ok(dst, B, H, W, C) || (uintptr_t)dst16 % 8 || dst16_cs % 4 ||
      (long long)B * H * W * dst16_cs >= (1LL << 31))
    return UPR_ERR_UNSUPPORTED;
  const int nv = (int)(n / 4);
  hipLaunchKernelGGL(copy4_kernel, dim3((nv + 255) / 256), dim3(256), 0, ST(stream), mkv4(src), mkv4(dst), H, W, C / 4,
                     nv, accumulate, (half_t*)dst16, dst16_cs);
  LAUNCH_CHECK();
}

int upr_t_bilinear16(const UprView* x, int B, int H, int W, int C, const UprView* y, int Ho, int Wo, int accumulate,
                     void* y16, int y16_cs, void* stream) {
  if (!x || !y || !y16 || Ho <= 0 || Wo <= 0 || accumulate < 0 || accumulate > 2) return UPR_ERR_ARG;
  const long long n = (long long)B * Ho * Wo * C;
  if (n == 0) return UPR_OK;
  if (!vec4_view_ok(x, B, H, W, C) || !vec4_view_ok(y, B, Ho, Wo, C) || (uintptr_t)y16 % 8 || y16_cs % 4 ||
      (long long)B * Ho * Wo * y16_cs >= (1LL << 31))
    return UPR_ERR_UNSUPPORTED;
  const int nv = (int)(n / 4);
  hipLaunchKernelGGL(bilinear4_kernel, dim3((nv + 255) / 256), dim3(256), 0, ST(stream), mkv4(x), H, W, C / 4, mkv4(y),
                     Ho, Wo, (float)H / Ho, (float)W / Wo, nv, accumulate, (half_t*)y16, y16_cs);
  LAUNCH_CHECK();
}

// out = a + b with its fp16 copy (a residual / skip sum feeding an autocast conv)
__global__ __launch_bounds__(256) void add16_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                    float* __restrict__ out, half_t* __restrict__ out16, int n4) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float4 u = ((const float4*)a)[i], v = ((const float4*)b)[i];
  const float4 r = make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w);
  ((float4*)out)[i] = r;
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  ((h4*)out16)[i] = h4{(half_t)r.x, (half_t)r.y, (half_t)r.z, (half_t)r.w};
}

int upr_t_add16(const float* a, const float* b, float* out, size_t n, void* out16, void* stream) {
  if (!a || !b || !out || !out16) return UPR_ERR_ARG;
  if (n % 4 || n / 4 >= (1ULL << 31) || ((uintptr_t)a | (uintptr_t)b | (uintptr_t)out) % 16 || (uintptr_t)out16 % 8)
    return UPR_ERR_UNSUPPORTED;
  if (n == 0) return UPR_OK;
  const int n4 = (int)(n / 4);
  hipLaunchKernelGGL(add16_kernel, dim3((n4 + 255) / 256), dim3(256), 0, ST(stream), a, b, out, (half_t*)out16, n4);
  LAUNCH_CHECK();
}

int upr_t_pixel_sum(const float* x, int B, int HW, int C, int cs, int coff, float scale, float* out, int accumulate,
                    void* stream) {
  if (!x || !out || B <= 0 || HW <= 0) return UPR_ERR_ARG;
  if (C % 4 == 0 && C <= 1024 && cs % 4 == 0 && coff % 4 == 0 && ((uintptr_t)x & 15) == 0) {
    hipStream_t st = ST(stream);
    int chunks = HW / 1024;
    chunks = chunks < 1 ? 1 : (chunks > 256 ? 256 : chunks);
    float* part = (float*)scratch(kSlotPart, sizeof(float) * (size_t)B * chunks * C, st);
    if (!part) return (int)hipErrorOutOfMemory;
    hipLaunchKernelGGL(pixel_sum4_kernel, dim3(chunks, B), dim3(256), 0, st, x, HW, C, cs, coff, part);
    UPR_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(pixel_sum_fin_kernel, dim3((B * C + 255) / 256), dim3(256), 0, st, (const float*)part, chunks,
                       B * C, C, scale, out, accumulate);
    LAUNCH_CHECK();
  }
  if (!accumulate) UPR_CHECK_HIP(hipMemsetAsync(out, 0, sizeof(float) * B * C, ST(stream)));
  int chunks = HW / 2048;
  chunks = chunks < 1 ? 1 : (chunks > 256 ? 256 : chunks);
  hipLaunchKernelGGL(pixel_sum_kernel, dim3(chunks, B), dim3(256), 0, ST(stream), x, HW, C, cs, coff, scale, out);
  LAUNCH_CHECK();
}

int upr_t_broadcast(const float* v, int B, int HW, int C, float scale, float* y, int y_cs, int y_coff, int accumulate,
                    void* stream) {
  if (!v || !y) return UPR_ERR_ARG;
  const long long n = (long long)B * HW * C;
  hipLaunchKernelGGL(broadcast_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), v, B, HW, C, scale, y, y_cs,
                     y_coff, accumulate);
  LAUNCH_CHECK();
}

int upr_t_broadcast16(const float* v, int B, int HW, int C, float scale, void* y16, int y_cs, int y_coff,
                      void* stream) {
  if (!v || !y16 || B <= 0 || HW <= 0 || C <= 0 || y_cs < y_coff + C) return UPR_ERR_ARG;
  if (C % 4 || y_cs % 4 || y_coff % 4 || (uintptr_t)y16 % 8) return UPR_ERR_UNSUPPORTED;
  const long long n = (long long)B * HW * (C / 4);
  hipLaunchKernelGGL(broadcast16_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), v, B, HW, C, scale,
                     (half_t*)y16, y_cs, y_coff);
  LAUNCH_CHECK();
}

int upr_t_fam_ca_apply(const float* o, const float* ca, int B, int HW, int C, float* o2, float* m, void* stream) {
  if (!o || !ca || !o2 || !m) return UPR_ERR_ARG;
  if (C == 32 && al16(o) && al16(ca) && al16(o2)) {
    hipLaunchKernelGGL(fam_ca_apply32_kernel, dim3(grid_for((long long)B * HW * 8)), dim3(256), 0, ST(stream), o, ca,
                       B, HW, o2, m);
    LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(fam_ca_apply_kernel, dim3(grid_for((long long)B * HW)), dim3(256), 0, ST(stream), o, ca, B, HW,
                     C, o2, m);
  LAUNCH_CHECK();
}

int upr_t_fam_sa_apply(const float* o2, const float* s_pre, int B, int HW, int C, float* sa, float* out,
                       void* stream) {
  if (!o2 || !s_pre || !sa || !out) return UPR_ERR_ARG;
  if (C == 32 && al16(o2) && al16(out)) {
    hipLaunchKernelGGL(fam_sa_apply32_kernel, dim3(grid_for((long long)B * HW * 8)), dim3(256), 0, ST(stream), o2,
                       s_pre, B, HW, sa, out);
    LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(fam_sa_apply_kernel, dim3(grid_for((long long)B * HW)), dim3(256), 0, ST(stream), o2, s_pre, B,
                     HW, C, sa, out);
  LAUNCH_CHECK();
}

int upr_t_fam_sa_bwd_cs(const float* g, int g_cs, const float* o2, const float* sa, int B, int HW, int C,
                        float* g_o2, float* g_spre, void* stream) {
  if (!g || !o2 || !sa || !g_o2 || !g_spre || g_cs < C) return UPR_ERR_ARG;
  if (C == 32 && g_cs % 4 == 0 && al16(g) && al16(o2) && al16(g_o2)) {
    hipLaunchKernelGGL(fam_sa_bwd32_kernel, dim3(grid_for((long long)B * HW * 8)), dim3(256), 0, ST(stream), g, g_cs,
                       o2, sa, B, HW, g_o2, g_spre);
    LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(fam_sa_bwd_kernel, dim3(grid_for((long long)B * HW)), dim3(256), 0, ST(stream), g, g_cs, o2, sa,
                     B, HW, C, g_o2, g_spre);
  LAUNCH_CHECK();
}

int upr_t_fam_sa_bwd(const float* g, const float* o2, const float* sa, int B, int HW, int C, float* g_o2,
                     float* g_spre, void* stream) {
  return upr_t_fam_sa_bwd_cs(g, C, o2, sa, B, HW, C, g_o2, g_spre, stream);
}

int upr_t_fam_ca_bwd(const float* g_o2, const float* g_m, const float* o, const float* o2, const float* ca, int B,
                     int HW, int C, float* g_o, float* g_ca, void* stream) {
  if (!g_o2 || !g_m || !o || !o2 || !ca || !g_o || !g_ca || C > 32) return UPR_ERR_ARG;
  if (C == 32 && al16(g_o2) && al16(o) && al16(o2) && al16(ca) && al16(g_o) && B > 0 && HW > 0) {
    hipStream_t st = ST(stream);
    int chunks = HW / 1024;
    chunks = chunks < 1 ? 1 : (chunks > 256 ? 256 : chunks);
    float* part = nullptr;
    part = (float*)scratch(kSlotPart, sizeof(float) * 32 * B * chunks, st);
    if (!part) return (int)hipErrorOutOfMemory;
    hipLaunchKernelGGL(fam_ca_bwd32_kernel, dim3(chunks, B), dim3(256), 0, st, g_o2, g_m, o, o2, ca, HW, g_o, part);
    hipLaunchKernelGGL(fam_ca_fin_kernel, dim3(B * 32), dim3(256), 0, st, (const float*)part, chunks, B * 32, g_ca);
    UPR_CHECK_HIP(hipGetLastError());
    return UPR_OK;
  }
  UPR_CHECK_HIP(hipMemsetAsync(g_ca, 0, sizeof(float) * B * C, ST(stream)));
  int chunks = HW / 4096;
  chunks = chunks < 1 ? 1 : (chunks > 256 ? 256 : chunks);
  hipLaunchKernelGGL(fam_ca_bwd_kernel, dim3(chunks, B), dim3(256), 0, ST(stream), g_o2, g_m, o, o2, ca, HW, C, g_o,
                     g_ca);
  LAUNCH_CHECK();
}

int upr_t_fam_pool_bwd16(float* g_o, const float* g_pool, const float* o, int B, int HW, int C, void* g16,
                         void* stream) {
  if (!g_o || !g_pool || !o || B <= 0 || HW <= 0 || C <= 0) return UPR_ERR_ARG;
  const long long n = (long long)B * HW * C;
  if (C % 4 == 0 && 256 % (C / 4) == 0 && n < (1LL << 31) && al16(g_o) && al16(g_pool) && al16(o) &&
      (uintptr_t)g16 % 8 == 0) {
    const long long M = (long long)B * HW;
    hipLaunchKernelGGL(fam_pool_bwd4_kernel, dim3(grid_for(M * (C / 4))), dim3(256), 0, ST(stream), g_o, g_pool, o,
                       (int)M, HW, C, (half_t*)g16);
    LAUNCH_CHECK();
  }
  if (g16) return UPR_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(fam_pool_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, ST(stream), g_o, g_pool, o, B, HW, C);
  LAUNCH_CHECK();
}

int upr_t_fam_pool_bwd(float* g_o, const float* g_pool, const float* o, int B, int HW, int C, void* stream) {
  return upr_t_fam_pool_bwd16(g_o, g_pool, o, B, HW, C, nullptr, stream);
}

int upr_t_head_fwd(const float* x, const float* r, float* illu, int B, int H, int W, void* stream) {
  if (!x || !r || !illu) return UPR_ERR_ARG;
  hipLaunchKernelGGL(head_fwd_kernel, dim3(grid_for((long long)B * H * W)), dim3(256), 0, ST(stream), x, r, illu, B,
                     H * W);
  LAUNCH_CHECK();
}

int upr_t_retinex_fwd(const float* x, const float* illu, const float* o, float* e, float* refl, float* enh, int B,
                      int H, int W, void* stream) {
  if (!x || !illu || !o || !e || !refl || !enh) return UPR_ERR_ARG;
  hipLaunchKernelGGL(retinex_fwd_kernel, dim3(grid_for((long long)B * H * W)), dim3(256), 0, ST(stream), x, illu, o,
                     e, refl, enh, B, H * W);
  LAUNCH_CHECK();
}

int upr_t_retinex_bwd(const float* x, const float* illu, const float* e, const float* refl, const float* g_enh,
                      const float* g_refl, const float* g_illu, float* g_o, float* g_r, int B, int H, int W,
                      void* stream) {
  if (!x || !illu || !e || !refl || !g_enh || !g_o || !g_r) return UPR_ERR_ARG;
  hipLaunchKernelGGL(retinex_bwd_kernel, dim3(grid_for((long long)B * H * W)), dim3(256), 0, ST(stream), x, illu, e,
                     refl, g_enh, g_refl, g_illu, g_o, g_r, B, H * W);
  LAUNCH_CHECK();
}

int upr_t_enhance_fwd(const float* refl, const float* o, float* e, float* enh, int B, int H, int W, void* stream) {
  if (!refl || !o || !e || !enh) return UPR_ERR_ARG;
  hipLaunchKernelGGL(enhance_fwd_kernel, dim3(grid_for((long long)B * H * W)), dim3(256), 0, ST(stream), refl, o, e,
                     enh, B, H * W);
  LAUNCH_CHECK();
}

int upr_t_enhance_bwd(const float* e, const float* refl, const float* g_enh, float* g_o, float* g_refl, int B, int H,
                      int W, void* stream) {
  if (!e || !refl || !g_enh || !g_o) return UPR_ERR_ARG;
  hipLaunchKernelGGL(enhance_bwd_kernel, dim3(grid_for((long long)B * H * W)), dim3(256), 0, ST(stream), e, refl,
                     g_enh, g_o, g_refl, B, H * W);
  LAUNCH_CHECK();
}

static const UprLossParams kLossDefaults = {16, 0.6f, 10.f, 1.f, 0.1f, 1.f, 0.5f, 1, 1};

size_t upr_t_loss_workspace(int B, int H, int W) { return upr_t_loss_workspace_p(B, H, W, 16); }

size_t upr_t_loss_workspace_p(int B, int H, int W, int patch) {
  if (B <= 0 || patch <= 0 || H < patch || W < patch || H < 2 || W < 2) return 0;
  return loss_ws_bytes(B, H, W, patch);
}

int upr_t_loss_pixel(const float* low, const float* enh, const float* illu, const float* refl, int B, int H, int W,
                     void* ws, float* terms, float* g_enh, float* g_illu, float* g_refl, int grads, float w_exp,
                     float w_col, float w_spa, float w_dec, float w_smooth, int texture, void* stream) {
  if (H % 16 || W % 16) return UPR_ERR_SHAPE;
  return upr_t_loss_pixel_p(low, enh, illu, refl, B, H, W, ws, terms, g_enh, g_illu, g_refl, grads, w_exp, w_col,
                            w_spa, w_dec, w_smooth, texture, &kLossDefaults, stream);
}

int upr_t_loss_pixel_p(const float* low, const float* enh, const float* illu, const float* refl, int B, int H, int W,
                       void* ws, float* terms, float* g_enh, float* g_illu, float* g_refl, int grads, float w_exp,
                       float w_col, float w_spa, float w_dec, float w_smooth, int texture,
                       const UprLossParams* prm, void* stream) {
  if (!low || !enh || !illu || !refl || !ws || !terms || !prm || B <= 0) return UPR_ERR_ARG;
  if (texture != 0 && texture != 1) return UPR_ERR_ARG;
  if (prm->patch <= 0 || H < prm->patch || W < prm->patch || H < 2 || W < 2) return UPR_ERR_SHAPE;
  if (grads && (!g_enh || !g_illu || !g_refl)) return UPR_ERR_ARG;
  const int CI = prm->illu_channels == 0 ? 1 : prm->illu_channels;
  if (CI != 1 && CI != 3) return UPR_ERR_UNSUPPORTED;
  hipStream_t st = ST(stream);
  const size_t zero_bytes = loss_ws_bytes(B, H, W, prm->patch) - loss_scal_bytes(B);
  UPR_CHECK_HIP(hipMemsetAsync(ws, 0, zero_bytes, st));
  LossWS l = loss_ws(ws, B, H, W, prm->patch);
  l.ps = prm->patch;
  l.base_exp = prm->base_exposure;
  l.lam_s = prm->smooth_lambda;
  l.alpha = prm->smooth_alpha;
  l.lam_d = prm->decouple_lambda;
  l.dynamic = prm->dynamic_smooth ? 1 : 0;
  int chunks = (H * W) / 4096;
  chunks = chunks < 1 ? 1 : (chunks > 128 ? 128 : chunks);
  const int ps = l.ps;
  const bool banded = ps <= 64 && (ps & (ps - 1)) == 0 && H % ps == 0 && W % ps == 0;
  const dim3 bgrid((W + 255) / 256, H / ps, B);
  if (CI == 1) {
    if (banded) hipLaunchKernelGGL(loss_pass1_band_kernel<1>, bgrid, dim3(256), 0, st, low, enh, illu, refl, H, W, l);
    else hipLaunchKernelGGL(loss_pass1_kernel<1>, dim3(chunks, B), dim3(256), 0, st, low, enh, illu, refl, H, W, l);
    UPR_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(loss_pass2_kernel<1>, dim3(chunks, B), dim3(256), 0, st, low, illu, H, W, l);
  } else {
    if (banded) hipLaunchKernelGGL(loss_pass1_band_kernel<3>, bgrid, dim3(256), 0, st, low, enh, illu, refl, H, W, l);
    else hipLaunchKernelGGL(loss_pass1_kernel<3>, dim3(chunks, B), dim3(256), 0, st, low, enh, illu, refl, H, W, l);
    UPR_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(loss_pass2_kernel<3>, dim3(chunks, B), dim3(256), 0, st, low, illu, H, W, l);
  }
  UPR_CHECK_HIP(hipGetLastError());
  if (texture == 1 && l.dynamic) {
    for (int mode = 0; mode < 2; ++mode) {
      hipLaunchKernelGGL(edge_density_kernel, dim3(chunks, B), dim3(256), 0, st, low, H, W, l, mode);
      UPR_CHECK_HIP(hipGetLastError());
    }
  }
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, st, B, H, W, l, terms, texture, w_smooth, CI);
  UPR_CHECK_HIP(hipGetLastError());
  if (grads) {
    if (CI == 1)
      hipLaunchKernelGGL(loss_grad_kernel<1>, dim3(grid_for((long long)B * H * W)), dim3(256), 0, st, low, enh, illu,
                         refl, B, H, W, l, g_enh, g_illu, g_refl, w_exp, w_col, w_spa, w_dec);
    else
      hipLaunchKernelGGL(loss_grad_kernel<3>, dim3(grid_for((long long)B * H * W)), dim3(256), 0, st, low, enh, illu,
                         refl, B, H, W, l, g_enh, g_illu, g_refl, w_exp, w_col, w_spa, w_dec);
  }
  LAUNCH_CHECK();
}

int upr_t_texture_complexity(const float* img, int B, int C, int H, int W, int method, double* acc, float* out,
                             void* stream) {
  if (!img || !acc || !out || B <= 0 || C <= 0 || (method != 0 && method != 1)) return UPR_ERR_ARG;
  if (H < 2 || W < 2) return UPR_ERR_SHAPE;  // a finite difference / a reflect pad needs two samples per axis
  hipStream_t st = ST(stream);
  UPR_CHECK_HIP(hipMemsetAsync(acc, 0, sizeof(double) * 2 * B, st));
  int chunks = (H * W) / 4096;
  chunks = chunks < 1 ? 1 : (chunks > 128 ? 128 : chunks);
  for (int mode = 0; mode < (method == 1 ? 2 : 1); ++mode) {
    hipLaunchKernelGGL(texture_kernel, dim3(chunks, B), dim3(256), 0, st, img, C, H, W, method, mode, acc);
    UPR_CHECK_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(texture_final_kernel, dim3((B + 63) / 64), dim3(64), 0, st, acc, B, C, H, W, method, out);
  LAUNCH_CHECK();
}

int upr_t_loss_total(float* terms, float w_exp, float w_col, float w_spa, float w_dec, float w_per, float w_freq,
                     void* stream) {
  if (!terms) return UPR_ERR_ARG;
  hipLaunchKernelGGL(loss_total_kernel, dim3(1), dim3(64), 0, ST(stream), terms, w_exp, w_col, w_spa, w_dec, w_per,
                     w_freq);
  LAUNCH_CHECK();
}

// the same over two fp16 tensors (the frozen VGG's features under autocast,
// which exist in fp16 only: the reference's mse_loss promotes them to fp32),
// 4 elements per thread
__global__ __launch_bounds__(256) void mse16_kernel(const half_t* __restrict__ a, const half_t* __restrict__ b,
                                                    long long n4, long long n, double* acc, float* g, float scale) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  double v[1] = {0.0};
  GSTRIDE(i, n4) {
    const h4 x = *(const h4*)(a + 4 * i), y = *(const h4*)(b + 4 * i);
    float d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      d[k] = (float)x[k] - (float)y[k];
      v[0] += (double)d[k] * d[k];
    }
    if (g) *(float4*)(g + 4 * i) = make_float4(scale * 2.f * d[0], scale * 2.f * d[1], scale * 2.f * d[2], scale * 2.f * d[3]);
  }
  v[0] /= (double)n;
  double* dst[1] = {acc};
  block_sum_atomic<1>(v, dst);
}

int upr_t_mse16(const void* a16, const void* b16, size_t n, double* acc, float* g, float scale, void* stream) {
  if (!a16 || !b16 || !acc) return UPR_ERR_ARG;
  if (n % 4 || ((uintptr_t)a16 | (uintptr_t)b16) % 8 || (uintptr_t)g % 16) return UPR_ERR_UNSUPPORTED;
  if (n == 0) return UPR_OK;
  const long long n4 = (long long)(n / 4);
  hipLaunchKernelGGL(mse16_kernel, dim3(grid_for(n4, 256, 4096)), dim3(256), 0, ST(stream), (const half_t*)a16,
                     (const half_t*)b16, n4, (long long)n, acc, g, scale);
  LAUNCH_CHECK();
}

int upr_t_mse(const float* a, const float* b, size_t n, double* acc, float* g, float scale, void* stream) {
  if (!a || !b || !acc) return UPR_ERR_ARG;
  hipLaunchKernelGGL(mse_kernel, dim3(grid_for((long long)n, 256, 4096)), dim3(256), 0, ST(stream), a, b,
                     (long long)n, acc, g, scale);
  LAUNCH_CHECK();
}

int upr_t_vgg_norm(const float* x, float* y, int B, int H, int W, void* stream) {
  if (!x || !y) return UPR_ERR_ARG;
  hipLaunchKernelGGL(vgg_norm_kernel, dim3(grid_for((long long)B * H * W)), dim3(256), 0, ST(stream), x, y, B, H * W);
  LAUNCH_CHECK();
}

int upr_t_vgg_norm_bwd(const float* g_y, float* g_x, int B, int H, int W, void* stream) {
  if (!g_y || !g_x) return UPR_ERR_ARG;
  hipLaunchKernelGGL(vgg_norm_bwd_kernel, dim3(grid_for((long long)B * H * W)), dim3(256), 0, ST(stream), g_y, g_x, B,
                     H * W);
  LAUNCH_CHECK();
}

int upr_t_freq(const float* Ze, const float* Zl, int BC, int H, int W, double* acc, float* G, float scale,
               void* stream) {
  return upr_t_freq_p(Ze, Zl, BC, H, W, acc, G, scale, 1.f, 0.5f, stream);
}

int upr_t_freq_p(const float* Ze, const float* Zl, int BC, int H, int W, double* acc, float* G, float scale,
                 float w_high, float w_low, void* stream) {
  if (!Ze || !Zl || !acc) return UPR_ERR_ARG;
  hipLaunchKernelGGL(freq_kernel, dim3(grid_for((long long)BC * H * W, 256, 4096)), dim3(256), 0, ST(stream),
                     (const float2*)Ze, (const float2*)Zl, BC, H, W, acc, (float2*)G, scale, w_high, w_low);
  LAUNCH_CHECK();
}

int upr_t_add_real(const float* z, float* g, size_t n, float scale, void* stream) {
  if (!z || !g) return UPR_ERR_ARG;
  hipLaunchKernelGGL(add_real_kernel, dim3(grid_for((long long)n)), dim3(256), 0, ST(stream), (const float2*)z, g,
                     (long long)n, scale);
  LAUNCH_CHECK();
}

int upr_t_scale_acc(const double* acc, int n, float scale, float* out, void* stream) {
  if (!acc || !out || n <= 0 || n > 256) return UPR_ERR_ARG;
  hipLaunchKernelGGL(scale_acc_kernel, dim3(1), dim3(256), 0, ST(stream), acc, n, scale, out);
  LAUNCH_CHECK();
}

int upr_t_sqsum(const float* g, size_t n, double* acc, void* stream) {
  if (!g || !acc) return UPR_ERR_ARG;
  hipLaunchKernelGGL(sqsum_kernel, dim3(grid_for((long long)n, 256, 2048)), dim3(256), 0, ST(stream), g,
                     (long long)n, acc);
  LAUNCH_CHECK();
}

int upr_t_unscale(float* g, size_t n, const float* scale, float* found_inf, void* stream) {
  if (!g || !scale || !found_inf) return UPR_ERR_ARG;
  hipLaunchKernelGGL(unscale_kernel, dim3(grid_for((long long)n, 256, 2048)), dim3(256), 0, ST(stream), g,
                     (long long)n, scale, found_inf);
  LAUNCH_CHECK();
}

int upr_t_adam(float* p, const float* g, float* m, float* v, size_t n, const double* sqsum, float max_norm, float lr,
               float beta1, float beta2, float eps, float weight_decay, int step, float* norm_out, void* stream) {
  if (!p || !g || !m || !v || !sqsum || step <= 0) return UPR_ERR_ARG;
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2s = sqrtf(1.f - powf(beta2, (float)step));
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for((long long)n)), dim3(256), 0, ST(stream), p, g, m, v, (long long)n,
                     sqsum, max_norm, lr, beta1, beta2, eps, weight_decay, bc1, bc2s, norm_out);
  LAUNCH_CHECK();
}

}  // extern "C"
