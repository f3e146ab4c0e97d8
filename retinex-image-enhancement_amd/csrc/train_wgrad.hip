// Weight gradient of the MFMA-path convs of the training step as a split-K
// GEMM over pixels (replaces round 1's per-tap 32x32 kernel with fp32
// atomics, 17 % of the bs-8 512^2 step at 0.27 of the fp32 MFMA peak):
//
//   dW[co][k] = sum_p dy[p][co] * im2col(x)[p][k],   k = (ky, kx, ci)
//
// * M = Cout, N = kh*kw*Cin, K = the B*Ho*Wo output pixels, split into
//   `splits` contiguous pixel ranges.  Block tile BM x BN (4 waves, each a
//   32 x 64 block of v_mfma_f32_32x32x2_f32 accumulators), K step = 32
//   pixels.
// * Both operands global -> LDS by LDS-DMA into two stages (one barrier per
//   step): A = the dy rows of the step's pixels (BM channels each), B = their
//   im2col rows (BN/32 runs of 32 channels, each at its tap's shifted pixel;
//   padded taps / pixels past the range read a zero line).  The MFMA
//   fragments are single floats: lane l takes row (pixel) 2s + l/32, column
//   l%32 -- ds_read_b32 over consecutive addresses, conflict free.
// * Each block writes its partial tile to its split's slab (plain stores);
//   a second kernel sums the slabs in split order and adds them to dwp:
//   deterministic (no float atomics), one pass over the slabs.
// * The slabs live in the caller stream's scratch slot (upr_common.h
//   scratch()), so concurrent streams never share them.
#include <cstdlib>
#include <cstring>

#include "upr_common.h"
#include "../../include/upr_train.h"

namespace upr {

typedef float f32x4_w2 __attribute__((ext_vector_type(4)));
typedef float f32x16_w2 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* lds_void_ptr_w2;

__device__ __attribute__((aligned(128))) uint4 g_wg_zero[8];

constexpr int WG_KP = 32;  // pixels per K step

struct WgArgs {
  const float* x;
  int B, H, W, Cin, x_cs, x_coff;
  const float* dy;
  int Ho, Wo, Cout, dy_cs, dy_coff;
  int kh, kw, s, p, d;
  int KT;       // kh*kw*Cin
  int P;        // B*Ho*Wo
  int splits, pix_per_split, mtiles, ntiles, ldn;  // ldn: slab row length (ntiles*BN)
  float* slab;  // [splits][Cout][ldn]
};

__device__ __forceinline__ void wg_glds16(const void* g, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_void_ptr_w2)lds, 16, 0, 0);
}

template <int BM, int BN>
__global__ __launch_bounds__(256) void wgrad_gemm_kernel(WgArgs a) {
  constexpr int WAVES_N = BN / 64;
  constexpr int WAVES_M = 4 / WAVES_N;
  static_assert(WAVES_M * 32 == BM, "tile");
  constexpr int A_BYTES = WG_KP * BM * 4, B_BYTES = WG_KP * BN * 4, STAGE = A_BYTES + B_BYTES;
  constexpr int AI = WG_KP * BM / 4 / 256;  // A DMA instructions per wave per step (64 lanes x 16 B each)
  constexpr int BI = WG_KP * BN / 4 / 256;
  extern __shared__ __attribute__((aligned(16))) unsigned char wsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  int bid = blockIdx.x;
  const int nt = bid % a.ntiles; bid /= a.ntiles;
  const int mt = bid % a.mtiles;
  const int split = bid / a.mtiles;
  const int co0 = mt * BM, k0 = nt * BN;
  const int pb = split * a.pix_per_split;
  const int pe = min(a.P, pb + a.pix_per_split);
  const int steps = (pe - pb + WG_KP - 1) / WG_KP;
  const float* zero = (const float*)g_wg_zero;
  const int HWo = a.Ho * a.Wo;
  const int cinq = a.Cin / 32;

  auto issue = [&](int step, int stage) {
    unsigned char* As = wsm + stage * STAGE;
    unsigned char* Bs = As + A_BYTES;
    const int ps = pb + step * WG_KP;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int c = (wave * AI + i) * 64 + lane;  // 16-byte chunk of the A tile
      const int pr = c / (BM / 4), q = c % (BM / 4);
      const int pix = ps + pr;
      const float* src = pix < pe ? a.dy + (size_t)pix * a.dy_cs + a.dy_coff + co0 + q * 4 : zero;
      wg_glds16(src, As + (wave * AI + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int c = (wave * BI + i) * 64 + lane;
      const int pr = c / (BN / 4), q = c % (BN / 4);
      const int pix = ps + pr;
      const int k = k0 + q * 4;
      const float* src = zero;
      if (pix < pe && k < a.KT) {
        const int kq = k >> 5;  // 32-channel run: (tap, ci chunk)
        const int tap = kq / cinq, ci = (kq - tap * cinq) * 32 + (k & 31);
        const int ky = tap / a.kw, kx = tap - ky * a.kw;
        const int b = pix / HWo, r = pix - b * HWo;
        const int oy = r / a.Wo, ox = r - oy * a.Wo;
        const int iy = oy * a.s - a.p + ky * a.d, ix = ox * a.s - a.p + kx * a.d;
        if ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
          src = a.x + (size_t)((b * a.H + iy) * a.W + ix) * a.x_cs + a.x_coff + ci;
      }
      wg_glds16(src, Bs + (wave * BI + i) * 1024);
    }
  };

  f32x16_w2 acc0, acc1;
#pragma unroll
  for (int e = 0; e < 16; ++e) { acc0[e] = 0.f; acc1[e] = 0.f; }
  const int half = lane >> 5, col = lane & 31;

  if (steps > 0) issue(0, 0);
  for (int step = 0; step < steps; ++step) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (step + 1 < steps) issue(step + 1, (step + 1) & 1);
    const float* As = (const float*)(wsm + (step & 1) * STAGE);
    const float* Bs = As + A_BYTES / 4;
#pragma unroll
    for (int s = 0; s < WG_KP / 2; ++s) {
      const int row = 2 * s + half;
      const float av = As[row * BM + wm * 32 + col];
      const float b0 = Bs[row * BN + wn * 64 + col];
      const float b1 = Bs[row * BN + wn * 64 + 32 + col];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b1, acc1, 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // partial tile -> this split's slab; D row = (e&3) + 8*(e>>2) + 4*half, column = lane & 31
  float* sl = a.slab + ((size_t)split * a.Cout + co0 + wm * 32) * a.ldn + k0 + wn * 64 + col;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int row = (e & 3) + 8 * (e >> 2) + 4 * half;
    sl[(size_t)row * a.ldn] = acc0[e];
    sl[(size_t)row * a.ldn + 32] = acc1[e];
  }
}

// dwp (+)= sum of all split slabs in ONE launch (replaces the group + reduce
// pair): a block owns 16 quads of outputs, its 16 thread rows add slabs
// j, j + 16, ... (4 independent sums, loads in flight), then the 16 row sums
// are added in row order -- a fixed order, deterministic run to run.  Output
// layouts: dwp[co][k] packed, or (torch_ci > 0) PyTorch's [Co][Ci][kh][kw] directly
// (k = tap * Ci + ci; the 4 k of a quad share the tap; no unpack pass).
__global__ __launch_bounds__(256) void wgrad_slab_reduce_kernel(const float* __restrict__ slab, int splits, int Cout,
                                                                int KT, int ldn, float* __restrict__ dwp,
                                                                int torch_ci) {
  __shared__ f32x4_w2 red[16][16];
  const int q = threadIdx.x & 15, j = threadIdx.x >> 4;
  const int n4 = Cout * KT / 4;
  const int i = blockIdx.x * 16 + q;
  const int e = i * 4;
  const int co = e / KT, k = e - co * KT;
  f32x4_w2 s[4] = {};
  if (i < n4) {
    const float* p = slab + (size_t)co * ldn + k;
    const size_t step = (size_t)Cout * ldn;
    int sp = j;
    for (; sp + 48 < splits; sp += 64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] += *(const f32x4_w2*)(p + (size_t)(sp + 16 * u) * step);
    }
    for (int u = 0; sp < splits; sp += 16, ++u) s[u & 3] += *(const f32x4_w2*)(p + (size_t)sp * step);
  }
  red[j][q] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  if (j != 0 || i >= n4) return;
  f32x4_w2 acc = red[0][q];
#pragma unroll
  for (int r = 1; r < 16; ++r) acc += red[r][q];
  if (torch_ci) {
    const int taps = KT / torch_ci, tap = k / torch_ci, ci = k - tap * torch_ci;
    float* o = dwp + ((size_t)co * torch_ci + ci) * taps + tap;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) o[(size_t)jj * taps] += acc[jj];
  } else {
    f32x4_w2* o = (f32x4_w2*)(dwp + e);
    *o = *o + acc;
  }
}

static int reduce_slabs(const float* slab, int splits, int Cout, int KT, int ldn, float* dwp, int torch_ci,
                        hipStream_t st) {
  const int n4 = Cout * KT / 4;
  hipLaunchKernelGGL(wgrad_slab_reduce_kernel, dim3((n4 + 15) / 16), dim3(256), 0, st, slab, splits, Cout, KT, ldn,
                     dwp, torch_ci);
  return (int)hipGetLastError();
}

template <int BM, int BN>
static int launch_wgrad_gemm(WgArgs a, float* dwp, hipStream_t st, int torch_ci) {
  constexpr int LDS = 2 * WG_KP * (BM + BN) * 4;
  static bool attr = false;
  if (!attr) {
    const hipError_t e =
        hipFuncSetAttribute((const void*)wgrad_gemm_kernel<BM, BN>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  a.mtiles = a.Cout / BM;
  a.ntiles = (a.KT + BN - 1) / BN;
  a.ldn = a.ntiles * BN;
  const int tiles = a.mtiles * a.ntiles;
  // ~1024 blocks (4 per CU), >= 4 K steps each
  int splits = (1024 + tiles - 1) / tiles;
  const int max_splits = (a.P + 4 * WG_KP - 1) / (4 * WG_KP);
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int pps = (a.P + splits - 1) / splits;
  pps = (pps + WG_KP - 1) / WG_KP * WG_KP;
  splits = (a.P + pps - 1) / pps;
  a.splits = splits;
  a.pix_per_split = pps;
  const size_t slab_elems = (size_t)a.Cout * a.ldn;
  void* buf = scratch(kSlotSlab, (size_t)splits * slab_elems * sizeof(float), st);
  if (!buf) return (int)hipErrorOutOfMemory;
  a.slab = (float*)buf;
  hipLaunchKernelGGL((wgrad_gemm_kernel<BM, BN>), dim3(tiles * splits), dim3(256), LDS, st, a);
  return reduce_slabs(a.slab, splits, a.Cout, a.KT, a.ldn, dwp, torch_ci, st);
}

// ---------------------------------------------------------------------------
// AMP weight gradient (trainers/train.py:72 runs the convs under autocast:
// their weight gradients are products of the fp16 input and the fp16 output
// gradient): v_mfma_f32_16x16x32_f16, fp32 accumulation, fp32 result.
//
// * K (the reduction) = output pixels in steps of 64 consecutive pixels of one
//   output row (Wo % 64 == 0); split-K over those row segments into slabs,
//   reduced in a fixed order by wgrad_slab_reduce (deterministic).
// * B = im2col(x16): x16 is the fp16 NHWC copy of the conv input the AMP
//   forward already made (compact, Cin channels); per step, NR 32-channel runs
//   (tap, ci32) of the 64 pixels go global -> LDS by LDS-DMA ([run][pixel][32]
//   fp16, 64-byte rows, the two 32-byte halves swapped on rows with bit 3 set).
// * A = dy (fp32 NHWC) through registers: loaded one step ahead, rounded to
//   fp16 and written [pixel][BM] into LDS (8-byte quads XOR-swizzled per row).
// * Both operands are pixel-major in LDS and the MFMA wants them pixel-
//   contiguous per lane: ds_read_b64_tr_b16 (16 lanes read a 4 x 16 block,
//   lane i gets column i) -- two per fragment.  The per-row swizzles make all
//   of these reads conflict-free (exhaustive check over the 32-lane halves).
// * 4 waves; every wave covers all BM/16 output-channel tiles and the runs
//   w, w+4, w+8 (2 k-tiles each).
// ---------------------------------------------------------------------------
typedef _Float16 f16x8_w2 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4_w2 __attribute__((ext_vector_type(4)));
typedef short s16x4_w2 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_w2* lds_s4_ptr;

constexpr int W16_KP = 64;  // pixels per step

struct Wg16Args {
  const half_t* x16;   // [B][H][W][Cin] fp16
  int B, H, W, Cin;
  const float* dy;
  const half_t* dy16;  // nullable: dy's fp16 copy in dy's layout (dy_cs, dy_coff; its producer's), read instead of dy
  int Ho, Wo, Cout, dy_cs, dy_coff;
  int kh, kw, s, p, d;
  int KT, nruns;       // kh*kw*Cin, KT / 32
  int units;           // B * Ho * (Wo / 64)
  int splits, units_per_split, mtiles, ntiles, ldn;
  float* slab;
};

// 8-byte quad swizzle of an LDS row of NQ quads (NQ = 8: 64-byte rows)
template <int NQ>
__device__ __forceinline__ int w16_swz(int r) {
  return (((r >> 3) & 1) << 2) ^ ((r & 3) * (NQ >= 32 ? 8 : NQ >= 16 ? 4 : 0));
}

__device__ __forceinline__ f16x4_w2 w16_tr(const unsigned char* p) {
  return __builtin_bit_cast(f16x4_w2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)p));
}

template <int BM, int NR>
__global__ __launch_bounds__(256) void wgrad16_kernel(Wg16Args a) {
  constexpr int NQA = BM / 4;                  // quads per A row
  constexpr int A_BYTES = W16_KP * BM * 2;
  constexpr int RUN_BYTES = W16_KP * 64;       // one 32-channel run of 64 pixels
  constexpr int B_BYTES = NR * RUN_BYTES;
  constexpr int MT = BM / 16;
  constexpr int RPW = (NR + 3) / 4;            // runs per wave (max)
  constexpr int AC = BM / 16;                  // A chunks (16 B fp32) per thread per step
  constexpr int BDMA = NR * W16_KP * 4 / 256;  // B DMA pieces (16 B) per thread per step
  static_assert((NR * W16_KP * 4) % 256 == 0, "B pieces");
  extern __shared__ __attribute__((aligned(16))) unsigned char wsm[];
  unsigned char* As = wsm;
  unsigned char* Bs0 = wsm + A_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int bid = blockIdx.x;
  const int nt = bid % a.ntiles; bid /= a.ntiles;
  const int mt = bid % a.mtiles;
  const int split = bid / a.mtiles;
  const int co0 = mt * BM, run0 = nt * NR;
  const int u0 = split * a.units_per_split;
  const int u1 = min(a.units, u0 + a.units_per_split);
  const int segs = a.Wo / W16_KP;
  const half_t* zero16 = (const half_t*)g_wg_zero;

  // A staging: chunk i of this thread = pixel tid / NQA + i * (256 / NQA), quad tid % NQA
  const int qa = tid % NQA;
  f32x4_w2 areg[AC];
  f16x4_w2 hreg[AC];
  const bool a16 = a.dy16 != nullptr;  // uniform
  auto load_a = [&](int u) {
    const int b = u / (a.Ho * segs), r = u - b * a.Ho * segs;
    const int oy = r / segs, ox0 = (r - oy * segs) * W16_KP;
    const size_t pix0 = (size_t)(b * a.Ho + oy) * a.Wo + ox0;
    if (a16) {  // the fp16 copy: half the bytes, the same RNE-rounded values
      const half_t* base = a.dy16 + pix0 * a.dy_cs + a.dy_coff + co0 + qa * 4;
#pragma unroll
      for (int i = 0; i < AC; ++i) {
        const int pr = tid / NQA + i * (256 / NQA);
        hreg[i] = *(const f16x4_w2*)(base + (size_t)pr * a.dy_cs);
      }
      return;
    }
    const float* base = a.dy + pix0 * a.dy_cs + a.dy_coff + co0 + qa * 4;
#pragma unroll
    for (int i = 0; i < AC; ++i) {
      const int pr = tid / NQA + i * (256 / NQA);
      areg[i] = *(const f32x4_w2*)(base + (size_t)pr * a.dy_cs);
    }
  };
  auto store_a = [&]() {
#pragma unroll
    for (int i = 0; i < AC; ++i) {
      const int pr = tid / NQA + i * (256 / NQA);
      f16x4_w2 h;
      if (a16) {
        h = hreg[i];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) h[e] = (half_t)areg[i][e];
      }
      *(f16x4_w2*)(As + pr * BM * 2 + ((qa ^ w16_swz<NQA>(pr)) * 8)) = h;
    }
  };
  // B DMA of unit u into stage stg: piece j = (run, pixel, 16-byte chunk) lane-linear per run
  auto issue_b = [&](int u, int stg) {
    const int b = u / (a.Ho * segs), r = u - b * a.Ho * segs;
    const int oy = r / segs, ox0 = (r - oy * segs) * W16_KP;
    unsigned char* Bs = Bs0 + stg * B_BYTES;
#pragma unroll
    for (int j = 0; j < BDMA; ++j) {
      const int q = (wave * BDMA + j) * 64 + lane;  // 16-byte chunk index in [run][pixel][4]
      const int run = q / (W16_KP * 4), w = q % (W16_KP * 4);
      const int pix = w >> 2, ch = (w & 3) ^ (((pix >> 3) & 1) << 1);  // halves swapped on rows with bit 3
      const int kr = run0 + run;  // global run: tap * (Cin / 32) + ci32
      const half_t* src = zero16;
      if (kr < a.nruns) {
        const int cq = a.Cin >> 5, tap = kr / cq, ci = (kr - tap * cq) * 32;
        const int ky = tap / a.kw, kx = tap - ky * a.kw;
        const int iy = oy * a.s - a.p + ky * a.d, ix = (ox0 + pix) * a.s - a.p + kx * a.d;
        if ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
          src = a.x16 + ((size_t)(b * a.H + iy) * a.W + ix) * a.Cin + ci + ch * 8;
      }
      wg_glds16(src, Bs + (wave * BDMA + j) * 1024);
    }
  };

  f32x4_w2 acc[MT][RPW * 2];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < RPW * 2; ++j) acc[i][j] = f32x4_w2{0.f, 0.f, 0.f, 0.f};
  const int fg = lane >> 4, l16 = lane & 15, tq = l16 >> 2, tp = l16 & 3;

  if (u0 < u1) {
    load_a(u0);
    issue_b(u0, 0);
  }
  for (int u = u0, it = 0; u < u1; ++u, ++it) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // A regs and B(u) landed
    __syncthreads();                                    // compute of u - 1 done: As, B stage (u+1)&1 free
    store_a();
    if (u + 1 < u1) {
      issue_b(u + 1, (it + 1) & 1);
      load_a(u + 1);
    }
    __syncthreads();  // As written
    const unsigned char* Bs = Bs0 + (it & 1) * B_BYTES;
#pragma unroll
    for (int ks = 0; ks < W16_KP / 32; ++ks) {
      // rows (pixels) of this lane's tr-read: ks*32 + fg*8 + 4h + tq
      f16x8_w2 af[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        f16x4_w2 lo, hi;
        {
          const int row = ks * 32 + fg * 8 + tq;
          lo = w16_tr(As + row * BM * 2 + (((m * 4 + tp) ^ w16_swz<NQA>(row)) * 8));
        }
        {
          const int row = ks * 32 + fg * 8 + 4 + tq;
          hi = w16_tr(As + row * BM * 2 + (((m * 4 + tp) ^ w16_swz<NQA>(row)) * 8));
        }
        af[m] = f16x8_w2{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const int run = wave + 4 * rr;
        if (run < NR) {
#pragma unroll
          for (int h16 = 0; h16 < 2; ++h16) {  // the run's two 16-channel k-tiles
            f16x4_w2 lo, hi;
            {
              const int row = ks * 32 + fg * 8 + tq;
              lo = w16_tr(Bs + run * RUN_BYTES + row * 64 + (((h16 * 4 + tp) ^ w16_swz<8>(row)) * 8));
            }
            {
              const int row = ks * 32 + fg * 8 + 4 + tq;
              hi = w16_tr(Bs + run * RUN_BYTES + row * 64 + (((h16 * 4 + tp) ^ w16_swz<8>(row)) * 8));
            }
            const f16x8_w2 bf = f16x8_w2{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
            for (int m = 0; m < MT; ++m)
              acc[m][rr * 2 + h16] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[m], bf, acc[m][rr * 2 + h16], 0, 0, 0);
          }
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // partial tile -> this split's slab: D[row = fg*4 + i][col = l16] of tile (m, run k-tile)
  float* sl = a.slab + ((size_t)split * a.Cout + co0) * a.ldn + (size_t)run0 * 32;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int run = wave + 4 * rr;
      if (run < NR) {
#pragma unroll
        for (int h16 = 0; h16 < 2; ++h16)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            sl[(size_t)(m * 16 + fg * 4 + i) * a.ldn + run * 32 + h16 * 16 + l16] = acc[m][rr * 2 + h16][i];
      }
    }
}

template <int BM, int NR>
static int launch_wgrad16(Wg16Args a, float* dwp, hipStream_t st, int torch_ci) {
  constexpr int LDS = W16_KP * BM * 2 + 2 * NR * W16_KP * 64;
  static bool attr = false;
  if (!attr) {
    const hipError_t e =
        hipFuncSetAttribute((const void*)wgrad16_kernel<BM, NR>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  a.mtiles = a.Cout / BM;
  a.ntiles = (a.nruns + NR - 1) / NR;
  a.ldn = a.ntiles * NR * 32;
  const int tiles = a.mtiles * a.ntiles;
  // ~1024 blocks, >= 4 steps each
  int splits = (1024 + tiles - 1) / tiles;
  const int max_splits = (a.units + 3) / 4;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  const int ups = (a.units + splits - 1) / splits;
  splits = (a.units + ups - 1) / ups;
  a.splits = splits;
  a.units_per_split = ups;
  const size_t slab_elems = (size_t)a.Cout * a.ldn;
  void* buf = scratch(kSlotSlab, (size_t)splits * slab_elems * sizeof(float), st);
  if (!buf) return (int)hipErrorOutOfMemory;
  a.slab = (float*)buf;
  hipLaunchKernelGGL((wgrad16_kernel<BM, NR>), dim3(tiles * splits), dim3(256), LDS, st, a);
  return reduce_slabs(a.slab, splits, a.Cout, a.KT, a.ldn, dwp, torch_ci, st);
}

template <int BM>
static int wgrad16_nr(const Wg16Args& a, float* dwp, hipStream_t st, int torch_ci) {
  const int nr = a.nruns;
  if (BM <= 64 && nr % 9 == 0) return launch_wgrad16<BM, 9>(a, dwp, st, torch_ci);
  if (BM <= 64 && nr % 8 == 0) return launch_wgrad16<BM, 8>(a, dwp, st, torch_ci);
  if (nr % 4 == 0) return launch_wgrad16<BM, 4>(a, dwp, st, torch_ci);
  if (nr % 2 == 0) return launch_wgrad16<BM, 2>(a, dwp, st, torch_ci);
  return launch_wgrad16<BM, 1>(a, dwp, st, torch_ci);
}

// ---------------------------------------------------------------------------
// Halo-tile AMP weight gradient for stride-1 3x3 convs (pad = dilation) over
// 32 / 64 channels -- the 512^2 decoder / FAM / head convs of the training
// step (models/model.py:49, 98-102, 413-425).  wgrad16_kernel above stages
// im2col(x): every input pixel crosses LDS nine times, 36 KiB per 64-pixel
// step, and with one step of prefetch the step time was the DMA round trip
// (0.25 ms per 32 -> 32 conv at bs 8, 150 TF/s).  Here a block walks TR = 4 *
// RPW output rows of one 64-pixel column segment per step and stages
//   * the input rows those rows' taps touch, 64 + 2d pixels each (halo
//     included, zero outside the image) -- NTAP 9: TR + 2d rows, every tap
//     read from them by a shifted LDS address; NTAP 3 (one kernel row ky per
//     block, for 64-channel shapes whose nine-tap tile would not fit the
//     registers -- measured no faster than the im2col kernel, not routed): TR
//     rows; NTAP 1: the 1x1 convs (no halo);
//   * dy of the TR rows (fp32 -> fp16 through registers, or the fp16 copy),
// double-buffered with one barrier per step.  The MFMA tiles are those of
// wgrad16_kernel (dy rows x input columns, both read pixel-contiguous with
// ds_read_b64_tr_b16, rows XOR-swizzled by w16_swz -- conflict-free for any
// uniform pixel shift of all lanes, so the tap shifts keep it).  Each wave
// owns RPW output rows of the step and the whole (co, k) tile of the block's
// taps; the four waves' tiles are summed through LDS at the end and the sum
// goes to the split's slab as in wgrad16_kernel (splits = (image, row block,
// segment); the tap groups of one split fill disjoint k ranges of its slab
// row), reduced in order.  Same-box timings, bs 8 (tools/wgrad_bench.py):
// 32 -> 32 at 512^2 0.192 -> 0.105 ms with dy's fp16 copy (0.203 -> 0.165 from
// fp32 dy), dilation 2 0.198 -> 0.135, 1x1 96 -> 32 0.234 -> 0.144.
// ---------------------------------------------------------------------------
struct Wg16hArgs {
  const half_t* x16;  // [B][H][W][CIN] fp16
  int B, H, W;        // = Ho, Wo
  const float* dy;
  const half_t* dy16;  // nullable fp16 copy of dy in dy's layout (dy_cs, dy_coff)
  int dy_cs, dy_coff;
  int steps_per_col;   // H / TR
  int spb;             // steps per block
  int nrb, segs, ntg;  // row blocks per image column, 64-pixel segments per row, tap groups
  int ldn;             // taps * CIN
  float* slab;
};

// D: dilation (= pad) of the 3x3 forms, 0 for the 1x1 form.  Input rows are
// CINP channels wide in LDS (CIN rounded up to a power of two, so the XOR
// swizzle of w16_swz stays inside the row; the pad chunks are never read).
template <int CIN, int COUT, int NTAP, int RPW, int D>
struct Wg16hCfg {
  static constexpr int TR = 4 * RPW;
  static constexpr int CINP = CIN == 96 ? 128 : CIN;
  static constexpr int CINB = CINP * 2, COUTB = COUT * 2;
  static constexpr int MT = COUT / 16, KTC = CIN / 16, NKT = NTAP * KTC;
  static constexpr int AQ = TR * 64 * COUT / 4 / 256;  // dy quads per thread per step
  static constexpr int PXR = 64 + 2 * D;                // pixels per staged input row
  static constexpr int IR = NTAP == 9 ? TR + 2 * D : TR;
  static constexpr int IN_BYTES = IR * PXR * CINB;
  static constexpr int STAGE = IN_BYTES + TR * 64 * COUTB;
  static constexpr int LDS = 2 * STAGE;
  static constexpr int TAPS = NTAP == 1 ? 1 : 9;
  // cross-wave reduction of the tile: 2 waves x MT x NKT x 1 KiB per stage, in NPASS k-slices
  static constexpr int RED = 2 * MT * NKT * 1024;
  static constexpr int NPASS = RED <= STAGE ? 1 : RED <= 2 * STAGE && NKT % 2 == 0 ? 2 : 3;
  static_assert(NKT % NPASS == 0 && RED / NPASS <= STAGE, "reduction passes");
};

template <int CIN, int COUT, int NTAP, int RPW, int D, bool A16>
__global__ __launch_bounds__(256) void wgrad16h_kernel(Wg16hArgs a) {
  using C = Wg16hCfg<CIN, COUT, NTAP, RPW, D>;
  constexpr int TR = C::TR, CINP = C::CINP, CINB = C::CINB, COUTB = C::COUTB, MT = C::MT, KTC = C::KTC,
                NKT = C::NKT, AQ = C::AQ, PXR = C::PXR, IR = C::IR, IN_BYTES = C::IN_BYTES, STAGE = C::STAGE;
  // the two stages are separate LDS objects: hipcc then knows that the DMA into one
  // and the fragment reads of the other do not alias, and does not drain the DMA
  // (vmcnt(0)) before every read (it did with one carved buffer)
  __shared__ __attribute__((aligned(16))) unsigned char stg0[STAGE];
  __shared__ __attribute__((aligned(16))) unsigned char stg1[STAGE];
  auto stage = [&](auto STG_) -> unsigned char* {
    if constexpr (decltype(STG_)::value == 0) return stg0;
    else return stg1;
  };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bid = blockIdx.x;
  const int tg = bid % a.ntg;
  const int split = bid / a.ntg;
  const int seg = split % a.segs;
  const int rest = split / a.segs;
  const int rb = rest % a.nrb, b = rest / a.nrb;
  const int s0 = rb * a.spb, s1 = min(a.steps_per_col, s0 + a.spb);
  const int ox0 = seg * 64;
  // input row 0 of a stage: NTAP 9 -> oy0 - D (every kernel row); NTAP 3 -> oy0 + (tg - 1) D;
  // NTAP 1 (1x1) -> oy0
  const int iy_off = NTAP == 9 ? -D : NTAP == 3 ? (tg - 1) * D : 0;
  const half_t* zero16 = (const half_t*)g_wg_zero;

  // input rows of step s -> stage STG: 16-byte slot q of the stage (LDS-linear per
  // wave-instruction) = pixel row R = q / (CINP/8), slot q % (CINP/8), which holds
  // data chunk slot ^ (w16_swz(R) / 2) (pad chunks >= CIN/8: not loaded)
  constexpr int NQ_IN = IR * PXR * (CINP / 8);
  auto issue_in = [&](int s, auto STG_) {
    const int iy0 = s * TR + iy_off;
#pragma unroll 4
    for (int q0 = 0; q0 < NQ_IN; q0 += 256) {
      const int q = q0 + tid;
      const int R = q / (CINP / 8), sl = q - R * (CINP / 8);
      const int c16 = sl ^ (w16_swz<CINP / 4>(R) >> 1);
      if (q < NQ_IN && (CINP == CIN || c16 < CIN / 8)) {
        const int r = R / PXR, px = R - r * PXR;
        const int iy = iy0 + r, ix = ox0 - D + px;
        const half_t* src = zero16;
        if ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
          src = a.x16 + ((size_t)(b * a.H + iy) * a.W + ix) * CIN + c16 * 8;
        wg_glds16(src, stage(STG_) + (q0 + wave * 64) * 16);
      }
    }
  };
  // dy of step s -> registers (quad i of this thread: q = i * 256 + tid -> pixel q / (COUT/4), quad q % (COUT/4))
  // A16: dy's fp16 copy is read (a compile-time choice: a runtime one put each load in
  // its own branch, and hipcc waited for every load at the join)
  f32x4_w2 areg[A16 ? 1 : AQ];
  f16x4_w2 hreg[A16 ? AQ : 1];
  auto load_dy = [&](int s) {
    const size_t pix0 = (size_t)(b * a.H + s * TR) * a.W + ox0;
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      const int q = i * 256 + tid;
      const int R = q / (COUT / 4), cq = q - R * (COUT / 4);
      const size_t pix = pix0 + (size_t)(R >> 6) * a.W + (R & 63);
      if constexpr (A16)
        hreg[i] = *(const f16x4_w2*)(a.dy16 + pix * a.dy_cs + a.dy_coff + cq * 4);
      else
        areg[i] = *(const f32x4_w2*)(a.dy + pix * a.dy_cs + a.dy_coff + cq * 4);
    }
  };
  auto store_dy = [&](auto STG_) {
    unsigned char* As = stage(STG_) + IN_BYTES;
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      const int q = i * 256 + tid;
      const int R = q / (COUT / 4), cq = q - R * (COUT / 4);
      f16x4_w2 h;
      if constexpr (A16) {
        h = hreg[i];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) h[e] = (half_t)areg[i][e];
      }
      *(f16x4_w2*)(As + R * COUTB + ((cq ^ w16_swz<COUT / 4>(R)) * 8)) = h;
    }
  };

  f32x4_w2 acc[MT][NKT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int k = 0; k < NKT; ++k) acc[m][k] = f32x4_w2{0.f, 0.f, 0.f, 0.f};
  const int fg = lane >> 4, l16 = lane & 15, tq = l16 >> 2, tp = l16 & 3;

  auto compute = [&](auto STG_) {
    // the lane's pixel term, opaque per step: hoisted, the ~150 tap / row /
    // swizzle addresses of a step stayed live across the loop and spilled
    int fgq = fg * 8 + tq;
    asm volatile("" : "+v"(fgq));
    const unsigned char* Bs = stage(STG_);
    const unsigned char* As = Bs + IN_BYTES;
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int lr = wave * RPW + rr;  // local output row
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int p = ks * 32 + fgq;  // this lane's pixel of the lo read (hi: + 4)
        f16x8_w2 af[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int r0 = lr * 64 + p, r1 = r0 + 4;
          const f16x4_w2 lo = w16_tr(As + r0 * COUTB + (((m * 4 + tp) ^ w16_swz<COUT / 4>(r0)) * 8));
          const f16x4_w2 hi = w16_tr(As + r1 * COUTB + (((m * 4 + tp) ^ w16_swz<COUT / 4>(r1)) * 8));
          af[m] = f16x8_w2{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int t = 0; t < NTAP; ++t) {
          const int ky = NTAP == 9 ? t / 3 : 0, kx = NTAP == 1 ? 0 : t % 3;
          const int r0 = (lr + ky * D) * PXR + p + kx * D, r1 = r0 + 4;
#pragma unroll
          for (int c = 0; c < KTC; ++c) {
            const f16x4_w2 lo = w16_tr(Bs + r0 * CINB + (((c * 4 + tp) ^ w16_swz<CINP / 4>(r0)) * 8));
            const f16x4_w2 hi = w16_tr(Bs + r1 * CINB + (((c * 4 + tp) ^ w16_swz<CINP / 4>(r1)) * 8));
            const f16x8_w2 bf = f16x8_w2{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
            for (int m = 0; m < MT; ++m)
              acc[m][t * KTC + c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[m], bf, acc[m][t * KTC + c], 0, 0, 0);
          }
        }
      }
    }
  };

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  // step s from stage CUR; the next step's rows / dy go to the other stage (last read by
  // step s - 1, before the barrier that ended it).  Stages are compile-time in the
  // unrolled pair, so hipcc sees that the DMA and the fragment reads touch disjoint LDS.
  auto step = [&](int s, auto CUR_) {
    constexpr int CUR = decltype(CUR_)::value;
    using NXT = std::integral_constant<int, CUR ^ 1>;
    const bool more = s + 1 < s1;  // uniform
    if (more) {
      issue_in(s + 1, NXT{});
      load_dy(s + 1);
    }
    compute(CUR_);
    if (more) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      store_dy(NXT{});
    }
    __syncthreads();
  };
  if (s0 < s1) {
    issue_in(s0, S0{});
    load_dy(s0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    store_dy(S0{});
    __syncthreads();
  }
  for (int s = s0; s < s1; s += 2) {
    step(s, S0{});
    if (s + 1 < s1) step(s + 1, S1{});
  }
  // every wave holds a partial of the whole (co, k) tile (its own output rows):
  // the four are summed through LDS (the stages are free after the loop's last
  // barrier), NPASS k-slices at a time, and the sum goes to the split's slab --
  // D[row = fg*4 + i][col = l16] of tile (m, k-tile) -- one 16-byte LDS chunk
  // per (wave, m, k-tile, lane), stored by consecutive threads as consecutive columns
  constexpr int NPASS = C::NPASS, NKP = NKT / NPASS;
  constexpr int WSTRIDE = MT * NKP * 64;  // f32x4 chunks per wave per pass
  // waves 0, 1 park in stage 0, waves 2, 3 in stage 1
  f32x4_w2* red0 = (f32x4_w2*)stg0;
  f32x4_w2* red1 = (f32x4_w2*)stg1;
  float* sl = a.slab + (size_t)split * COUT * a.ldn + (size_t)tg * NTAP * CIN;
#pragma unroll
  for (int ps = 0; ps < NPASS; ++ps) {
    if (ps) __syncthreads();  // the previous pass's sums are read
    f32x4_w2* mine = (wave < 2 ? red0 : red1) + (wave & 1) * WSTRIDE;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int k = 0; k < NKP; ++k) mine[(m * NKP + k) * 64 + lane] = acc[m][ps * NKP + k];
    __syncthreads();
    for (int c = tid; c < WSTRIDE; c += 256) {
      const f32x4_w2 v = red0[c] + red0[WSTRIDE + c] + red1[c] + red1[WSTRIDE + c];
      const int ln = c & 63, mk = c >> 6, m = mk / NKP, k = ps * NKP + mk % NKP;
#pragma unroll
      for (int i = 0; i < 4; ++i) sl[(size_t)(m * 16 + (ln >> 4) * 4 + i) * a.ldn + k * 16 + (ln & 15)] = v[i];
    }
  }
}

template <int CIN, int COUT, int NTAP, int RPW, int D>
static int launch_wgrad16h(Wg16hArgs a, float* dwp, hipStream_t st, int torch_ci) {
  using C = Wg16hCfg<CIN, COUT, NTAP, RPW, D>;
  static_assert(C::LDS <= 160 * 1024, "LDS");
  if (a.H % C::TR) return kErrUnsupported;
  a.ntg = C::TAPS / NTAP;
  a.segs = a.W / 64;
  a.steps_per_col = a.H / C::TR;
  a.ldn = C::TAPS * CIN;
  // ~512 blocks (one per CU at a time, two rounds), >= 2 steps each
  const long long cols = (long long)a.B * a.segs * a.ntg;
  int nrb = (int)((512 + cols - 1) / cols);
  const int max_nrb = (a.steps_per_col + 1) / 2;
  if (nrb > max_nrb) nrb = max_nrb;
  if (nrb < 1) nrb = 1;
  a.spb = (a.steps_per_col + nrb - 1) / nrb;
  a.nrb = (a.steps_per_col + a.spb - 1) / a.spb;
  const int splits = a.B * a.nrb * a.segs;
  const size_t slab_elems = (size_t)COUT * a.ldn;
  void* buf = scratch(kSlotSlab, (size_t)splits * slab_elems * sizeof(float), st);
  if (!buf) return (int)hipErrorOutOfMemory;
  a.slab = (float*)buf;
  if (a.dy16)
    hipLaunchKernelGGL((wgrad16h_kernel<CIN, COUT, NTAP, RPW, D, true>), dim3(splits * a.ntg), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((wgrad16h_kernel<CIN, COUT, NTAP, RPW, D, false>), dim3(splits * a.ntg), dim3(256), 0, st, a);
  const int KT = C::TAPS * CIN;
  return reduce_slabs(a.slab, splits, COUT, KT, a.ldn, dwp, torch_ci, st);
}

// 32 -> 32 only: the one-kernel-row forms of 64 -> 32 / 32 -> 64 / 64 -> 64 measured
// even / slower than the im2col kernel (bs 8: 0.333 vs 0.337, 0.370 vs 0.235, 0.476
// vs 0.132 ms -- the 64-channel tiles spill), so those shapes stay there
template <int D>
static int wgrad16h_d(const Wg16hArgs& a, int Cin, int Cout, float* dwp, hipStream_t st, int torch_ci) {
  if (Cin == 32 && Cout == 32) return launch_wgrad16h<32, 32, 9, D == 1 ? 2 : 1, D>(a, dwp, st, torch_ci);
  return kErrUnsupported;
}

// the halo form's shapes (k 3: pad = dil <= 2; k 1: stride 1, no padding); kErrUnsupported otherwise
static int wgrad16h(const void* x16, int B, int H, int W, int Cin, const float* dy, int Cout, int dy_cs, int dy_coff,
                    int k, int dil, float* dwp, hipStream_t st, int torch_ci, const void* dy16) {
  if (W % 64) return kErrUnsupported;
  Wg16hArgs a;
  memset(&a, 0, sizeof(a));
  a.x16 = (const half_t*)x16; a.B = B; a.H = H; a.W = W;
  a.dy = dy; a.dy16 = (const half_t*)dy16; a.dy_cs = dy_cs; a.dy_coff = dy_coff;
  if (k == 1) {
    // the multi-scale head fusion 96 -> 32 and the EnhancedFAM fusion 128 -> 32 (model.py:49, 413-414)
    if (Cin == 96 && Cout == 32) return launch_wgrad16h<96, 32, 1, 1, 0>(a, dwp, st, torch_ci);
    if (Cin == 128 && Cout == 32) return launch_wgrad16h<128, 32, 1, 1, 0>(a, dwp, st, torch_ci);
    return kErrUnsupported;
  }
  if (k != 3) return kErrUnsupported;
  if (dil == 1) return wgrad16h_d<1>(a, Cin, Cout, dwp, st, torch_ci);
  if (dil == 2) return wgrad16h_d<2>(a, Cin, Cout, dwp, st, torch_ci);
  return kErrUnsupported;
}

// AMP entry (upr_t_conv_wgrad16): x16 = the compact fp16 copy of x ([B][H][W][Cin]);
// kErrUnsupported when the shape does not fit (the caller falls back to fp32)
int wgrad16_gemm(const void* x16, int B, int H, int W, int Cin, const float* dy, int Ho, int Wo, int Cout, int dy_cs,
                 int dy_coff, int kh, int kw, int stride, int pad, int dil, float* dwp, hipStream_t st, int torch_ci,
                 const void* dy16) {
  if (Wo % W16_KP || Cin % 32 || Cout % 32 || dy_cs % 4 || dy_coff % 4 || ((uintptr_t)dy % 16) ||
      ((uintptr_t)x16 % 16) || (!torch_ci && ((uintptr_t)dwp % 16)))
    return kErrUnsupported;
  const long long P = (long long)B * Ho * Wo;
  if (P >= (1ll << 30) || (long long)B * H * W * Cin >= (1ll << 31)) return kErrUnsupported;
  Wg16Args a;
  memset(&a, 0, sizeof(a));
  a.x16 = (const half_t*)x16; a.B = B; a.H = H; a.W = W; a.Cin = Cin;
  a.dy = dy; a.Ho = Ho; a.Wo = Wo; a.Cout = Cout; a.dy_cs = dy_cs; a.dy_coff = dy_coff;
  a.dy16 = ((uintptr_t)dy16 % 8) ? nullptr : (const half_t*)dy16;
  a.kh = kh; a.kw = kw; a.s = stride; a.p = pad; a.d = dil;
  a.KT = kh * kw * Cin;
  a.nruns = a.KT / 32;
  a.units = (int)(P / W16_KP);
  if (((kh == 3 && kw == 3 && pad == dil) || (kh == 1 && kw == 1 && pad == 0)) && stride == 1 && Ho == H &&
      Wo == W) {
    const int rc = wgrad16h(x16, B, H, W, Cin, dy, Cout, dy_cs, dy_coff, kh, dil, dwp, st, torch_ci, a.dy16);
    if (rc != kErrUnsupported) return rc;
  }
  if (Cout % 128 == 0) return wgrad16_nr<128>(a, dwp, st, torch_ci);
  if (Cout % 64 == 0) return wgrad16_nr<64>(a, dwp, st, torch_ci);
  return wgrad16_nr<32>(a, dwp, st, torch_ci);
}

// Entry from train.hip's upr_t_conv_wgrad (same contract: dwp += ...).
int wgrad_gemm(const float* x, int B, int H, int W, int Cin, int x_cs, int x_coff, const float* dy, int Ho, int Wo,
               int Cout, int dy_cs, int dy_coff, int kh, int kw, int stride, int pad, int dil, float* dwp,
               hipStream_t st, int torch_ci) {
  if (x_cs % 4 || x_coff % 4 || dy_cs % 4 || dy_coff % 4 || ((uintptr_t)x % 16) || ((uintptr_t)dy % 16) ||
      (!torch_ci && ((uintptr_t)dwp % 16)))
    return kErrUnsupported;
  const long long P = (long long)B * Ho * Wo;
  if (P >= (1ll << 30) || (long long)B * H * W >= (1ll << 31)) return kErrUnsupported;
  WgArgs a;
  memset(&a, 0, sizeof(a));
  a.x = x; a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.x_cs = x_cs; a.x_coff = x_coff;
  a.dy = dy; a.Ho = Ho; a.Wo = Wo; a.Cout = Cout; a.dy_cs = dy_cs; a.dy_coff = dy_coff;
  a.kh = kh; a.kw = kw; a.s = stride; a.p = pad; a.d = dil;
  a.KT = kh * kw * Cin;
  a.P = (int)P;
  if (Cout % 128 == 0) return launch_wgrad_gemm<128, 64>(a, dwp, st, torch_ci);
  if (Cout % 64 == 0) return launch_wgrad_gemm<64, 128>(a, dwp, st, torch_ci);
  return launch_wgrad_gemm<32, 256>(a, dwp, st, torch_ci);
}

}  // namespace upr
