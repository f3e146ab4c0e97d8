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

// out[g][co][k] = sum of slabs [g*G, min((g+1)*G, splits)) in order (grid.y = group)
constexpr int WG_GROUP = 16;
__global__ __launch_bounds__(256) void wgrad_group_kernel(const float* __restrict__ slab, int splits, int Cout, int KT,
                                                          int ldn, float* __restrict__ out) {
  const int n4 = Cout * KT / 4;
  const int g = blockIdx.y;
  const int s0 = g * WG_GROUP, s1 = min(splits, s0 + WG_GROUP);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) {
    const int e = i * 4;
    const int co = e / KT, k = e - co * KT;  // KT % 4 == 0: a quad never crosses rows
    f32x4_w2 acc = *(const f32x4_w2*)(slab + ((size_t)s0 * Cout + co) * ldn + k);
    for (int sp = s0 + 1; sp < s1; ++sp) acc += *(const f32x4_w2*)(slab + ((size_t)sp * Cout + co) * ldn + k);
    *(f32x4_w2*)(out + ((size_t)g * Cout + co) * ldn + k) = acc;
  }
}

// dwp[co][k] += sum over n partial slabs (in order); torch_ci > 0: the
// gradient goes straight into PyTorch's [Co][Ci][kh][kw] layout instead
// (k = tap * Ci + ci; the 4 k of a quad share the tap), no packed buffer /
// unpack pass
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int n, int Cout, int KT,
                                                           int ldn, float* __restrict__ dwp, int torch_ci) {
  const int n4 = Cout * KT / 4;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) {
    const int e = i * 4;
    const int co = e / KT, k = e - co * KT;
    f32x4_w2 acc = *(const f32x4_w2*)(part + (size_t)co * ldn + k);
    for (int sp = 1; sp < n; ++sp) acc += *(const f32x4_w2*)(part + ((size_t)sp * Cout + co) * ldn + k);
    if (torch_ci) {
      const int taps = KT / torch_ci, tap = k / torch_ci, ci = k - tap * torch_ci;
      float* o = dwp + ((size_t)co * torch_ci + ci) * taps + tap;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[(size_t)j * taps] += acc[j];
    } else {
      f32x4_w2* o = (f32x4_w2*)(dwp + e);
      *o = *o + acc;
    }
  }
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
  const int groups = splits > WG_GROUP ? (splits + WG_GROUP - 1) / WG_GROUP : 0;
  const size_t slab_elems = (size_t)a.Cout * a.ldn;
  void* buf = scratch(kSlotSlab, (size_t)(splits + groups) * slab_elems * sizeof(float), st);
  if (!buf) return (int)hipErrorOutOfMemory;
  a.slab = (float*)buf;
  hipLaunchKernelGGL((wgrad_gemm_kernel<BM, BN>), dim3(tiles * splits), dim3(256), LDS, st, a);
  const int n4 = a.Cout * a.KT / 4;
  const int g1 = (n4 + 255) / 256 < 1024 ? (n4 + 255) / 256 : 1024;
  const float* part = a.slab;
  int nparts = splits;
  if (groups) {
    float* out = a.slab + (size_t)splits * slab_elems;
    hipLaunchKernelGGL(wgrad_group_kernel, dim3(g1, groups), dim3(256), 0, st, (const float*)a.slab, splits, a.Cout,
                       a.KT, a.ldn, out);
    part = out;
    nparts = groups;
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(g1), dim3(256), 0, st, part, nparts, a.Cout, a.KT, a.ldn, dwp,
                     torch_ci);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// AMP weight gradient (trainers/train.py:72 runs the convs under autocast:
// their weight gradients are products of the fp16 input and the fp16 output
// gradient): v_mfma_f32_16x16x32_f16, fp32 accumulation, fp32 result.
//
// * K (the reduction) = output pixels in steps of 64 consecutive pixels of one
//   output row (Wo % 64 == 0); split-K over those row segments into slabs,
//   reduced in order by wgrad_group / wgrad_reduce (deterministic).
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
  const half_t* dy16;  // nullable: dy's compact [pixel][Cout] fp16 copy (its producer's), read instead of dy
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
      const half_t* base = a.dy16 + pix0 * a.Cout + co0 + qa * 4;
#pragma unroll
      for (int i = 0; i < AC; ++i) {
        const int pr = tid / NQA + i * (256 / NQA);
        hreg[i] = *(const f16x4_w2*)(base + (size_t)pr * a.Cout);
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
  const int groups = splits > WG_GROUP ? (splits + WG_GROUP - 1) / WG_GROUP : 0;
  const size_t slab_elems = (size_t)a.Cout * a.ldn;
  void* buf = scratch(kSlotSlab, (size_t)(splits + groups) * slab_elems * sizeof(float), st);
  if (!buf) return (int)hipErrorOutOfMemory;
  a.slab = (float*)buf;
  hipLaunchKernelGGL((wgrad16_kernel<BM, NR>), dim3(tiles * splits), dim3(256), LDS, st, a);
  const int n4 = a.Cout * a.KT / 4;
  const int g1 = (n4 + 255) / 256 < 1024 ? (n4 + 255) / 256 : 1024;
  const float* part = a.slab;
  int nparts = splits;
  if (groups) {
    float* out = a.slab + (size_t)splits * slab_elems;
    hipLaunchKernelGGL(wgrad_group_kernel, dim3(g1, groups), dim3(256), 0, st, (const float*)a.slab, splits, a.Cout,
                       a.KT, a.ldn, out);
    part = out;
    nparts = groups;
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(g1), dim3(256), 0, st, part, nparts, a.Cout, a.KT, a.ldn, dwp,
                     torch_ci);
  return (int)hipGetLastError();
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
