// Streaming halo convolution for the HBM-bound fp16 layers: stride-1 3x3 over
// 32 or 64 channels at the 512^2 / 256^2 levels (UpBlock convs of dec1/dec2,
// models/model.py:261-269; the residual head + illumination, :324-328 and
// :351-358; EnhancedFAM's fused branch3/branch4 first convs, :35-44).
//
// These layers move ~130 B per output pixel for ~18 KFLOP: at 8 TB/s the HBM
// time is ~2x the fp16 MFMA time, so what matters is keeping enough bytes in
// flight per CU.  Structure:
//
// * Persistent blocks (256 threads, 4 waves) walk TH x 32 output tiles; the
//   tiles of each XCD are one contiguous band, so the halo rows shared by
//   neighbouring tiles meet in that XCD's L2.
// * The input REGION of a tile ((TH+2) x 34 pixels, all C channels) is
//   staged global -> LDS by LDS-DMA (global_load_lds_dwordx4) into one of two
//   slots; the DMA of tile t+1 is issued before the MFMAs of tile t and stays
//   in flight through tile t's epilogue (raw s_barrier + counted vmcnt: the
//   epilogue's residual / input loads are inline asm so that hipcc does not
//   drain the DMA with a vmcnt(0) at their use).
// * The whole filter sits in LDS for the block's lifetime.
// * Roles swapped in the MFMA (A = weights, B = pixels): every lane ends with
//   4 consecutive output channels of one pixel, so the epilogue stores 8-byte
//   channel runs straight from the accumulators (no LDS transpose) and the
//   residual head reduces over channels with two lane shuffles.
// * LDS images are lane-linear (LDS-DMA), 16-byte chunks XOR-swizzled on the
//   source address: pixel q of a 64-byte row image stores logical chunk c at
//   c ^ (((q >> 2) & 1) << 1), of a 128-byte image at c ^ (q & 7): the
//   fragment reads (16 consecutive pixels from ANY start) are then conflict
//   free in every ds_read_b128 lane group (checked exhaustively on the host
//   for all 16 start offsets).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "upr_common.h"

namespace upr {

typedef float f32x4_s __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8_s __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4_s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_void_ptr_s;

// zero source for out-of-image taps; write sink for out-of-image outputs (every
// lane issues the same number of memory instructions in every tile, which is
// what makes the counted vmcnt waits exact)
__device__ __attribute__((aligned(256))) uint4 g_stream_zero[16];
__device__ __attribute__((aligned(256))) uint2 g_stream_sink[64 * 64];

constexpr int ST_TW = 32;  // tile width (output pixels)
// L2 prefetch of tile t+2 (prefetch_region): measured 5-8% SLOWER on the FAM
// fusion and the 3x3 stream kernels (1.05 -> 1.14 ms, 0.50 -> 0.54 ms), so off
constexpr bool kStreamPrefetch = false;

template <int C, int NB, int TH, bool HEAD>
struct StreamCfg {
  static constexpr int RB = C * 2;                  // bytes per region pixel
  static constexpr int CPP = RB / 16;               // chunks per pixel
  static constexpr int RW = ST_TW + 2, RH = TH + 2;
  static constexpr int RPX = RW * RH;               // region pixels
  static constexpr int NI = (RPX * RB + 4096 - 1) / 4096;  // DMA instructions per wave (4 waves x 1 KiB)
  static constexpr int SLOT = NI * 4096;            // bytes per region slot
  static constexpr int WBYTES = 9 * C * NB * 2;     // resident filter
  static constexpr int LDS = WBYTES + 2 * SLOT + 1024;  // + per-wave prefetch dummy rows
  static constexpr int GPW = TH / 2;                // 16-pixel groups per wave (tile has 2*TH groups)
  static constexpr int NT = NB / 16;                // 16-channel tiles
  static constexpr int KS = C / 32;                 // 32-deep k slices per tap
  // memory instructions per wave per tile (constant by construction)
  static constexpr int G = NI;                      // region DMA
  static constexpr int R = HEAD ? 3 * GPW : 0;      // asm loads (x for the head; residual handled separately)
  static constexpr int S = HEAD ? GPW : GPW * NT;   // stores
  static constexpr int NPF = kStreamPrefetch ? (RH * ((RW * RB + 127) / 128 + 1) + 255) / 256 : 0;
};

__device__ __forceinline__ int region_swz(int q, int cpp) {
  return cpp == 4 ? (((q >> 2) & 1) << 1) : (q & 7);
}

// inline-asm loads: invisible to hipcc's vmcnt bookkeeping (waited for by hand)
__device__ __forceinline__ uint2 asm_load_b64(const void* p) {
  uint2 v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ unsigned asm_load_u16(const void* p) {
  unsigned v;
  asm volatile("global_load_ushort %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ unsigned asm_load_b32(const void* p) {
  unsigned v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// L2 prefetch of a future tile's region: one 4-byte LDS-DMA per 128-byte line
// into a per-wave dummy LDS row (never read), so that the region DMA issued
// one tile later hits L2.  LDS-DMA has no VGPR destination, so nothing has to
// stay allocated while it flies.  Each thread issues exactly NPF of them
// (out-of-image lines read the zero line): the per-wave memory-instruction
// count stays constant for the counted vmcnt waits.
template <int NPF>
__device__ __forceinline__ void prefetch_region(const half_t* src, int cs, int b, int H, int W, int iy0, int ix0,
                                                int rh, int rw, int tid, const void* zero, unsigned char* dummy) {
  const int ix_lo = max(ix0, 0), ix_hi = min(ix0 + rw, W);
  const int row_bytes = (ix_hi - ix_lo) * cs * 2;
  const int lpr = (rw * cs * 2 + 127) / 128 + 1;
#pragma unroll
  for (int k = 0; k < NPF; ++k) {
    const int li = tid + 256 * k;
    const int row = li / lpr, l = li - row * lpr;
    const int iy = iy0 + row;
    const void* p = zero;
    if (row < rh && (unsigned)iy < (unsigned)H && l * 128 < row_bytes)
      p = (const unsigned char*)(src + ((size_t)(b * H + iy) * W + ix_lo) * cs) + l * 128;
    __builtin_amdgcn_global_load_lds(p, (lds_void_ptr_s)dummy, 4, 0, 0);
  }
}

struct StreamArgs {
  ConvOp op;
  int tiles_x, tiles_y, ntiles;
  int res_count;  // residual loads per wave per tile (0 or GPW*NT)
};

template <int C, int NB, int TH, bool HEAD>
__global__ __launch_bounds__(256) void conv_stream_kernel(StreamArgs args) {
  using K = StreamCfg<C, NB, TH, HEAD>;
  const ConvOp& op = args.op;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* Wl = smem;                  // filter [tap][kslice][n][64 B]
  unsigned char* slots = smem + K::WBYTES;   // 2 region slots

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const ConvSeg& sg = op.seg[0];
  const int H = op.Ho, W = op.Wo;

  // ---- tiles of this block: XCD-contiguous bands --------------------------
  const int nblk = gridDim.x;
  const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3;
  const int per_xcd = nblk >> 3;             // grid is a multiple of 8
  const int band0 = (int)((long long)args.ntiles * xcd / 8), band1 = (int)((long long)args.ntiles * (xcd + 1) / 8);
  // tile sequence: band0 + idx, band0 + idx + per_xcd, ...
  auto tile_coords = [&](int t, int& b, int& oy0, int& ox0) {
    const int tx = t % args.tiles_x;
    const int r = t / args.tiles_x;
    const int ty = r % args.tiles_y;
    b = r / args.tiles_y;
    oy0 = ty * TH;
    ox0 = tx * ST_TW;
  };

  // ---- resident filter: global [N][Kpad] (k = tap*C + c) -> LDS ------------
  {
    const half_t* Wg = (const half_t*)op.W;
    constexpr int CH = 9 * C * NB / 8;  // 16-byte chunks
    for (int i = tid; i < CH; i += 256) {
      // LDS chunk i: row-block (tap, ks), row n, chunk pc (4 per 64-B row)
      const int pc = i & 3;
      const int n = (i >> 2) % NB;
      const int tk = (i >> 2) / NB;  // tap * KS + ks
      const int tap = tk / K::KS, ks = tk % K::KS;
      const int c = pc ^ (((n >> 2) & 1) << 1);
      const uint4 v = *(const uint4*)(Wg + (size_t)n * op.Kpad + tap * C + ks * 32 + c * 8);
      *(uint4*)(Wl + (size_t)i * 16) = v;
    }
  }

  // ---- per-lane DMA geometry (tile invariant) ------------------------------
  // instruction j of this wave covers region bytes [(wave*NI + j)*1024, +1024)
  int dq[K::NI];  // packed hy<<16 | hx<<8 | logical chunk, or -1 past the region
#pragma unroll
  for (int j = 0; j < K::NI; ++j) {
    const int u = (wave * K::NI + j) * 64 + lane;  // 16-byte unit
    const int q = u / K::CPP, pc = u % K::CPP;
    if (q < K::RPX) {
      const int c = pc ^ region_swz(q, K::CPP);
      dq[j] = ((q / K::RW) << 16) | ((q % K::RW) << 8) | c;
    } else {
      dq[j] = -1;
    }
  }
  const half_t* src = (const half_t*)sg.src + sg.coff;
  const half_t* zero = (const half_t*)g_stream_zero;

  auto issue_region = [&](int t, int slot) {
    int b, oy0, ox0;
    tile_coords(t, b, oy0, ox0);
    unsigned char* dst = slots + slot * K::SLOT + wave * K::NI * 1024;
#pragma unroll
    for (int j = 0; j < K::NI; ++j) {
      const half_t* p = zero;
      if (dq[j] >= 0) {
        const int iy = oy0 - 1 + (dq[j] >> 16);
        const int ix = ox0 - 1 + ((dq[j] >> 8) & 255);
        if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
          p = src + (size_t)((b * H + iy) * W + ix) * sg.cs + (dq[j] & 255) * 8;
      }
      __builtin_amdgcn_global_load_lds(p, (lds_void_ptr_s)(dst + j * 1024), 16, 0, 0);
    }
  };

  const int first = band0 + idx;
  const int step = per_xcd;
  __syncthreads();  // filter in LDS (ordinary loads: hipcc waited for them)
  if (first < band1) issue_region(first, 0);

  // epilogue constants
  const float* bias = op.bias;
  float bv[K::NT][4];
#pragma unroll
  for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[nt][i] = bias ? bias[nt * 16 + fg * 4 + i] : 0.f;
  float hw2[K::NT][4];
  if constexpr (HEAD) {
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) hw2[nt][i] = op.head_w[nt * 16 + fg * 4 + i];
  }
  const int wswz = ((fr >> 2) & 1) << 1;  // filter row swizzle (rows fr + 16k)

  unsigned char* pf_dummy = slots + 2 * K::SLOT + wave * 256;
  int it = 0;
  for (int t = first; t < band1; t += step, ++it) {
    const int slot = it & 1;
    // (A) the region of tile t has landed: younger than its DMA are only the
    // previous tile's S stores
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::S + K::NPF) : "memory");
    __builtin_amdgcn_s_barrier();
    int b, oy0, ox0;
    tile_coords(t, b, oy0, ox0);
    // residual / head inputs of tile t (asm loads, before the next DMA)
    uint2 res[K::GPW][K::NT];
    unsigned xin[K::GPW][3];
    size_t opix[K::GPW];
    bool ovalid[K::GPW];
#pragma unroll
    for (int g = 0; g < K::GPW; ++g) {
      const int gy = (wave * K::GPW + g) >> 1, gx = ((wave * K::GPW + g) & 1) * 16 + fr;
      const int y = oy0 + gy, x = ox0 + gx;
      ovalid[g] = y < H && x < W;
      opix[g] = ovalid[g] ? (size_t)(b * H + y) * W + x : 0;
      if (args.res_count) {
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt)
          res[g][nt] = asm_load_b64(ovalid[g] ? (const void*)((const half_t*)op.res2 + opix[g] * op.res2_cs + nt * 16 + fg * 4)
                                              : (const void*)zero);
      }
      if constexpr (HEAD) {
        const size_t HW = (size_t)H * W;
        const size_t pb = (size_t)b * 3 * HW + (opix[g] - (size_t)b * HW);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          if (op.x_f16) xin[g][c] = asm_load_u16(ovalid[g] ? (const void*)((const half_t*)op.x_nchw + pb + c * HW) : (const void*)zero);
          else xin[g][c] = asm_load_b32(ovalid[g] ? (const void*)(op.x_nchw + pb + c * HW) : (const void*)zero);
        }
      }
    }
    const bool has_next = t + step < band1;
    if (has_next) issue_region(t + step, slot ^ 1);
    {
      int pb = 0, py = 0, px = 0;
      const bool pf = t + 2 * step < band1;
      if (pf) tile_coords(t + 2 * step, pb, py, px);
      prefetch_region<K::NPF>(src, sg.cs, pb, H, W, pf ? py - 1 : -1000, px - 1, K::RH, K::RW, tid, zero, pf_dummy);
    }

    // ---- MFMAs: D[n][px] = sum_k W[n][k] * X[px][k] -------------------------
    f32x4_s acc[K::NT][K::GPW];
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
      for (int g = 0; g < K::GPW; ++g) acc[nt][g] = f32x4_s{0.f, 0.f, 0.f, 0.f};
    const unsigned char* reg = slots + slot * K::SLOT;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int r = tap / 3, s = tap % 3;
#pragma unroll
      for (int ks = 0; ks < K::KS; ++ks) {
        f16x8_s wf[K::NT];
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt)
          wf[nt] = *(const f16x8_s*)(Wl + ((size_t)((tap * K::KS + ks) * NB + nt * 16 + fr) * 64) + ((fg ^ wswz) * 16));
#pragma unroll
        for (int g = 0; g < K::GPW; ++g) {
          const int gy = (wave * K::GPW + g) >> 1, gx = ((wave * K::GPW + g) & 1) * 16;
          const int q = (gy + r) * K::RW + gx + fr + s;
          const int c = (ks * 4 + fg) ^ region_swz(q, K::CPP);
          const f16x8_s xf = *(const f16x8_s*)(reg + q * K::RB + c * 16);
#pragma unroll
          for (int nt = 0; nt < K::NT; ++nt)
            acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nt], xf, acc[nt][g], 0, 0, 0);
        }
      }
    }

    // (B) this tile's asm loads are done; the next region's DMA (and the L2
    // prefetch behind it) may fly on
    if (has_next) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::G + K::NPF) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // pin every use of the asm-loaded registers below the wait (volatile asm
    // statements keep their order; plain arithmetic could float above it)
#pragma unroll
    for (int g = 0; g < K::GPW; ++g) {
      if (args.res_count) {
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt) asm volatile("" : "+v"(res[g][nt].x), "+v"(res[g][nt].y));
      }
      if constexpr (HEAD) asm volatile("" : "+v"(xin[g][0]), "+v"(xin[g][1]), "+v"(xin[g][2]));
    }

    // ---- epilogue -------------------------------------------------------------
    if constexpr (HEAD) {
      // r = sum_n relu(v_n) * w2_n ; illu = sigmoid(mean_c(x) + r + b2)
#pragma unroll
      for (int g = 0; g < K::GPW; ++g) {
        float part = 0.f;
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) part += fmaxf(acc[nt][g][i] + bv[nt][i], 0.f) * hw2[nt][i];
        part += __shfl_xor(part, 16);
        part += __shfl_xor(part, 32);
        float x0, x1, x2;
        if (op.x_f16) {
          x0 = (float)__builtin_bit_cast(half_t, (unsigned short)(xin[g][0] & 0xffff));
          x1 = (float)__builtin_bit_cast(half_t, (unsigned short)(xin[g][1] & 0xffff));
          x2 = (float)__builtin_bit_cast(half_t, (unsigned short)(xin[g][2] & 0xffff));
        } else {
          x0 = __builtin_bit_cast(float, xin[g][0]);
          x1 = __builtin_bit_cast(float, xin[g][1]);
          x2 = __builtin_bit_cast(float, xin[g][2]);
        }
        const float z = (x0 + x1 + x2) / 3.f + (part + op.head_b);
        const float il = 1.f / (1.f + expf(-z));
        float* dst = (ovalid[g] && fg == 0) ? op.illu + opix[g] : (float*)(g_stream_sink + tid);
        *dst = il;
      }
    } else {
#pragma unroll
      for (int g = 0; g < K::GPW; ++g) {
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = acc[nt][g][i] + bv[nt][i];
            if (op.relu) v[i] = fmaxf(v[i], 0.f);
          }
          if (args.res_count) {
            const f16x4_s rr = __builtin_bit_cast(f16x4_s, res[g][nt]);
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] += (float)rr[i];
          }
          f16x4_s o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = (half_t)v[i];
          uint2* dst = ovalid[g] ? (uint2*)((half_t*)op.out + opix[g] * op.out_cs + op.out_coff + nt * 16 + fg * 4)
                                 : g_stream_sink + tid;
          *dst = __builtin_bit_cast(uint2, o);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// EnhancedFAM fusion GEMM (models/model.py:29-44, :66-78) on the same streaming
// structure: y = relu(Wf3.conv3x3(h3) + Wf4.conv3x3_d2(h4) + Wf1.x + Wf2.maxpool3(x) + b)
// with the fusion 1x1 composed into every branch (model.hip), K = 640, N = 32,
// plus the per-image channel sums of y for the channel attention.
//   * two regions per 4 x 32 tile: h (64 channels = [h3 | h4], 2-pixel halo,
//     8 x 36 px x 128 B) and x (32 channels, 1-pixel halo, 6 x 34 px x 64 B,
//     -inf outside the image: the max-pool ignores padding);
//   * the max-pool branch's operand is the 3x3 max of the x region, taken from
//     LDS while building the MFMA fragment.
// ---------------------------------------------------------------------------
__device__ __attribute__((aligned(256))) unsigned g_stream_ninf[64] = {
#define NINF4 0xFC00FC00u, 0xFC00FC00u, 0xFC00FC00u, 0xFC00FC00u
    NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4
#undef NINF4
};

struct FamCfg {
  static constexpr int TH = 4, GPW = 2, NT = 2, NB = 32;
  static constexpr int HRW = ST_TW + 4, HRH = TH + 4, HPX = HRW * HRH;  // 36 x 8
  static constexpr int XRW = ST_TW + 2, XRH = TH + 2, XPX = XRW * XRH;  // 34 x 6
  static constexpr int HNI = (HPX * 128 + 4095) / 4096;                 // 9
  static constexpr int XNI = (XPX * 64 + 4095) / 4096;                  // 4
  static constexpr int G = HNI + XNI;
  static constexpr int HSLOT = HNI * 4096, XSLOT = XNI * 4096;
  static constexpr int SLOT = HSLOT + XSLOT;
  static constexpr int NSL = 20;                                        // 32-deep k slices
  static constexpr int WBYTES = NSL * NB * 64;
  static constexpr int LDS = WBYTES + 2 * SLOT + 1024;                  // + prefetch dummy rows
  static constexpr int S = GPW * NT;                                    // stores per wave per tile
  static constexpr int HPF = kStreamPrefetch ? (HRH * ((HRW * 128 + 127) / 128 + 1) + 255) / 256 : 0;
  static constexpr int XPF = kStreamPrefetch ? (XRH * ((XRW * 64 + 127) / 128 + 1) + 255) / 256 : 0;
  static constexpr int NPF = HPF + XPF;
};

__global__ __launch_bounds__(256) void conv_stream_fam_kernel(StreamArgs args) {
  using K = FamCfg;
  const ConvOp& op = args.op;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* Wl = smem;
  unsigned char* slots = smem + K::WBYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int H = op.Ho, W = op.Wo;
  const int nblk = gridDim.x;
  const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3;
  const int per_xcd = nblk >> 3;
  const int band0 = (int)((long long)args.ntiles * xcd / 8), band1 = (int)((long long)args.ntiles * (xcd + 1) / 8);
  auto tile_coords = [&](int t, int& b, int& oy0, int& ox0) {
    const int tx = t % args.tiles_x;
    const int r = t / args.tiles_x;
    b = r / args.tiles_y;
    oy0 = (r % args.tiles_y) * K::TH;
    ox0 = tx * ST_TW;
  };
  // resident filter: slice sl = global k [32 sl, 32 sl + 32)
  {
    const half_t* Wg = (const half_t*)op.W;
    for (int i = tid; i < K::NSL * K::NB * 4; i += 256) {
      const int pc = i & 3, n = (i >> 2) % K::NB, sl = (i >> 2) / K::NB;
      const int c = pc ^ (((n >> 2) & 1) << 1);
      *(uint4*)(Wl + (size_t)i * 16) = *(const uint4*)(Wg + (size_t)n * op.Kpad + sl * 32 + c * 8);
    }
  }
  int hq[K::HNI], xq[K::XNI];
#pragma unroll
  for (int j = 0; j < K::HNI; ++j) {
    const int u = (wave * K::HNI + j) * 64 + lane, q = u >> 3, pc = u & 7;
    hq[j] = q < K::HPX ? ((q / K::HRW) << 16) | ((q % K::HRW) << 8) | (pc ^ (q & 7)) : -1;
  }
#pragma unroll
  for (int j = 0; j < K::XNI; ++j) {
    const int u = (wave * K::XNI + j) * 64 + lane, q = u >> 2, pc = u & 3;
    xq[j] = q < K::XPX ? ((q / K::XRW) << 16) | ((q % K::XRW) << 8) | (pc ^ region_swz(q, 4)) : -1;
  }
  const ConvSeg& sh = op.seg[0];
  const ConvSeg& sx = op.seg[2];
  const half_t* hsrc = (const half_t*)sh.src;  // [h3 | h4], pixel stride sh.cs
  const half_t* xsrc = (const half_t*)sx.src + sx.coff;
  const half_t* zero = (const half_t*)g_stream_zero;
  const half_t* ninf = (const half_t*)g_stream_ninf;
  auto issue_region = [&](int t, int slot) {
    int b, oy0, ox0;
    tile_coords(t, b, oy0, ox0);
    unsigned char* hd = slots + slot * K::SLOT + wave * K::HNI * 1024;
    unsigned char* xd = slots + slot * K::SLOT + K::HSLOT + wave * K::XNI * 1024;
#pragma unroll
    for (int j = 0; j < K::HNI; ++j) {
      const half_t* p = zero;
      if (hq[j] >= 0) {
        const int iy = oy0 - 2 + (hq[j] >> 16), ix = ox0 - 2 + ((hq[j] >> 8) & 255);
        if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
          p = hsrc + (size_t)((b * H + iy) * W + ix) * sh.cs + (hq[j] & 255) * 8;
      }
      __builtin_amdgcn_global_load_lds(p, (lds_void_ptr_s)(hd + j * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < K::XNI; ++j) {
      const half_t* p = ninf;
      if (xq[j] >= 0) {
        const int iy = oy0 - 1 + (xq[j] >> 16), ix = ox0 - 1 + ((xq[j] >> 8) & 255);
        if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
          p = xsrc + (size_t)((b * H + iy) * W + ix) * sx.cs + (xq[j] & 255) * 8;
      }
      __builtin_amdgcn_global_load_lds(p, (lds_void_ptr_s)(xd + j * 1024), 16, 0, 0);
    }
  };
  const int first = band0 + idx, step = per_xcd;
  __syncthreads();
  if (first < band1) issue_region(first, 0);
  float bv[K::NT][4];
#pragma unroll
  for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[nt][i] = op.bias ? op.bias[nt * 16 + fg * 4 + i] : 0.f;
  const int wswz = ((fr >> 2) & 1) << 1;
  float pool[K::NT][4];
#pragma unroll
  for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) pool[nt][i] = 0.f;
  int pool_img = -1;
  bool flushed = false;
  unsigned char* pf_dummy = slots + 2 * K::SLOT + wave * 256;
  // flush this lane's pooled sums of image pool_img (reduced over the 16 pixel lanes)
  auto flush = [&]() {
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = pool[nt][i];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        if (fr == 0) atomicAdd(op.pool + (size_t)pool_img * op.N + nt * 16 + fg * 4 + i, v);
        pool[nt][i] = 0.f;
      }
  };

  int it = 0;
  for (int t = first; t < band1; t += step, ++it) {
    const int slot = it & 1;
    if (it == 0 || flushed) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::S + K::NPF) : "memory");
    __builtin_amdgcn_s_barrier();
    flushed = false;
    int b, oy0, ox0;
    tile_coords(t, b, oy0, ox0);
    const bool has_next = t + step < band1;
    if (has_next) issue_region(t + step, slot ^ 1);
    {
      int pb = 0, py = 0, px = 0;
      const bool pf = t + 2 * step < band1;
      if (pf) tile_coords(t + 2 * step, pb, py, px);
      prefetch_region<K::HPF>(hsrc, sh.cs, pb, H, W, pf ? py - 2 : -1000, px - 2, K::HRH, K::HRW, tid, zero, pf_dummy);
      prefetch_region<K::XPF>(xsrc, sx.cs, pb, H, W, pf ? py - 1 : -1000, px - 1, K::XRH, K::XRW, tid, zero, pf_dummy);
    }

    f32x4_s acc[K::NT][K::GPW];
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
      for (int g = 0; g < K::GPW; ++g) acc[nt][g] = f32x4_s{0.f, 0.f, 0.f, 0.f};
    const unsigned char* hreg = slots + slot * K::SLOT;
    const unsigned char* xreg = hreg + K::HSLOT;
    auto wfrag = [&](int sl, f16x8_s (&wf)[K::NT]) {
#pragma unroll
      for (int nt = 0; nt < K::NT; ++nt)
        wf[nt] = *(const f16x8_s*)(Wl + ((size_t)(sl * K::NB + nt * 16 + fr) * 64) + ((fg ^ wswz) * 16));
    };
    // h3 (3x3, d1) and h4 (3x3, d2): slices 0..8 and 9..17
#pragma unroll
    for (int seg = 0; seg < 2; ++seg) {
      const int d = seg + 1;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int r = tap / 3, s = tap % 3;
        f16x8_s wf[K::NT];
        wfrag(seg * 9 + tap, wf);
#pragma unroll
        for (int g = 0; g < K::GPW; ++g) {
          const int gx = g * 16;
          const int q = (wave + 2 + (r - 1) * d) * K::HRW + gx + 2 + (s - 1) * d + fr;
          const int c = (seg * 4 + fg) ^ (q & 7);
          const f16x8_s xf = *(const f16x8_s*)(hreg + q * 128 + c * 16);
#pragma unroll
          for (int nt = 0; nt < K::NT; ++nt)
            acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nt], xf, acc[nt][g], 0, 0, 0);
        }
      }
    }
    // x (1x1) and maxpool3(x) (1x1): slices 18, 19
    {
      f16x8_s w1[K::NT], w2[K::NT];
      wfrag(18, w1);
      wfrag(19, w2);
#pragma unroll
      for (int g = 0; g < K::GPW; ++g) {
        const int gx = g * 16;
        f16x8_s ctr = {}, mx = {};
#pragma unroll
        for (int dr = 0; dr < 3; ++dr)
#pragma unroll
          for (int ds = 0; ds < 3; ++ds) {
            const int q = (wave + dr) * K::XRW + gx + ds + fr;
            const f16x8_s v = *(const f16x8_s*)(xreg + q * 64 + ((fg ^ region_swz(q, 4)) * 16));
            if (dr == 0 && ds == 0) mx = v;
            else mx = __builtin_elementwise_max(mx, v);
            if (dr == 1 && ds == 1) ctr = v;
          }
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt) {
          acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[nt], ctr, acc[nt][g], 0, 0, 0);
          acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w2[nt], mx, acc[nt][g], 0, 0, 0);
        }
      }
    }
    if (has_next) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::G + K::NPF) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // epilogue: y = relu(acc + b) in fp16, pooled sums of the stored values
    if (op.pool && pool_img != b) {
      if (pool_img >= 0) { flush(); flushed = true; }
      pool_img = b;
    }
#pragma unroll
    for (int g = 0; g < K::GPW; ++g) {
      const int y = oy0 + wave, x = ox0 + g * 16 + fr;
      const bool ok = y < H && x < W;
      const size_t opix = ok ? (size_t)(b * H + y) * W + x : 0;
#pragma unroll
      for (int nt = 0; nt < K::NT; ++nt) {
        f16x4_s o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          o[i] = (half_t)fmaxf(acc[nt][g][i] + bv[nt][i], 0.f);
          if (ok) pool[nt][i] += (float)o[i];
        }
        uint2* dst = ok ? (uint2*)((half_t*)op.out + opix * op.out_cs + op.out_coff + nt * 16 + fg * 4)
                        : g_stream_sink + tid;
        *dst = __builtin_bit_cast(uint2, o);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (op.pool && pool_img >= 0) flush();
}

static int launch_stream_fam(const ConvOp& op, hipStream_t st) {
  static int occ = 0;
  if (!occ) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_stream_fam_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       FamCfg::LDS);
    if (e != hipSuccess) return (int)e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)conv_stream_fam_kernel, 256, FamCfg::LDS);
    if (e != hipSuccess) return (int)e;
    if (occ < 1) occ = 1;
  }
  int cus = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  StreamArgs a;
  a.op = op;
  a.tiles_x = cdiv(op.Wo, ST_TW);
  a.tiles_y = cdiv(op.Ho, FamCfg::TH);
  a.ntiles = op.B * a.tiles_x * a.tiles_y;
  a.res_count = 0;
  int grid = std::min(cus * occ, cdiv(a.ntiles, 8) * 8);
  grid = std::max(8, grid / 8 * 8);
  hipLaunchKernelGGL(conv_stream_fam_kernel, dim3(grid), dim3(256), FamCfg::LDS, st, a);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Whole EnhancedFAM conv stack in one pass (fp16): h = relu([branch3_conv1;
// branch4_conv1](x) + b) is computed for the tile's 2-pixel-halo region
// straight into LDS (zero outside the image = the fusion convs' padding) and
// consumed there by the fusion GEMM of conv_stream_fam_kernel — h never
// touches HBM (models/model.py:35-44, :66-78).  Per 4 x 32 tile: x region
// 10 x 38 px (3-pixel halo, zero fill; the max-pool masks out-of-image
// neighbours itself), h region 8 x 36 px x 64 ch, filters of both convs
// resident: 76 + 36 + 2 x 24 KiB = 160 KiB of LDS, one block per CU.
// ---------------------------------------------------------------------------
struct FamFusedCfg {
  static constexpr int TH = 4, GPW = 2, NT = 2, NB = 32;
  static constexpr int XRW = ST_TW + 6, XRH = TH + 6, XPX = XRW * XRH;  // 38 x 10
  static constexpr int HRW = ST_TW + 4, HRH = TH + 4, HPX = HRW * HRH;  // 36 x 8
  static constexpr int XNI = (XPX * 64 + 4095) / 4096;                  // 6
  static constexpr int XSLOT = XNI * 4096;
  static constexpr int HBYTES = HPX * 128;
  static constexpr int W34 = 9 * 64 * 64;                              // [tap][n 64][64 B]
  static constexpr int WF = 20 * NB * 64;                              // [slice][n 32][64 B]
  static constexpr int LDS = W34 + WF + HBYTES + 2 * XSLOT;
  static constexpr int HG = HPX / 16;                                  // 18 groups of 16 h pixels
  static constexpr int HGW = (HG + 3) / 4;                             // per wave (5, last ones partial)
  static constexpr int G = XNI;
  static constexpr int S = GPW * NT;
};

struct FamFusedArgs {
  const half_t* x; int x_cs;
  const half_t* w34; int w34_kpad; const float* b34;   // [64][Kpad] (k = tap*32 + c), bias [64]
  const half_t* wf; int wf_kpad; const float* bf;      // [32][640]
  half_t* out; int out_cs;
  float* pool;
  int B, H, W;
  int tiles_x, tiles_y, ntiles;
};

__global__ __launch_bounds__(256) void conv_fam_fused_kernel(FamFusedArgs a) {
  using K = FamFusedCfg;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* W34l = smem;
  unsigned char* WFl = smem + K::W34;
  unsigned char* hreg = WFl + K::WF;
  unsigned char* xslots = hreg + K::HBYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int H = a.H, W = a.W;
  const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3, per_xcd = gridDim.x >> 3;
  const int band0 = (int)((long long)a.ntiles * xcd / 8), band1 = (int)((long long)a.ntiles * (xcd + 1) / 8);
  auto tile_coords = [&](int t, int& b, int& oy0, int& ox0) {
    const int tx = t % a.tiles_x, r = t / a.tiles_x;
    b = r / a.tiles_y;
    oy0 = (r % a.tiles_y) * K::TH;
    ox0 = tx * ST_TW;
  };
  // resident filters (64-B rows, chunk ^ ((n >> 2) & 1) * 2)
  for (int i = tid; i < 9 * 64 * 4; i += 256) {
    const int pc = i & 3, n = (i >> 2) & 63, tap = i >> 8;
    const int c = pc ^ (((n >> 2) & 1) << 1);
    *(uint4*)(W34l + (size_t)i * 16) = *(const uint4*)(a.w34 + (size_t)n * a.w34_kpad + tap * 32 + c * 8);
  }
  for (int i = tid; i < 20 * K::NB * 4; i += 256) {
    const int pc = i & 3, n = (i >> 2) % K::NB, sl = (i >> 2) / K::NB;
    const int c = pc ^ (((n >> 2) & 1) << 1);
    *(uint4*)(WFl + (size_t)i * 16) = *(const uint4*)(a.wf + (size_t)n * a.wf_kpad + sl * 32 + c * 8);
  }
  int xq[K::XNI];
#pragma unroll
  for (int j = 0; j < K::XNI; ++j) {
    const int u = (wave * K::XNI + j) * 64 + lane, q = u >> 2, pc = u & 3;
    xq[j] = q < K::XPX ? ((q / K::XRW) << 16) | ((q % K::XRW) << 8) | (pc ^ region_swz(q, 4)) : -1;
  }
  const half_t* zero = (const half_t*)g_stream_zero;
  auto issue_region = [&](int t, int slot) {
    int b, oy0, ox0;
    tile_coords(t, b, oy0, ox0);
    unsigned char* xd = xslots + slot * K::XSLOT + wave * K::XNI * 1024;
#pragma unroll
    for (int j = 0; j < K::XNI; ++j) {
      const half_t* p = zero;
      if (xq[j] >= 0) {
        const int iy = oy0 - 3 + (xq[j] >> 16), ix = ox0 - 3 + ((xq[j] >> 8) & 255);
        if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
          p = a.x + (size_t)((b * H + iy) * W + ix) * a.x_cs + (xq[j] & 255) * 8;
      }
      __builtin_amdgcn_global_load_lds(p, (lds_void_ptr_s)(xd + j * 1024), 16, 0, 0);
    }
  };
  const int first = band0 + idx, step = per_xcd;
  __syncthreads();
  if (first < band1) issue_region(first, 0);

  const int wswz = ((fr >> 2) & 1) << 1;
  float b34v[4][4], bfv[K::NT][4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) b34v[nt][i] = a.b34[nt * 16 + fg * 4 + i];
#pragma unroll
  for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) bfv[nt][i] = a.bf[nt * 16 + fg * 4 + i];
  float pool[K::NT][4];
#pragma unroll
  for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) pool[nt][i] = 0.f;
  int pool_img = -1;
  bool flushed = false;
  auto flush = [&]() {
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = pool[nt][i];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        if (fr == 0) atomicAdd(a.pool + (size_t)pool_img * K::NB + nt * 16 + fg * 4 + i, v);
        pool[nt][i] = 0.f;
      }
  };

  int it = 0;
  for (int t = first; t < band1; t += step, ++it) {
    const int slot = it & 1;
    if (it == 0 || flushed) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::S) : "memory");
    __builtin_amdgcn_s_barrier();
    flushed = false;
    int b, oy0, ox0;
    tile_coords(t, b, oy0, ox0);
    const bool has_next = t + step < band1;
    if (has_next) issue_region(t + step, slot ^ 1);
    const unsigned char* xreg = xslots + slot * K::XSLOT;

    // ---- phase 1: h over the 8 x 36 region, into LDS -------------------------
    {
      f32x4_s hacc[4][K::HGW];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int g = 0; g < K::HGW; ++g) hacc[nt][g] = f32x4_s{0.f, 0.f, 0.f, 0.f};
      int hb[K::HGW];  // x-region pixel of this lane's h pixel (tap 0,0)
      // 18 groups over 4 waves: group min(wave + 4g, 17) -> waves 2, 3 redo
      // group 17 as their 5th (same values written twice; no branch inside
      // the MFMA loop)
#pragma unroll
      for (int g = 0; g < K::HGW; ++g) {
        const int q = min(wave + 4 * g, K::HG - 1) * 16 + fr;
        hb[g] = (q / K::HRW) * K::XRW + (q % K::HRW);
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int r = tap / 3, s = tap % 3;
        f16x8_s wf[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          wf[nt] = *(const f16x8_s*)(W34l + ((size_t)(tap * 64 + nt * 16 + fr) * 64) + ((fg ^ wswz) * 16));
#pragma unroll
        for (int g = 0; g < K::HGW; ++g) {
          const int q = hb[g] + r * K::XRW + s;
          const f16x8_s xf = *(const f16x8_s*)(xreg + q * 64 + ((fg ^ region_swz(q, 4)) * 16));
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
            hacc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nt], xf, hacc[nt][g], 0, 0, 0);
        }
      }
#pragma unroll
      for (int g = 0; g < K::HGW; ++g) {
        const int q = min(wave + 4 * g, K::HG - 1) * 16 + fr;
        const int iy = oy0 - 2 + q / K::HRW, ix = ox0 - 2 + q % K::HRW;
        const bool in = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          f16x4_s o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = in ? (half_t)fmaxf(hacc[nt][g][i] + b34v[nt][i], 0.f) : (half_t)0.f;
          const int c = nt * 2 + (fg >> 1);  // 16-byte chunk of channels nt*16 + 4fg
          *(f16x4_s*)(hreg + q * 128 + ((c ^ (q & 7)) * 16) + (fg & 1) * 8) = o;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // ---- phase 2: fusion GEMM (as conv_stream_fam_kernel) --------------------
    f32x4_s acc[K::NT][K::GPW];
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
      for (int g = 0; g < K::GPW; ++g) acc[nt][g] = f32x4_s{0.f, 0.f, 0.f, 0.f};
    auto wfrag = [&](int sl, f16x8_s (&wf)[K::NT]) {
#pragma unroll
      for (int nt = 0; nt < K::NT; ++nt)
        wf[nt] = *(const f16x8_s*)(WFl + ((size_t)(sl * K::NB + nt * 16 + fr) * 64) + ((fg ^ wswz) * 16));
    };
#pragma unroll
    for (int seg = 0; seg < 2; ++seg) {
      const int d = seg + 1;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int r = tap / 3, s = tap % 3;
        f16x8_s wf[K::NT];
        wfrag(seg * 9 + tap, wf);
#pragma unroll
        for (int g = 0; g < K::GPW; ++g) {
          const int q = (wave + 2 + (r - 1) * d) * K::HRW + g * 16 + 2 + (s - 1) * d + fr;
          const int c = (seg * 4 + fg) ^ (q & 7);
          const f16x8_s xf = *(const f16x8_s*)(hreg + q * 128 + c * 16);
#pragma unroll
          for (int nt = 0; nt < K::NT; ++nt)
            acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nt], xf, acc[nt][g], 0, 0, 0);
        }
      }
    }
    {
      f16x8_s w1[K::NT], w2[K::NT];
      wfrag(18, w1);
      wfrag(19, w2);
      const half_t ninf = (half_t)(-INFINITY);
#pragma unroll
      for (int g = 0; g < K::GPW; ++g) {
        const int oy = oy0 + wave, ox = ox0 + g * 16 + fr;
        f16x8_s ctr = {}, mx;
#pragma unroll
        for (int e = 0; e < 8; ++e) mx[e] = ninf;
#pragma unroll
        for (int dr = 0; dr < 3; ++dr)
#pragma unroll
          for (int ds = 0; ds < 3; ++ds) {
            const int q = (wave + 2 + dr) * K::XRW + g * 16 + 2 + ds + fr;
            const f16x8_s v = *(const f16x8_s*)(xreg + q * 64 + ((fg ^ region_swz(q, 4)) * 16));
            const bool in = (unsigned)(oy + dr - 1) < (unsigned)H && (unsigned)(ox + ds - 1) < (unsigned)W;
            if (in) mx = __builtin_elementwise_max(mx, v);
            if (dr == 1 && ds == 1) ctr = v;
          }
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt) {
          acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[nt], ctr, acc[nt][g], 0, 0, 0);
          acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w2[nt], mx, acc[nt][g], 0, 0, 0);
        }
      }
    }
    if (has_next) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::G) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.pool && pool_img != b) {
      if (pool_img >= 0) { flush(); flushed = true; }
      pool_img = b;
    }
#pragma unroll
    for (int g = 0; g < K::GPW; ++g) {
      const int y = oy0 + wave, x = ox0 + g * 16 + fr;
      const bool ok = y < H && x < W;
      const size_t opix = ok ? (size_t)(b * H + y) * W + x : 0;
#pragma unroll
      for (int nt = 0; nt < K::NT; ++nt) {
        f16x4_s o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          o[i] = (half_t)fmaxf(acc[nt][g][i] + bfv[nt][i], 0.f);
          if (ok) pool[nt][i] += (float)o[i];
        }
        uint2* dst = ok ? (uint2*)(a.out + opix * a.out_cs + nt * 16 + fg * 4) : g_stream_sink + tid;
        *dst = __builtin_bit_cast(uint2, o);
      }
    }
  }
  if (a.pool && pool_img >= 0) flush();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int launch_fam_fused(const void* x, int x_cs, const void* w34, int w34_kpad, const float* b34, const void* wf,
                     int wf_kpad, const float* bf, void* out, int out_cs, float* pool, int B, int H, int W,
                     hipStream_t st) {
  if (x_cs % 8 || out_cs % 4 || wf_kpad < 640 || w34_kpad < 288 || (uintptr_t)x % 16) return kErrShape;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)conv_fam_fused_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, FamFusedCfg::LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  int cus = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  FamFusedArgs a;
  a.x = (const half_t*)x; a.x_cs = x_cs;
  a.w34 = (const half_t*)w34; a.w34_kpad = w34_kpad; a.b34 = b34;
  a.wf = (const half_t*)wf; a.wf_kpad = wf_kpad; a.bf = bf;
  a.out = (half_t*)out; a.out_cs = out_cs; a.pool = pool;
  a.B = B; a.H = H; a.W = W;
  a.tiles_x = cdiv(W, ST_TW);
  a.tiles_y = cdiv(H, FamFusedCfg::TH);
  a.ntiles = B * a.tiles_x * a.tiles_y;
  int grid = std::min(cus, cdiv(a.ntiles, 8) * 8);
  grid = std::max(8, grid / 8 * 8);
  hipLaunchKernelGGL(conv_fam_fused_kernel, dim3(grid), dim3(256), FamFusedCfg::LDS, st, a);
  return (int)hipGetLastError();
}

template <int C, int NB, int TH, bool HEAD>
static int launch_stream_cfg(const ConvOp& op, hipStream_t st) {
  using K = StreamCfg<C, NB, TH, HEAD>;
  static int occ = 0;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_stream_kernel<C, NB, TH, HEAD>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS);
    if (e != hipSuccess) return (int)e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)conv_stream_kernel<C, NB, TH, HEAD>, 256,
                                                     K::LDS);
    if (e != hipSuccess) return (int)e;
    if (occ < 1) occ = 1;
    attr = true;
  }
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  StreamArgs a;
  a.op = op;
  a.tiles_x = cdiv(op.Wo, ST_TW);
  a.tiles_y = cdiv(op.Ho, TH);
  a.ntiles = op.B * a.tiles_x * a.tiles_y;
  a.res_count = op.res2 ? 1 : 0;
  int grid = cus * occ;
  grid = std::min(grid, cdiv(a.ntiles, 8) * 8);
  grid = std::max(8, grid / 8 * 8);
  hipLaunchKernelGGL((conv_stream_kernel<C, NB, TH, HEAD>), dim3(grid), dim3(256), K::LDS, st, a);
  return (int)hipGetLastError();
}

// UPR_CONV_STREAM=0 disables this path (A/B timing)
static bool stream_enabled() {
  static int en = -1;
  if (en < 0) {
    const char* e = getenv("UPR_CONV_STREAM");
    en = (e && strcmp(e, "0") == 0) ? 0 : 1;
  }
  return en == 1;
}

// fp16 only; kErrUnsupported for every op this kernel does not take
static bool fam_program(const ConvOp& op) {
  if (op.nseg != 4 || op.N != 32 || op.store != kStoreNHWC || op.res1 || op.res2 || op.img_bias || op.scale) return false;
  if (op.Kpad != 640 || op.Wo < 24 || op.Ho < 8 || op.out_cs % 4 || op.out_coff % 4) return false;
  const ConvSeg* s = op.seg;
  auto same_res = [&](const ConvSeg& q) { return q.Hin == op.Ho && q.Win == op.Wo && q.stride == 1 && q.C == 32; };
  for (int i = 0; i < 4; ++i)
    if (!same_res(s[i]) || s[i].kbase != (i < 2 ? 288 * i : 576 + 32 * (i - 2))) return false;
  if (s[0].kh != 3 || s[0].dil != 1 || s[0].pad != 1 || s[0].pre != kPreNone || s[0].coff != 0) return false;
  if (s[1].kh != 3 || s[1].dil != 2 || s[1].pad != 2 || s[1].pre != kPreNone || s[1].coff != 32) return false;
  if (s[0].src != s[1].src || s[0].cs != 64 || s[1].cs != 64 || (uintptr_t)s[0].src % 16) return false;
  if (s[2].kh != 1 || s[2].pre != kPreNone || s[3].kh != 1 || s[3].pre != kPreMaxPool3) return false;
  if (s[2].src != s[3].src || s[2].cs != s[3].cs || s[2].coff != s[3].coff || s[2].cs % 8 || s[2].coff % 8) return false;
  return (uintptr_t)s[2].src % 16 == 0;
}

int launch_conv_stream(const ConvOp& op, hipStream_t st) {
  if (!stream_enabled()) return kErrUnsupported;
  if (fam_program(op)) return launch_stream_fam(op, st);
  if (op.nseg != 1) return kErrUnsupported;
  const ConvSeg& s = op.seg[0];
  if (s.kh != 3 || s.kw != 3 || s.stride != 1 || s.dil != 1 || s.pad != 1 || s.pre != kPreNone) return kErrUnsupported;
  if (s.Hin != op.Ho || s.Win != op.Wo) return kErrUnsupported;
  if ((s.C != 32 && s.C != 64) || s.cs % 8 || s.coff % 8 || (uintptr_t)s.src % 16) return kErrUnsupported;
  if (op.res1 || op.img_bias || op.pool || op.scale || op.Kpad % 8 || s.kbase != 0) return kErrUnsupported;
  if (op.Wo < 24 || op.Ho < 8) return kErrUnsupported;
  if (op.store == kStoreHeadIllu) {
    if (op.N != 32 || s.C != 32 || op.res2) return kErrUnsupported;
    return launch_stream_cfg<32, 32, 8, true>(op, st);
  }
  if (op.store != kStoreNHWC || op.out_cs % 4 || op.out_coff % 4) return kErrUnsupported;
  if (op.res2 && op.res2_cs % 4) return kErrUnsupported;
  if (s.C == 32 && op.N == 32) return launch_stream_cfg<32, 32, 8, false>(op, st);
  if (s.C == 32 && op.N == 64) return launch_stream_cfg<32, 64, 8, false>(op, st);
  if (s.C == 64 && op.N == 64) return launch_stream_cfg<64, 64, 4, false>(op, st);
  return kErrUnsupported;
}

}  // namespace upr
