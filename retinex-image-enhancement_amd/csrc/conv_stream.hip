// Streaming halo convolution for the HBM-bound fp16 layers: stride-1 3x3 over
// 32 or 64 channels at the 512^2 / 256^2 levels (UpBlock convs of dec1/dec2,
// models/model.py:261-269; the residual head + illumination, :324-328 and
// :351-358; EnhancedFAM's fused branch3/branch4 first convs, :35-44) and the
// EnhancedFAM fusion GEMM (:29-44, :66-78).
//
// * Persistent blocks (256 threads, 4 waves) walk TH x 32 output tiles; the
//   tiles of each XCD are one contiguous band, so the halo rows shared by
//   neighbouring tiles meet in that XCD's L2.
// * The input REGION of a tile (tile + halo, all channels) is staged global ->
//   LDS by LDS-DMA (global_load_lds_dwordx4) into one of two slots; the DMA of
//   tile t+1 is issued before the MFMAs of tile t and stays in flight through
//   tile t's epilogue (raw s_barrier + counted vmcnt: the epilogue's residual /
//   input loads are inline asm so that hipcc does not drain the DMA with a
//   vmcnt(0) at their use).
// * Region LDS image = "chunk planes": plane c holds 16-byte chunk c (channels
//   8c..8c+7) of every region pixel, pixel-major.  One DMA instruction fills 64
//   consecutive pixels of one plane (lane-linear as LDS-DMA requires), and an
//   MFMA fragment (16 consecutive pixels x one chunk) is 256 contiguous bytes:
//   conflict-free ds_read_b128 whose address is a per-lane base plus a
//   compile-time immediate -- no per-read swizzle arithmetic (the XOR-swizzled
//   pixel-major image of the first version spent ~7 VALU per MFMA on it and
//   was issue-bound, PMC SQ_INSTS_VALU / SQ_INSTS_MFMA).
// * The whole filter sits in LDS for the block's lifetime (64-byte rows,
//   chunk ^ ((n >> 2) & 1) * 2: conflict-free, lane-constant swizzle).
// * Roles swapped in the MFMA (A = weights, B = pixels): every lane ends with
//   4 consecutive output channels of one pixel, so the epilogue stores 8-byte
//   channel runs straight from the accumulators (no LDS transpose) and the
//   residual head reduces over channels with two lane shuffles.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "upr_common.h"

namespace upr {

typedef float f32x4_s __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8_s __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4_s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_void_ptr_s;

// zero / -inf sources for out-of-image region pixels (>= 8 chunks each); write
// sink for out-of-image outputs (every lane issues the same number of memory
// instructions in every tile, which is what makes the counted vmcnt waits exact)
__device__ __attribute__((aligned(256))) uint4 g_stream_zero[16];
__device__ __attribute__((aligned(256))) uint2 g_stream_sink[64 * 64];
__device__ __attribute__((aligned(256))) unsigned g_stream_ninf[64] = {
#define NINF4 0xFC00FC00u, 0xFC00FC00u, 0xFC00FC00u, 0xFC00FC00u
    NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4
#undef NINF4
};

constexpr int ST_TW = 32;  // tile width (output pixels)

// A region of RW x RH pixels x NPL chunk planes.  DMA: wave w fills planes
// w, w+4, ... for all NPI 64-pixel groups (the pixel address is computed once
// per group and reused for the wave's planes).
template <int NPL, int RW, int RH>
struct Region {
  static constexpr int RPX = RW * RH;
  static constexpr int NPI = (RPX + 63) / 64;     // 64-pixel groups
  static constexpr int PLANE = NPI * 1024;        // bytes per chunk plane
  static constexpr int BYTES = NPL * PLANE;
  static constexpr int PPW = NPL / 4;             // planes per wave
  static constexpr int G = NPI * PPW;             // DMA instructions per wave per region
  static_assert(NPL % 4 == 0, "planes are split over the 4 waves");
};

// per-lane packed (hy << 16 | hx) of pixel group i, or -1 past the region
template <int RW, int RPX, int NPI>
__device__ __forceinline__ void region_geometry(int (&pq)[NPI], int lane) {
#pragma unroll
  for (int i = 0; i < NPI; ++i) {
    const int q = i * 64 + lane;
    pq[i] = q < RPX ? ((q / RW) << 16) | (q % RW) : -1;
  }
}

// DMA of one region: origin (iy0, ix0) in the image, source pixel stride cs
// (elements) at channel offset 0 of src; `fill` for pixels outside the image
template <int NPL, int RW, int RH>
__device__ __forceinline__ void region_issue(const int (&pq)[Region<NPL, RW, RH>::NPI], const half_t* src, int cs,
                                             int b, int H, int W, int iy0, int ix0, const half_t* fill,
                                             unsigned char* dst, int wave) {
  using R = Region<NPL, RW, RH>;
#pragma unroll
  for (int i = 0; i < R::NPI; ++i) {
    const half_t* p = fill;
    if (pq[i] >= 0) {
      const int iy = iy0 + (pq[i] >> 16), ix = ix0 + (pq[i] & 0xffff);
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) p = src + (size_t)((b * H + iy) * W + ix) * cs;
    }
#pragma unroll
    for (int k = 0; k < R::PPW; ++k) {
      const int c = wave + 4 * k;
      __builtin_amdgcn_global_load_lds(p + c * 8, (lds_void_ptr_s)(dst + c * R::PLANE + i * 1024), 16, 0, 0);
    }
  }
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

// filter [k rows of 32][n] -> LDS [slice][n][64 B], chunk ^ ((n >> 2) & 1) * 2
template <int NB>
__device__ __forceinline__ void load_filter(unsigned char* Wl, const half_t* Wg, int kpad, int nslices, int tid) {
  for (int i = tid; i < nslices * NB * 4; i += 256) {
    const int pc = i & 3, n = (i >> 2) % NB, sl = (i >> 2) / NB;
    const int c = pc ^ (((n >> 2) & 1) << 1);
    *(uint4*)(Wl + (size_t)i * 16) = *(const uint4*)(Wg + (size_t)n * kpad + sl * 32 + c * 8);
  }
}

template <int NT, int NB>
__device__ __forceinline__ void filter_frags(const unsigned char* Wl, int sl, int fr, int fg, int wswz,
                                             f16x8_s (&wf)[NT]) {
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    wf[nt] = *(const f16x8_s*)(Wl + ((size_t)(sl * NB + nt * 16 + fr) * 64) + ((fg ^ wswz) * 16));
}

struct StreamArgs {
  ConvOp op;
  int tiles_x, tiles_y, ntiles;
  int res_count;  // 1: residual (res2) loads in the epilogue
};

// tile t of a persistent block: XCD-contiguous bands
struct TileWalk {
  int band0, band1, first, step;
  __device__ TileWalk(int ntiles) {
    const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3, per_xcd = gridDim.x >> 3;  // grid % 8 == 0
    band0 = (int)((long long)ntiles * xcd / 8);
    band1 = (int)((long long)ntiles * (xcd + 1) / 8);
    first = band0 + idx;
    step = per_xcd;
  }
};

template <int C, int NB, int TH, bool HEAD>
struct StreamCfg {
  using R = Region<C / 8, ST_TW + 2, TH + 2>;
  static constexpr int WBYTES = 9 * C * NB * 2;     // resident filter
  static constexpr int LDS = WBYTES + 2 * R::BYTES;
  static constexpr int GPW = TH / 2;                // 16-pixel groups per wave (tile has 2*TH groups)
  static constexpr int NT = NB / 16;                // 16-channel tiles
  static constexpr int KS = C / 32;                 // 32-deep k slices per tap
  static constexpr int G = R::G;                    // DMA instructions per wave per tile
  static constexpr int S = HEAD ? GPW : GPW * NT;   // stores per wave per tile
};

template <int C, int NB, int TH, bool HEAD>
__global__ __launch_bounds__(256) void conv_stream_kernel(StreamArgs args) {
  using K = StreamCfg<C, NB, TH, HEAD>;
  using R = typename K::R;
  const ConvOp& op = args.op;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* Wl = smem;                  // filter [tap*KS + ks][n][64 B]
  unsigned char* slots = smem + K::WBYTES;   // 2 region slots

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const ConvSeg& sg = op.seg[0];
  const int H = op.Ho, W = op.Wo;
  const TileWalk tw(args.ntiles);
  auto tile_coords = [&](int t, int& b, int& oy0, int& ox0) {
    const int tx = t % args.tiles_x, r = t / args.tiles_x;
    b = r / args.tiles_y;
    oy0 = (r % args.tiles_y) * TH;
    ox0 = tx * ST_TW;
  };

  load_filter<NB>(Wl, (const half_t*)op.W, op.Kpad, 9 * K::KS, tid);
  int pq[R::NPI];
  region_geometry<ST_TW + 2, R::RPX, R::NPI>(pq, lane);
  const half_t* src = (const half_t*)sg.src + sg.coff;
  const half_t* zero = (const half_t*)g_stream_zero;
  auto issue = [&](int t, int slot) {
    int b, oy0, ox0;
    tile_coords(t, b, oy0, ox0);
    region_issue<C / 8, ST_TW + 2, TH + 2>(pq, src, sg.cs, b, H, W, oy0 - 1, ox0 - 1, zero, slots + slot * R::BYTES,
                                          wave);
  };

  __syncthreads();  // filter in LDS (ordinary loads: hipcc waited for them)
  if (tw.first < tw.band1) issue(tw.first, 0);

  float bv[K::NT][4];
#pragma unroll
  for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[nt][i] = op.bias ? op.bias[nt * 16 + fg * 4 + i] : 0.f;
  float hw2[K::NT][4];
  if constexpr (HEAD) {
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) hw2[nt][i] = op.head_w[nt * 16 + fg * 4 + i];
  }
  const int wswz = ((fr >> 2) & 1) << 1;
  // fragment base of this lane: chunk plane fg, pixel (wave's first tile row, fr)
  const int xbase = fg * R::PLANE + (wave * (K::GPW / 2) * (ST_TW + 2) + fr) * 16;

  int it = 0;
  for (int t = tw.first; t < tw.band1; t += tw.step, ++it) {
    const int slot = it & 1;
    // (A) the region of tile t has landed: younger than its DMA are only the
    // previous tile's S stores
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::S) : "memory");
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
      const int gy = wave * (K::GPW / 2) + (g >> 1), gx = (g & 1) * 16 + fr;
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
    const bool has_next = t + tw.step < tw.band1;
    if (has_next) issue(t + tw.step, slot ^ 1);

    // ---- MFMAs: D[n][px] = sum_k W[n][k] * X[px][k] -------------------------
    f32x4_s acc[K::NT][K::GPW];
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
      for (int g = 0; g < K::GPW; ++g) acc[nt][g] = f32x4_s{0.f, 0.f, 0.f, 0.f};
    const unsigned char* xr = slots + slot * R::BYTES + xbase;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int r = tap / 3, s = tap % 3;
#pragma unroll
      for (int ks = 0; ks < K::KS; ++ks) {
        f16x8_s wf[K::NT];
        filter_frags<K::NT, NB>(Wl, tap * K::KS + ks, fr, fg, wswz, wf);
#pragma unroll
        for (int g = 0; g < K::GPW; ++g) {
          const int qc = ((g >> 1) + r) * (ST_TW + 2) + (g & 1) * 16 + s;  // compile-time pixel offset
          const f16x8_s xf = *(const f16x8_s*)(xr + ks * 4 * R::PLANE + qc * 16);
#pragma unroll
          for (int nt = 0; nt < K::NT; ++nt)
            acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nt], xf, acc[nt][g], 0, 0, 0);
        }
      }
    }

    // (B) this tile's asm loads are done; the next region's DMA may fly on
    if (has_next) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::G) : "memory");
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
//     8 x 36 px, 8 planes) and x (32 channels, 1-pixel halo, 6 x 34 px, 4
//     planes, -inf outside the image: the max-pool ignores padding);
//   * the max-pool branch's operand is the 3x3 max of the x region, taken from
//     LDS while building the MFMA fragment.
// ---------------------------------------------------------------------------
struct FamCfg {
  static constexpr int TH = 4, GPW = 2, NT = 2, NB = 32;
  using RH_ = Region<8, ST_TW + 4, TH + 4>;  // h
  using RX_ = Region<4, ST_TW + 2, TH + 2>;  // x
  static constexpr int SLOT = RH_::BYTES + RX_::BYTES;
  static constexpr int NSL = 20;             // 32-deep k slices
  static constexpr int WBYTES = NSL * NB * 64;
  static constexpr int LDS = WBYTES + 2 * SLOT;
  static constexpr int G = RH_::G + RX_::G;
  static constexpr int S = GPW * NT;         // stores per wave per tile
};

__global__ __launch_bounds__(256) void conv_stream_fam_kernel(StreamArgs args) {
  using K = FamCfg;
  using RHh = K::RH_;
  using RXx = K::RX_;
  const ConvOp& op = args.op;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* Wl = smem;
  unsigned char* slots = smem + K::WBYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int H = op.Ho, W = op.Wo;
  const TileWalk tw(args.ntiles);
  auto tile_coords = [&](int t, int& b, int& oy0, int& ox0) {
    const int tx = t % args.tiles_x, r = t / args.tiles_x;
    b = r / args.tiles_y;
    oy0 = (r % args.tiles_y) * K::TH;
    ox0 = tx * ST_TW;
  };
  load_filter<K::NB>(Wl, (const half_t*)op.W, op.Kpad, K::NSL, tid);
  int hq[RHh::NPI], xq[RXx::NPI];
  region_geometry<ST_TW + 4, RHh::RPX, RHh::NPI>(hq, lane);
  region_geometry<ST_TW + 2, RXx::RPX, RXx::NPI>(xq, lane);
  const ConvSeg& sh = op.seg[0];
  const ConvSeg& sx = op.seg[2];
  const half_t* hsrc = (const half_t*)sh.src;  // [h3 | h4], pixel stride sh.cs
  const half_t* xsrc = (const half_t*)sx.src + sx.coff;
  const half_t* zero = (const half_t*)g_stream_zero;
  const half_t* ninf = (const half_t*)g_stream_ninf;
  auto issue = [&](int t, int slot) {
    int b, oy0, ox0;
    tile_coords(t, b, oy0, ox0);
    unsigned char* base = slots + slot * K::SLOT;
    region_issue<8, ST_TW + 4, K::TH + 4>(hq, hsrc, sh.cs, b, H, W, oy0 - 2, ox0 - 2, zero, base, wave);
    region_issue<4, ST_TW + 2, K::TH + 2>(xq, xsrc, sx.cs, b, H, W, oy0 - 1, ox0 - 1, ninf, base + RHh::BYTES, wave);
  };
  __syncthreads();
  if (tw.first < tw.band1) issue(tw.first, 0);
  float bv[K::NT][4];
#pragma unroll
  for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[nt][i] = op.bias ? op.bias[nt * 16 + fg * 4 + i] : 0.f;
  const int wswz = ((fr >> 2) & 1) << 1;
  // lane fragment bases: chunk plane fg, pixel (row `wave` of the tile, fr)
  const int hbase = fg * RHh::PLANE + (wave * (ST_TW + 4) + fr) * 16;
  const int xbase = RHh::BYTES + fg * RXx::PLANE + (wave * (ST_TW + 2) + fr) * 16;
  float pool[K::NT][4];
#pragma unroll
  for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) pool[nt][i] = 0.f;
  int pool_img = -1;
  bool flushed = false;
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
        if (fr == 0) pool_add(op.pool, (size_t)pool_img * op.N + nt * 16 + fg * 4 + i, v);
        pool[nt][i] = 0.f;
      }
  };

  int it = 0;
  for (int t = tw.first; t < tw.band1; t += tw.step, ++it) {
    const int slot = it & 1;
    if (it == 0 || flushed) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::S) : "memory");
    __builtin_amdgcn_s_barrier();
    flushed = false;
    int b, oy0, ox0;
    tile_coords(t, b, oy0, ox0);
    const bool has_next = t + tw.step < tw.band1;
    if (has_next) issue(t + tw.step, slot ^ 1);

    f32x4_s acc[K::NT][K::GPW];
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
      for (int g = 0; g < K::GPW; ++g) acc[nt][g] = f32x4_s{0.f, 0.f, 0.f, 0.f};
    const unsigned char* sl = slots + slot * K::SLOT;
    // h3 (3x3, d1) and h4 (3x3, d2): slices 0..8 and 9..17, planes 0-3 / 4-7
#pragma unroll
    for (int seg = 0; seg < 2; ++seg) {
      const int d = seg + 1;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int r = tap / 3, s = tap % 3;
        f16x8_s wf[K::NT];
        filter_frags<K::NT, K::NB>(Wl, seg * 9 + tap, fr, fg, wswz, wf);
#pragma unroll
        for (int g = 0; g < K::GPW; ++g) {
          const int qc = (2 + (r - 1) * d) * (ST_TW + 4) + g * 16 + 2 + (s - 1) * d;
          const f16x8_s xf = *(const f16x8_s*)(sl + hbase + seg * 4 * RHh::PLANE + qc * 16);
#pragma unroll
          for (int nt = 0; nt < K::NT; ++nt)
            acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nt], xf, acc[nt][g], 0, 0, 0);
        }
      }
    }
    // x (1x1) and maxpool3(x) (1x1): slices 18, 19
    {
      f16x8_s w1[K::NT], w2[K::NT];
      filter_frags<K::NT, K::NB>(Wl, 18, fr, fg, wswz, w1);
      filter_frags<K::NT, K::NB>(Wl, 19, fr, fg, wswz, w2);
#pragma unroll
      for (int g = 0; g < K::GPW; ++g) {
        f16x8_s ctr = {}, mx = {};
#pragma unroll
        for (int dr = 0; dr < 3; ++dr)
#pragma unroll
          for (int ds = 0; ds < 3; ++ds) {
            const int qc = dr * (ST_TW + 2) + g * 16 + ds;
            const f16x8_s v = *(const f16x8_s*)(sl + xbase + qc * 16);
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
    if (has_next) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::G) : "memory");
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

static int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

template <typename KernelFn>
static int launch_persistent(KernelFn kern, int lds, StreamArgs& a, int th, const ConvOp& op, int& occ,
                             hipStream_t st) {
  if (!occ) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return (int)e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)kern, 256, lds);
    if (e != hipSuccess) return (int)e;
    if (occ < 1) occ = 1;
  }
  a.op = op;
  a.tiles_x = cdiv(op.Wo, ST_TW);
  a.tiles_y = cdiv(op.Ho, th);
  a.ntiles = op.B * a.tiles_x * a.tiles_y;
  int grid = std::min(device_cus() * occ, cdiv(a.ntiles, 8) * 8);
  grid = std::max(8, grid / 8 * 8);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, a);
  return (int)hipGetLastError();
}

template <int C, int NB, int TH, bool HEAD>
static int launch_stream_cfg(const ConvOp& op, hipStream_t st) {
  static int occ = 0;
  StreamArgs a;
  a.res_count = op.res2 ? 1 : 0;
  return launch_persistent(conv_stream_kernel<C, NB, TH, HEAD>, StreamCfg<C, NB, TH, HEAD>::LDS, a, TH, op, occ, st);
}

static int launch_stream_fam(const ConvOp& op, hipStream_t st) {
  static int occ = 0;
  StreamArgs a;
  a.res_count = 0;
  return launch_persistent(conv_stream_fam_kernel, FamCfg::LDS, a, FamCfg::TH, op, occ, st);
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

// fp16 only; kErrUnsupported for every op this kernel does not take
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
