// Row-ring streaming convolution for the HBM-bound fp16 layers: stride-1 3x3
// over 32 / 64 channels at the 512^2 / 256^2 / 128^2 levels (UpBlock convs,
// models/model.py:261-269; the residual head + illumination, :324-328 and
// :351-358; EnhancedFAM's fused branch3/branch4 first convs, :35-44) and the
// EnhancedFAM fusion GEMM over the virtual concat (:29-44, :66-78).
//
// Why not tiles: a tile kernel re-stages its halo for every tile (a 4 x 32 FAM
// tile with a 2-pixel halo DMAs 2.25x its output's input bytes) and can keep
// only one tile of loads in flight per LDS slot, which at the loaded HBM
// latency of ~2 us caps a CU near 16-20 GB/s (~4 TB/s chip-wide,
// profiles/r1_fp16_preact_aspp_pmc_conv_v11.txt: wait_any 0.49).
//
// * Work unit = one 32-pixel-wide column strip of one image over a band of
//   rows.  A persistent block (4 waves) walks its units top to bottom in
//   STEPS of 4 output rows (wave w computes row 4s + w: 2 x 16-pixel groups x
//   all output channels with v_mfma_f32_16x16x32_f16, weights = A, pixels = B).
// * The input rows live in a 16-row LDS RING per 16-byte channel chunk
//   ("chunk planes": plane c = chunk c of every ring pixel, row-major, so an
//   MFMA fragment of 16 consecutive pixels is 256 contiguous bytes and every
//   fragment address is a per-lane base + a wave-uniform row offset + an
//   immediate).  Each step DMAs (global_load_lds_dwordx4) only the 4 NEW rows
//   its successors need -- every input row is staged once per strip -- into
//   ring group (k+1) & 3, two steps ahead: the ring holds the 2 live groups
//   and 2 in flight, ~2 x 4 rows of loads per wave queue across each barrier.
// * One barrier per step.  Every wave issues the same number of memory
//   instructions every step (out-of-image pixels DMA from a zero / -inf line,
//   out-of-range outputs store to a sink, steps past the block's work DMA
//   fill), so the waits are constant `s_waitcnt vmcnt(N)`; the epilogue's
//   residual / input loads are inline asm (invisible to hipcc's counter
//   bookkeeping, waited for by hand) so the two DMAs in flight are never
//   drained.
// * Each unit starts with one DMA-only step (its first rows); units are
//   ordered strip-fastest and handed out XCD-contiguously, so neighbouring
//   strips (which share halo columns) run on one XCD's L2.
// * Filter fragments resident in registers for the block's lifetime where
//   they fit (FAM: 40 fragments = 160 VGPRs; halves the LDS reads per MFMA),
//   else in LDS (64-byte rows, chunk ^ ((n >> 2) & 1) * 2: conflict-free,
//   lane-constant swizzle).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "upr_common.h"

namespace upr {

typedef float f32x4_r __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8_r __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4_r __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_void_ptr_r;

// zero / -inf 16-byte chunks for out-of-image pixels (>= 8 chunks each); a
// write sink for out-of-range outputs (one 8-byte slot per thread)
__device__ __attribute__((aligned(256))) uint4 g_ring_zero[16];
__device__ __attribute__((aligned(256))) uint2 g_ring_sink[256];
__device__ __attribute__((aligned(256))) unsigned g_ring_ninf[64] = {
#define NINF4 0xFC00FC00u, 0xFC00FC00u, 0xFC00FC00u, 0xFC00FC00u
    NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4
#undef NINF4
};

constexpr int RG_TW = 32;  // strip width (output pixels)
constexpr int RG_RR = 16;  // ring rows

enum RingMode : int { kRingConv = 0, kRingHead = 1, kRingFam = 2 };

// A ring of NPL chunk planes over RG_RR rows of RG_TW + 2*HALO pixels.
template <int NPL, int HALO>
struct Ring {
  static constexpr int RW = RG_TW + 2 * HALO;   // ring row width (pixels)
  static constexpr int PLANE = RG_RR * RW * 16;  // bytes per chunk plane
  static constexpr int BYTES = NPL * PLANE;
  static constexpr int GPX = 4 * RW;             // pixels per 4-row group
  static constexpr int NI = (GPX + 63) / 64;     // DMA instructions per plane per step
  static constexpr int PPW = NPL / 4;            // planes per wave
  static constexpr int G = NI * PPW;             // DMA instructions per wave per step
  static_assert(NPL % 4 == 0, "planes are split over the 4 waves");
};

// Per-lane DMA geometry of one ring: for DMA instruction i the lane's group
// pixel (row dr, column col) and its element offset (dr * W + col) * cs from
// the group origin; dr = -1 for the idle lanes of the last, partial
// instruction of a plane (exec-masked: they write nothing).
template <class R>
struct RingLanes {
  int dr[R::NI], col[R::NI], off[R::NI];
  __device__ __forceinline__ void init(int lane, int W, int cs) {
#pragma unroll
    for (int i = 0; i < R::NI; ++i) {
      const int q = i * 64 + lane;
      dr[i] = q < R::GPX ? q / R::RW : -1;
      col[i] = q % R::RW;
      off[i] = (dr[i] * W + col[i]) * cs;
    }
  }
  // DMA of one 4-row group: group pixel (dr, col) <- image pixel
  // (iy0 + dr, ix0 + col) of image b (fill outside the image or when !live)
  __device__ __forceinline__ void issue(const half_t* src, int cs, int b, int H, int W, int iy0, int ix0, bool live,
                                        const half_t* fill, unsigned char* ring, int grp, int wave) const {
    const half_t* base = src + ((size_t)(b * H + iy0) * W + ix0) * cs;
#pragma unroll
    for (int i = 0; i < R::NI; ++i) {
      if (dr[i] >= 0) {
        const bool ok = live && (unsigned)(iy0 + dr[i]) < (unsigned)H && (unsigned)(ix0 + col[i]) < (unsigned)W;
        const half_t* p = ok ? base + off[i] : fill;
#pragma unroll
        for (int k = 0; k < R::PPW; ++k) {
          const int c = wave + 4 * k;
          __builtin_amdgcn_global_load_lds(p + c * 8, (lds_void_ptr_r)(ring + c * R::PLANE + grp * R::GPX * 16 + i * 1024),
                                           16, 0, 0);
        }
      }
    }
  }
};

__device__ __forceinline__ uint2 ring_load_b64(const void* p) {
  uint2 v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ unsigned ring_load_u16(const void* p) {
  unsigned v;
  asm volatile("global_load_ushort %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ unsigned ring_load_b32(const void* p) {
  unsigned v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// filter [nslices x 32 k][NB] -> LDS [slice][n][64 B], chunk ^ ((n >> 2) & 1) * 2
template <int NB>
__device__ __forceinline__ void ring_load_filter(unsigned char* Wl, const half_t* Wg, int kpad, int nslices, int tid) {
  for (int i = tid; i < nslices * NB * 4; i += 256) {
    const int pc = i & 3, n = (i >> 2) % NB, sl = (i >> 2) / NB;
    const int c = pc ^ (((n >> 2) & 1) << 1);
    *(uint4*)(Wl + (size_t)i * 16) = *(const uint4*)(Wg + (size_t)n * kpad + sl * 32 + c * 8);
  }
}

template <int NT, int NB>
__device__ __forceinline__ void ring_filter_frags(const unsigned char* Wl, int sl, int fr, int fg, int wswz,
                                                  f16x8_r (&wf)[NT]) {
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    wf[nt] = *(const f16x8_r*)(Wl + ((size_t)(sl * NB + nt * 16 + fr) * 64) + ((fg ^ wswz) * 16));
}

struct RingArgs {
  ConvOp op;
  int nstrips, nseg, rs;  // strips per image row, row bands per image, rows per band (multiple of 4)
  int nunits, steps;      // units; steps per unit = rs / 4 + 1 (first = DMA only)
};

template <int MODE, int C, int NB, bool RES>
struct RingCfg {
  static constexpr bool FAM = MODE == kRingFam, HEAD = MODE == kRingHead;
  using RA = Ring<FAM ? 8 : C / 8, FAM ? 2 : 1>;  // main input ([h3 | h4] for FAM)
  using RB = Ring<4, 1>;                          // FAM: x (32 channels, -inf outside)
  static constexpr int NSL = FAM ? 20 : 9 * (C / 32);
  // filter fragments held in registers for the block's lifetime when they fit
  // (<= 160 VGPRs: FAM, C 32 -> N 32 / 64), else resident in LDS
  static constexpr bool WREG = NSL * (NB / 16) <= 40;
  static constexpr int WBYTES = WREG ? 0 : NSL * NB * 64;
  static constexpr int LDS = WBYTES + RA::BYTES + (FAM ? RB::BYTES : 0);
  static constexpr int NT = NB / 16;
  static constexpr int KS = C / 32;
  static constexpr int G = RA::G + (FAM ? RB::G : 0);       // DMA per wave per step
  static constexpr int S = HEAD ? 2 : 2 * NT;               // stores per wave per step
  static constexpr int R = HEAD ? 6 : (RES ? 2 * NT : 0);   // epilogue loads per wave per step
  static constexpr int W0 = G;                              // wait at step 0
  static constexpr int W1 = R + G + S;                      // step 1
  static constexpr int WK = 2 * S + R + G;                  // steps >= 2
  static constexpr int WF = WK + (FAM ? 4 * NT : 0);        // after a FAM pool flush (its atomics)
  static_assert(WF <= 63, "vmcnt immediate");
};

template <int MODE, int C, int NB, bool RES>
__global__ __launch_bounds__(256) void conv_ring_kernel(RingArgs a) {
  using K = RingCfg<MODE, C, NB, RES>;
  using RA = typename K::RA;
  using RB = typename K::RB;
  constexpr bool FAM = K::FAM, HEAD = K::HEAD;
  constexpr int HA = FAM ? 2 : 1;
  const ConvOp& op = a.op;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* Wl = smem;
  unsigned char* ringA = smem + K::WBYTES;
  unsigned char* ringB = ringA + RA::BYTES;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR) row index
  const int fr = lane & 15, fg = lane >> 4;
  const int wswz = ((fr >> 2) & 1) << 1;
  const int H = op.Ho, W = op.Wo;
  // XCD-contiguous unit order: block -> v (units v, v + grid, ...)
  const int per_xcd = gridDim.x >> 3;
  const int v0 = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  const int nu = v0 < a.nunits ? (a.nunits - 1 - v0) / (int)gridDim.x + 1 : 0;
  const int KT = nu * a.steps;  // steps of this block

  f16x8_r wr[K::WREG ? K::NSL : 1][K::NT];
  if constexpr (K::WREG) {
    // lane (fr, fg) of fragment (slice, nt): W[nt*16 + fr][slice*32 + fg*8 .. +7]
#pragma unroll
    for (int sl = 0; sl < K::NSL; ++sl)
#pragma unroll
      for (int nt = 0; nt < K::NT; ++nt)
        wr[sl][nt] = *(const f16x8_r*)((const half_t*)op.W + (size_t)(nt * 16 + fr) * op.Kpad + sl * 32 + fg * 8);
  } else {
    ring_load_filter<NB>(Wl, (const half_t*)op.W, op.Kpad, K::NSL, tid);
  }
  auto frags = [&](int sl, f16x8_r (&wf)[K::NT]) {
    if constexpr (K::WREG) {
#pragma unroll
      for (int nt = 0; nt < K::NT; ++nt) wf[nt] = wr[sl][nt];
    } else {
      ring_filter_frags<K::NT, NB>(Wl, sl, fr, fg, wswz, wf);
    }
  };
  const ConvSeg& sa = op.seg[0];
  const half_t* srcA = (const half_t*)sa.src + sa.coff;
  const half_t* srcB = FAM ? (const half_t*)op.seg[2].src + op.seg[2].coff : nullptr;
  const int csA = sa.cs, csB = FAM ? op.seg[2].cs : 0;
  const half_t* zero = (const half_t*)g_ring_zero;
  const half_t* ninf = (const half_t*)g_ring_ninf;
  RingLanes<RA> la;
  RingLanes<RB> lb;
  la.init(lane, W, csA);
  if constexpr (FAM) lb.init(lane, W, csB);

  // unit j of this block -> (image b, first row y0, strip origin x0)
  auto unit_of = [&](int j, int& b, int& y0, int& x0) {
    const int u = v0 + j * (int)gridDim.x;
    const int sx = u % a.nstrips, r = u / a.nstrips;
    b = r / a.nseg;
    y0 = (r % a.nseg) * a.rs;
    x0 = sx * RG_TW;
  };
  // step cursors (wave-uniform): the compute cursor is at step kk, the DMA
  // cursor two steps ahead; the integer divisions run once per unit
  const int S = a.steps - 1;  // compute steps per unit (s = -1 is DMA only)
  struct Cursor {
    int j, s, b, y0, x0;
  };
  Cursor cc{0, -1, 0, 0, 0};
  if (nu > 0) unit_of(0, cc.b, cc.y0, cc.x0);
  Cursor dc = cc;
  auto advance = [&](Cursor& c) {
    if (++c.s == S) {
      c.s = -1;
      if (++c.j < nu) unit_of(c.j, c.b, c.y0, c.x0);
    }
  };
  // DMA of the 4 rows step dc.s of its unit first needs, into ring group (k+1) & 3
  auto issue = [&](int k) {
    const bool live = dc.j < nu;
    const int grp = (k + 1) & 3;
    la.issue(srcA, csA, dc.b, H, W, dc.y0 + 4 * dc.s + HA, dc.x0 - HA, live, zero, ringA, grp, wave);
    if constexpr (FAM) lb.issue(srcB, csB, dc.b, H, W, dc.y0 + 4 * dc.s + 1, dc.x0 - 1, live, ninf, ringB, grp, wave);
    advance(dc);
  };

  __syncthreads();  // filter in LDS (ordinary loads, waited for by hipcc)
  issue(0);
  issue(1);

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
  const int abase = fg * RA::PLANE + fr * 16;  // chunk plane fg, pixel fr of a ring row
  const int bbase = fg * RB::PLANE + fr * 16;
  // lane parts of the epilogue addresses (pixel g*16 + fr of the row, channels fg*4..)
  const int ocs = op.out_cs, rcs = RES ? op.res2_cs : 0;
  int oloff[2], rloff[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    oloff[g] = (g * 16 + fr) * ocs + fg * 4;
    rloff[g] = (g * 16 + fr) * rcs + fg * 4;
  }
  const size_t HWs = (size_t)H * W;

  float pool[K::NT][4];
#pragma unroll
  for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) pool[nt][i] = 0.f;
  bool flushed = false;

  for (int kk = 0; kk < KT; ++kk) {
    // (A) DMA(kk) has landed (younger: stores(kk-2), loads(kk-1), DMA(kk+1), stores(kk-1))
    // (+ the previous step's pool atomics when it ended a FAM unit)
    if (kk == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::W0) : "memory");
    else if (kk == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::W1) : "memory");
    else if (flushed) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::WF) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::WK) : "memory");
    __builtin_amdgcn_s_barrier();
    flushed = false;
    const int s = cc.s, b = cc.b, x0 = cc.x0;
    const int yend = min(H, cc.y0 + a.rs);
    const int y = cc.y0 + 4 * s + wave;
    const bool rowok = s >= 0 && y < yend;
    const size_t prow = (size_t)(b * H + (rowok ? y : 0)) * W + x0;  // first pixel of this wave's output row

    // epilogue inputs of this step (asm loads, before the next DMA)
    uint2 res[2][K::NT];
    unsigned xin[2][3];
    bool ovalid[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      ovalid[g] = rowok && x0 + g * 16 + fr < W;
      if constexpr (RES) {
        const half_t* rp = (const half_t*)op.res2 + prow * rcs + rloff[g];
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt)
          res[g][nt] = ring_load_b64(ovalid[g] ? (const void*)(rp + nt * 16) : (const void*)zero);
      }
      if constexpr (HEAD) {
        const size_t pb = (size_t)b * 2 * HWs + prow + g * 16 + fr;  // (b*3 + c)*HW + y*W + x
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          if (op.x_f16) xin[g][c] = ring_load_u16(ovalid[g] ? (const void*)((const half_t*)op.x_nchw + pb + c * HWs) : (const void*)zero);
          else xin[g][c] = ring_load_b32(ovalid[g] ? (const void*)(op.x_nchw + pb + c * HWs) : (const void*)zero);
        }
      }
    }
    issue(kk + 2);

    // ---- MFMAs: D[n][px] = sum_k W[n][k] * X[px][k] ---------------------------
    f32x4_r acc[K::NT][2];
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
      for (int g = 0; g < 2; ++g) acc[nt][g] = f32x4_r{0.f, 0.f, 0.f, 0.f};
    // LDS pipeline per "chunk" (one ring row's fragments): [reads of chunk c+1]
    // [MFMAs of chunk c] [lgkmcnt(0)].  The wait is a real s_waitcnt
    // (__builtin_amdgcn_s_waitcnt, which hipcc's counter pass sees) placed
    // after the MFMAs that covered the reads' latency; sched_barrier(0) fences
    // keep hipcc from hoisting the next reads above it (it would then wait for
    // those too: its own waits are always lgkmcnt(0) here).
#define RING_FENCE __builtin_amdgcn_sched_barrier(0)
#define RING_LDS_DONE                                                               \
  do {                                                                              \
    RING_FENCE;                                                                     \
    __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0); vmcnt / expcnt untouched */ \
    RING_FENCE;                                                                     \
  } while (0)
    if (s >= 0) {
      // ring row of input row y + dy: (4kk + 4 + wave - HALO + dy) & 15
      auto rowA = [&](int dy) { return ((4 * kk + 4 + wave - HA + dy) & 15) * (RA::RW * 16); };
      if constexpr (!FAM) {
        // chunk c = (tap row r, 32-channel slice ks): 3 taps x 2 pixel groups of
        // X fragments (+ the 3 x NT filter fragments when the filter is in LDS);
        // the same [reads c+1] [MFMAs c] [lgkmcnt(0)] pipeline as the FAM path
        constexpr int NCH = 3 * K::KS;
        constexpr int NW = K::WREG ? 1 : 3;
        f16x8_r bx[2][6], bw[2][NW][K::NT];
        auto ld = [&](int c, f16x8_r (&x)[6], f16x8_r (&w)[NW][K::NT]) {
          const int r = c / K::KS, ks = c % K::KS;
          const unsigned char* xr = ringA + abase + rowA(r - 1) + ks * 4 * RA::PLANE;
#pragma unroll
          for (int sc = 0; sc < 3; ++sc)
#pragma unroll
            for (int g = 0; g < 2; ++g) x[sc * 2 + g] = *(const f16x8_r*)(xr + (g * 16 + sc) * 16);
          if constexpr (!K::WREG) {
#pragma unroll
            for (int sc = 0; sc < 3; ++sc) ring_filter_frags<K::NT, NB>(Wl, (r * 3 + sc) * K::KS + ks, fr, fg, wswz, w[sc]);
          }
        };
        auto mm = [&](int c, const f16x8_r (&x)[6], const f16x8_r (&w)[NW][K::NT]) {
          const int r = c / K::KS, ks = c % K::KS;
#pragma unroll
          for (int sc = 0; sc < 3; ++sc)
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
              for (int nt = 0; nt < K::NT; ++nt) {
                f16x8_r wf;
                if constexpr (K::WREG) wf = wr[(r * 3 + sc) * K::KS + ks][nt];
                else wf = w[sc][nt];
                acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf, x[sc * 2 + g], acc[nt][g], 0, 0, 0);
              }
        };
        ld(0, bx[0], bw[0]);
        ld(1, bx[1], bw[1]);
        RING_LDS_DONE;
        mm(0, bx[0], bw[0]);
#pragma unroll
        for (int c = 1; c < NCH; ++c) {
          RING_FENCE;
          if (c + 1 < NCH) ld(c + 1, bx[(c + 1) & 1], bw[(c + 1) & 1]);
          RING_FENCE;
          mm(c, bx[c & 1], bw[c & 1]);
          RING_LDS_DONE;
        }
      } else {
        // h3 (3x3, d1): slices 0..8, planes 0-3; h4 (3x3, d2): slices 9..17, planes 4-7;
        // then x (1x1, slice 18) and maxpool3(x) (1x1, slice 19) from the x ring.
        // Software-pipelined by ring row ("chunk": 3 taps x 2 pixel groups = 6
        // fragments): the reads of chunk c+1 are issued before the MFMAs of
        // chunk c, so one wave per SIMD still keeps the LDS latency covered.
        static_assert(K::WREG, "FAM keeps its filter in registers");
        auto rowB = [&](int dy) { return ((4 * kk + 4 + wave - 1 + dy) & 15) * (RB::RW * 16); };
        auto ld_h = [&](int c, f16x8_r (&buf)[6]) {
          const int seg = c / 3, r = c % 3, d = seg + 1;
          const unsigned char* xr = ringA + abase + seg * 4 * RA::PLANE + rowA((r - 1) * d);
#pragma unroll
          for (int sc = 0; sc < 3; ++sc)
#pragma unroll
            for (int g = 0; g < 2; ++g) buf[sc * 2 + g] = *(const f16x8_r*)(xr + (g * 16 + 2 + (sc - 1) * d) * 16);
        };
        auto ld_x = [&](int dr, f16x8_r (&buf)[6]) {
          const unsigned char* xr = ringB + bbase + rowB(dr - 1);
#pragma unroll
          for (int ds = 0; ds < 3; ++ds)
#pragma unroll
            for (int g = 0; g < 2; ++g) buf[ds * 2 + g] = *(const f16x8_r*)(xr + (g * 16 + ds) * 16);
        };
        auto mm_h = [&](int c, const f16x8_r (&buf)[6]) {
          const int seg = c / 3, r = c % 3;
#pragma unroll
          for (int sc = 0; sc < 3; ++sc)
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
              for (int nt = 0; nt < K::NT; ++nt)
                acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[seg * 9 + r * 3 + sc][nt], buf[sc * 2 + g],
                                                                    acc[nt][g], 0, 0, 0);
        };
        f16x8_r ctr[2], mx[2];
        auto mp = [&](int dr, const f16x8_r (&buf)[6]) {
#pragma unroll
          for (int ds = 0; ds < 3; ++ds)
#pragma unroll
            for (int g = 0; g < 2; ++g) {
              const f16x8_r v = buf[ds * 2 + g];
              if (dr == 0 && ds == 0) mx[g] = v;
              else mx[g] = __builtin_elementwise_max(mx[g], v);
              if (dr == 1 && ds == 1) ctr[g] = v;
            }
        };
        f16x8_r b0[6], b1[6];
        ld_h(0, b0);
        ld_h(1, b1);
        RING_LDS_DONE;
        mm_h(0, b0);
        RING_FENCE;
        ld_h(2, b0);
        RING_FENCE;
        mm_h(1, b1);
        RING_LDS_DONE;
        ld_h(3, b1);
        RING_FENCE;
        mm_h(2, b0);
        RING_LDS_DONE;
        ld_h(4, b0);
        RING_FENCE;
        mm_h(3, b1);
        RING_LDS_DONE;
        ld_h(5, b1);
        RING_FENCE;
        mm_h(4, b0);
        RING_LDS_DONE;
        ld_x(0, b0);
        RING_FENCE;
        mm_h(5, b1);
        RING_LDS_DONE;
        ld_x(1, b1);
        RING_FENCE;
        mp(0, b0);
        RING_LDS_DONE;
        ld_x(2, b0);
        RING_FENCE;
        mp(1, b1);
        RING_LDS_DONE;
        mp(2, b0);
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
          for (int nt = 0; nt < K::NT; ++nt) {
            acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[18][nt], ctr[g], acc[nt][g], 0, 0, 0);
            acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[19][nt], mx[g], acc[nt][g], 0, 0, 0);
          }
      }
    }

#undef RING_LDS_DONE
#undef RING_FENCE
    // (B) this step's asm loads are done; DMA(kk+2) may fly on
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::G) : "memory");
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if constexpr (RES) {
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt) asm volatile("" : "+v"(res[g][nt].x), "+v"(res[g][nt].y));
      }
      if constexpr (HEAD) asm volatile("" : "+v"(xin[g][0]), "+v"(xin[g][1]), "+v"(xin[g][2]));
    }

    // ---- epilogue ---------------------------------------------------------------
    if constexpr (HEAD) {
      // r = sum_n relu(v_n) * w2_n ; illu = sigmoid(mean_c(x) + r + b2)
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        float part = 0.f;
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) part += fmaxf(acc[nt][g][i] + bv[nt][i], 0.f) * hw2[nt][i];
        part += __shfl_xor(part, 16);
        part += __shfl_xor(part, 32);
        float x0f, x1f, x2f;
        if (op.x_f16) {
          x0f = (float)__builtin_bit_cast(half_t, (unsigned short)(xin[g][0] & 0xffff));
          x1f = (float)__builtin_bit_cast(half_t, (unsigned short)(xin[g][1] & 0xffff));
          x2f = (float)__builtin_bit_cast(half_t, (unsigned short)(xin[g][2] & 0xffff));
        } else {
          x0f = __builtin_bit_cast(float, xin[g][0]);
          x1f = __builtin_bit_cast(float, xin[g][1]);
          x2f = __builtin_bit_cast(float, xin[g][2]);
        }
        const float z = (x0f + x1f + x2f) / 3.f + (part + op.head_b);
        const float il = 1.f / (1.f + expf(-z));
        float* dst = (ovalid[g] && fg == 0) ? op.illu + prow + g * 16 + fr : (float*)(g_ring_sink + tid);
        *dst = il;
      }
    } else {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = acc[nt][g][i] + bv[nt][i];
            if (FAM || op.relu) v[i] = fmaxf(v[i], 0.f);
          }
          if constexpr (RES) {
            const f16x4_r rr = __builtin_bit_cast(f16x4_r, res[g][nt]);
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] += (float)rr[i];
          }
          f16x4_r o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = (half_t)v[i];
          if constexpr (FAM) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (ovalid[g]) pool[nt][i] += (float)o[i];
          }
          uint2* dst = ovalid[g] ? (uint2*)((half_t*)op.out + prow * ocs + op.out_coff + oloff[g] + nt * 16)
                                 : g_ring_sink + tid;
          *dst = __builtin_bit_cast(uint2, o);
        }
      }
    }
    // FAM: per-image channel sums, flushed at the end of every unit (a unit is one image)
    if constexpr (FAM) {
      if (op.pool && s == a.steps - 2) {
#pragma unroll
        for (int nt = 0; nt < K::NT; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v = pool[nt][i];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if (fr == 0) atomicAdd(op.pool + (size_t)b * op.N + nt * 16 + fg * 4 + i, v);
            pool[nt][i] = 0.f;
          }
        flushed = true;
      }
    }
    advance(cc);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

static int ring_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

template <int MODE, int C, int NB, bool RES>
static int launch_ring_cfg(const ConvOp& op, hipStream_t st) {
  using K = RingCfg<MODE, C, NB, RES>;
  auto kern = conv_ring_kernel<MODE, C, NB, RES>;
  static int occ = 0;
  if (!occ) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS);
    if (e != hipSuccess) return (int)e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)kern, 256, K::LDS);
    if (e != hipSuccess) return (int)e;
    if (occ < 1) occ = 1;
  }
  RingArgs a;
  a.op = op;
  a.nstrips = cdiv(op.Wo, RG_TW);
  const int grid = ring_cus() * occ;  // a multiple of 8 (XCD-contiguous unit order)
  const int per_band = op.B * a.nstrips;
  // row bands: minimise the makespan ceil(units / grid) * steps per unit
  long best = -1;
  for (int nb = 1; nb <= 16; ++nb) {
    int rs = (cdiv(op.Ho, nb) + 3) / 4 * 4;
    if (rs < 8) rs = 8;
    const int nseg = cdiv(op.Ho, rs);
    const long cost = (long)cdiv(per_band * nseg, grid) * (rs / 4 + 1);
    if (best < 0 || cost < best) {
      best = cost;
      a.rs = rs;
      a.nseg = nseg;
    }
  }
  a.nunits = per_band * a.nseg;
  a.steps = a.rs / 4 + 1;
  int g = std::min(grid, cdiv(a.nunits, 8) * 8);
  g = std::max(8, g / 8 * 8);
  hipLaunchKernelGGL(kern, dim3(g), dim3(256), K::LDS, st, a);
  return (int)hipGetLastError();
}

// UPR_CONV_RING=0 disables this path (A/B timing against conv_stream)
static bool ring_enabled() {
  static int en = -1;
  if (en < 0) {
    const char* e = getenv("UPR_CONV_RING");
    en = (e && strcmp(e, "0") == 0) ? 0 : 1;
  }
  return en == 1;
}

static bool ring_fam_program(const ConvOp& op) {
  if (op.nseg != 4 || op.N != 32 || op.store != kStoreNHWC || op.res1 || op.res2 || op.img_bias || op.scale) return false;
  if (op.Kpad != 640 || op.out_cs % 4 || op.out_coff % 4) return false;
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
int launch_conv_ring(const ConvOp& op, hipStream_t st) {
  if (!ring_enabled()) return kErrUnsupported;
  if (op.Ho < 4 || op.Wo < 16) return kErrUnsupported;
  if (ring_fam_program(op)) return launch_ring_cfg<kRingFam, 32, 32, false>(op, st);
  if (op.nseg != 1) return kErrUnsupported;
  const ConvSeg& s = op.seg[0];
  if (s.kh != 3 || s.kw != 3 || s.stride != 1 || s.dil != 1 || s.pad != 1 || s.pre != kPreNone) return kErrUnsupported;
  if (s.Hin != op.Ho || s.Win != op.Wo) return kErrUnsupported;
  if ((s.C != 32 && s.C != 64) || s.cs % 8 || s.coff % 8 || (uintptr_t)s.src % 16) return kErrUnsupported;
  if (op.res1 || op.img_bias || op.pool || op.scale || op.Kpad % 8 || s.kbase != 0) return kErrUnsupported;
  if (op.store == kStoreHeadIllu) {
    if (op.N != 32 || s.C != 32 || op.res2 || op.illu_f16) return kErrUnsupported;
    return launch_ring_cfg<kRingHead, 32, 32, false>(op, st);
  }
  if (op.store != kStoreNHWC || op.out_cs % 4 || op.out_coff % 4) return kErrUnsupported;
  if (op.res2 && op.res2_cs % 4) return kErrUnsupported;
  const bool res = op.res2 != nullptr;
  if (s.C == 32 && op.N == 32) return res ? launch_ring_cfg<kRingConv, 32, 32, true>(op, st)
                                          : launch_ring_cfg<kRingConv, 32, 32, false>(op, st);
  if (s.C == 32 && op.N == 64) return res ? launch_ring_cfg<kRingConv, 32, 64, true>(op, st)
                                          : launch_ring_cfg<kRingConv, 32, 64, false>(op, st);
  if (s.C == 64 && op.N == 64) return res ? launch_ring_cfg<kRingConv, 64, 64, true>(op, st)
                                          : launch_ring_cfg<kRingConv, 64, 64, false>(op, st);
  return kErrUnsupported;
}

}  // namespace upr
