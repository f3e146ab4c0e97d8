// Row-ring streaming convolution for the HBM-bound fp16 layers at the 512^2 /
// 256^2 / 128^2 levels:
//   * stride-1 3x3 over 32 / 64 channels: UpBlock convs (models/model.py:261-269),
//     the residual head + illumination (:324-328, :351-358), EnhancedFAM's fused
//     branch3/branch4 first convs (:35-44), enc1.conv2 with its projecting
//     shortcut (conv1x1 s2 + BN of ResBlock / PreActResBlock, :100-178) as a
//     register-fed second K segment;
//   * stride-2 3x3, 32 -> 64 channels: enc1.conv1 (:100-178);
//   * the EnhancedFAM fusion GEMM over the virtual concat (:29-44, :66-78).
//
// Why not tiles: a tile kernel re-stages its halo for every tile (a 4 x 32 FAM
// tile with a 2-pixel halo DMAs 2.25x its output's input bytes) and keeps one
// tile of loads in flight per LDS slot.
//
// * Work unit = one column strip (32 output pixels; 16 for stride 2) of one
//   image over a band of rows.  A persistent block (4 waves) walks its units
//   top to bottom in STEPS of 4 output rows (wave w computes row 4s + w: all
//   output channels of the strip's 16-pixel groups, v_mfma_f32_16x16x32_f16,
//   weights = A, pixels = B).
// * The input rows live in an LDS RING per 16-byte channel chunk ("chunk
//   planes": plane c = chunk c of every ring pixel, row-major, so an MFMA
//   fragment of 16 consecutive pixels is 256 contiguous bytes and every
//   fragment address is a per-lane base + a wave-uniform row offset + an
//   immediate).  Each step DMAs (global_load_lds_dwordx4) only the rows its
//   successors first need -- every input row is staged once per strip -- into
//   ring group (k+1) & 3, two steps ahead: the ring holds 2 live groups and 2
//   in flight.  Stride 2 stores each ring row de-interleaved (even source
//   columns, then odd), so the three taps of a row are three contiguous
//   16-pixel runs.
// * One barrier per step.  Every wave issues the same number of memory
//   instructions every step (out-of-image pixels DMA from a zero / -inf line,
//   out-of-range outputs store to a sink, steps past the block's work DMA
//   fill), so the waits are constant `s_waitcnt vmcnt(N)`.  The epilogue's
//   inputs (residual, shortcut source pixels, network input) are LDS-DMA'd
//   too, into a per-wave landing zone at the top of the step: the two input
//   DMAs in flight are never drained, and no register is in flight behind
//   hipcc's back.
// * LDS fragment reads are software-pipelined by ring row ("chunk"): [reads of
//   chunk c+1] [MFMAs of chunk c] [lgkmcnt(0)], fenced with sched_barrier.
// * Each unit starts with one DMA-only step; units are ordered strip-fastest
//   and handed out XCD-contiguously (neighbouring strips share halo columns in
//   one XCD's L2); step cursors are advanced incrementally (the integer
//   divisions run once per unit).
// * Filter fragments resident in registers for the block's lifetime where
//   they fit (<= 40 fragments), else in LDS (64-byte rows, chunk ^ ((n >> 2) &
//   1) * 2: conflict-free, lane-constant swizzle).  The bias is the
//   accumulators' initial value.
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
// write sink for out-of-range outputs (128 bytes per thread, <= 512 threads)
__device__ __attribute__((aligned(256))) uint4 g_ring_zero[16];
__device__ __attribute__((aligned(256))) uint2 g_ring_sink[512 * 16];
__device__ __attribute__((aligned(256))) float g_ring_sink32[512 * 64];  // fp32 outputs: 256 bytes per thread
__device__ __attribute__((aligned(256))) unsigned g_ring_ninf32[64] = {  // fp32 -inf line (16 chunks)
#define NINF4 0xFF800000u, 0xFF800000u, 0xFF800000u, 0xFF800000u
    NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4
#undef NINF4
};
__device__ __attribute__((aligned(256))) unsigned g_ring_ninf[64] = {
#define NINF4 0xFC00FC00u, 0xFC00FC00u, 0xFC00FC00u, 0xFC00FC00u
    NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4, NINF4
#undef NINF4
};

enum RingMode : int { kRingConv = 0, kRingHead = 1, kRingFam = 2, kRingS2 = 3 };
// kRingOcc3: 4-wave blocks compiled for 3 waves per SIMD (<= 168 VGPRs, three
// blocks per CU); only the configs that fit without spilling (no residual / head)
// kRingWide: 64-pixel strips (4 pixel groups per wave row): twice the MFMAs per
// step for the same per-step barrier / DMA / cursor work (32 -> 32 convs)
// kRingOut2: the epilogue also writes relu(fma(o, pre2_scale, pre2_shift)) (ConvOp::out2)
// kRingOut32: fp32 output (ConvOp::out32) instead of the fp16 store; kRingR32:
// + ConvOp::res32 (an accumulated fp32 input gradient) in that epilogue
// fp32 ring only: kRingDil2 = the segment is a 3x3 dilation-2 conv (2-pixel halo ring);
// kRingResPre = the residual is ConvOp::res1 (added before the ReLU) instead of
// res2 (after it); kRingPool = per-image channel sums of the output into ConvOp::pool
enum RingFlags : int {
  kRingRes = 1, kRingRelu = 2, kRingSc = 4, kRingOcc3 = 8, kRingWide = 16, kRingOut2 = 32, kRingOut32 = 64,
  kRingDil2 = 128, kRingResPre = 256, kRingPool = 512, kRingXPool = 1024, kRingR32 = 2048,
  // timing ablations only (results garbage; UPR_RING_ABL, tools/convbench.py):
  // no ring DMA after the first two steps / no MFMAs / no output stores
  kRingAblDma = 4096, kRingAblMma = 8192, kRingAblSt = 16384
};
// kRingXPool (fp32 ring): two more K slices after the 3x3 segment, a 1x1 over
// x and a 1x1 over maxpool3x3(x) (EnhancedFAM branch1 / branch2 composed with
// the fusion), x staged in a second ring with a -inf halo

// A ring of NPL chunk planes: 4 groups of GROWS rows of RW pixels.  DEINT:
// ring column p holds source column 2p (p < (RW+1)/2) or 2(p - (RW+1)/2) + 1.
template <int NPL, int RW_, int GROWS_, bool DEINT_ = false>
struct Ring {
  static constexpr int RW = RW_;
  static constexpr int GROWS = GROWS_;
  static constexpr int RR = 4 * GROWS;           // ring rows (power of two)
  static constexpr int PLANE = RR * RW * 16;     // bytes per chunk plane
  static constexpr int BYTES = NPL * PLANE;
  static constexpr int GPX = GROWS * RW;         // pixels per group
  static constexpr int NI = (GPX + 63) / 64;     // DMA instructions per plane per step
  static constexpr int PPW = NPL / 4;            // planes per wave
  static constexpr int G = NI * PPW;             // DMA instructions per wave per step
  static constexpr bool DEINT = DEINT_;
  static constexpr int HALF = (RW + 1) / 2;
  static_assert(NPL % 4 == 0, "planes are split over the 4 waves");
  static_assert((RR & (RR - 1)) == 0, "ring rows: power of two");
};

// Per-lane DMA geometry of one ring: for DMA instruction i the lane's group
// pixel (row dr, source column col) and its element offset (dr * W + col) * cs
// from the group origin; dr = -1 for the idle lanes of the last, partial
// instruction of a plane (exec-masked: they write nothing).
template <class R>
struct RingLanes {
  int dr[R::NI], col[R::NI], off[R::NI];
  __device__ __forceinline__ void init(int lane, int W, int cs) {
#pragma unroll
    for (int i = 0; i < R::NI; ++i) {
      const int q = i * 64 + lane;
      const int p = q % R::RW;
      dr[i] = q < R::GPX ? q / R::RW : -1;
      col[i] = R::DEINT ? (p < R::HALF ? 2 * p : 2 * (p - R::HALF) + 1) : p;
      off[i] = (dr[i] * W + col[i]) * cs;
    }
  }
  // DMA of one group: group pixel (dr, col) <- image pixel (iy0 + dr, ix0 +
  // col) of image b (fill outside the image or when !live)
  __device__ __forceinline__ void issue(const half_t* src, int cs, int b, int H, int W, int iy0, int ix0, bool live,
                                        const half_t* fill, unsigned char* ring, int grp, int wave) const {
    const half_t* base = src + ((long long)(b * H + iy0) * W + ix0) * cs;
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

// Output-channel order of the fp16 ring's MFMA rows: fragment nt, row r holds
// channel 32 (nt >> 1) + 8 (r >> 2) + 4 (nt & 1) + (r & 3), so a lane's
// accumulators of fragments 2p and 2p + 1 are 8 CONSECUTIVE channels (32p +
// 8 fg .. + 7) and the epilogue stores 16 bytes per lane (8-byte stores of 4
// channels moved the 32/64-channel outputs at ~3 TB/s: every store
// instruction wrote half-lines of 16 pixels).  The filter rows and every
// per-channel parameter are read in this order.
__device__ __forceinline__ int ring_ch(int nt, int r) { return 32 * (nt >> 1) + 8 * (r >> 2) + 4 * (nt & 1) + (r & 3); }
// PAIR = false (the FAM fusion and the fp32-output programs: their registers
// are full, and the fp32 stores are 16 bytes either way) keeps the plain order
template <bool PAIR>
__device__ __forceinline__ int ring_chm(int nt, int r) {
  if constexpr (PAIR) return ring_ch(nt, r);
  else return nt * 16 + r;
}

// filter [nslices x 32 k][NB] -> LDS [slice][n][64 B], chunk ^ ((n >> 2) & 1) * 2
// (LDS row n holds filter row ring_ch(n >> 4, n & 15))
template <int NB, int THREADS, bool PAIR = true>
__device__ __forceinline__ void ring_load_filter(unsigned char* Wl, const half_t* Wg, int kpad, int nslices, int tid) {
  for (int i = tid; i < nslices * NB * 4; i += THREADS) {
    const int pc = i & 3, n = (i >> 2) % NB, sl = (i >> 2) / NB;
    const int c = pc ^ (((n >> 2) & 1) << 1);
    *(uint4*)(Wl + (size_t)i * 16) = *(const uint4*)(Wg + (size_t)ring_chm<PAIR>(n >> 4, n & 15) * kpad + sl * 32 + c * 8);
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

// chunk permutation of landing pixel l (CPP 16-byte chunks per pixel) for
// conflict-free epilogue reads: 8-byte reads (fp16, CPP 4/8) spread 16 pixels
// over the 256-byte bank row; 16-byte reads (fp32, CPP 8/16) over its 16 slots
template <int CPP>
__device__ __forceinline__ int ring_res_swz(int l) {
  if constexpr (CPP == 16) return l & 15;
  else return ((l * CPP) >> 4) & (CPP - 1);
}

template <int MODE, int C, int NB, int FL>
struct RingCfg {
  static constexpr bool FAM = MODE == kRingFam, HEAD = MODE == kRingHead, S2 = MODE == kRingS2;
  static constexpr bool RES = FL & kRingRes, RELU = FAM || (FL & kRingRelu), SC = FL & kRingSc;
  static constexpr int HA = FAM ? 2 : 1;           // main ring halo (stride 1)
  static constexpr int TW = S2 ? 16 : (FL & kRingWide) ? 64 : 32;  // strip width (output pixels)
  static constexpr int NG = TW / 16;               // 16-pixel groups per output row
  using RA = Ring<FAM ? 8 : C / 8, S2 ? 2 * TW + 1 : TW + 2 * HA, S2 ? 8 : 4, S2>;
  using RB = Ring<4, TW + 2, 4>;                   // FAM: x (32 channels, -inf outside)
  static constexpr int NSL = FAM ? 20 : 9 * (C / 32);  // k slices of the ring segment(s)
  static constexpr int NT = NB / 16;
  static constexpr int KS = C / 32;
  // filter fragments in registers for the block's lifetime when they fit
  static constexpr bool WREG = NSL * NT <= 40;
  static constexpr int WBYTES = WREG ? 0 : NSL * NB * 64;
  // 8 waves when a row has two 16-pixel groups (wave w: row w & 3, group
  // w >> 2; two waves per SIMD to hide each other's MFMA / LDS latency), else 4
  // (measured: FAM fusion 0.61 -> 0.44 ms at 512^2 bs 32); the 32 -> 32 convs
  // keep 4-wave blocks, two to three per CU (an 8-wave block of them is slower)
  static constexpr int NWV = NG == 2 && !(C == 32 && NB == 32 && !FAM) ? 8 : 4;
  static constexpr int THREADS = NWV * 64;
  // waves per SIMD the register budget is sized for (one 8-wave block per CU)
  static constexpr int MINW = NWV == 8 || (FL & kRingWide) ? 2 : (FL & kRingOcc3) ? 3 : 1;
  static constexpr int GPW = NG * 4 / NWV;         // pixel groups per wave
  static constexpr int EPX = 16 * GPW;             // output pixels per wave per step
  // per-wave LDS landing zone of the epilogue inputs of its pixels (DMA'd at
  // the top of the step, read after the MFMAs): residual (EPX px x NB
  // channels), shortcut source pixels (EPX px x 32 channels), network input
  // (3 channel rows of EPX px, fp32 or fp16)
  static constexpr int EW = RES ? EPX * NB * 2 : SC ? EPX * 64 : HEAD ? 256 * GPW : 0;
  static constexpr int E = RES ? EPX * NB / 512 : SC ? EPX / 16 : HEAD ? 1 : 0;  // DMA instructions per wave per step
  static constexpr int LDS = WBYTES + RA::BYTES + (FAM ? RB::BYTES : 0) + NWV * EW;
  static constexpr int G = RA::G + (FAM ? RB::G : 0);              // ring DMA per step (waves 0-3)
  static constexpr bool OUT2 = (FL & kRingOut2) != 0;
  static constexpr bool OUT32 = (FL & kRingOut32) != 0;
  static constexpr bool R32 = (FL & kRingR32) != 0;
  static_assert(!R32 || OUT32, "res32 with the fp32 output");
  static_assert(!OUT32 || (!RES && !SC && !OUT2 && MODE != kRingHead && MODE != kRingFam), "fp32 output: plain convs");
  // stores per wave per step: one 16-byte store per fragment pair (ring_ch),
  // two with OUT2; OUT32 issues one or two more (its fp32 halves / fp16 copy,
  // runtime flags): counted at the minimum, so the waits below stay safe
  static constexpr bool PAIR = !FAM && !OUT32;
  static_assert(!PAIR || NT % 2 == 0, "fragment pairs");
  static constexpr int S = HEAD ? GPW : PAIR ? GPW * (NT / 2) * (OUT2 ? 2 : 1) : GPW * NT * (OUT2 ? 2 : 1);
  // vmcnt waits, waves 0-3 (ring DMA) / waves 4-7 (none): DMA(kk) has landed
  // at step 0 / step 1 / steps >= 2 / after a FAM pool flush (its atomics)
  static constexpr int W0 = G, W1 = E + G + S, WK = 2 * S + E + G, WF = WK + (FAM ? 4 * NT : 0);
  static constexpr int W1B = E + S, WKB = 2 * S + E, WFB = WKB + (FAM ? 4 * NT : 0);
  static_assert(WF <= 63, "vmcnt immediate");
  static_assert(!SC || (C == 64 && NB == 64 && MODE == kRingConv), "shortcut segment: enc1.conv2 only");
};

template <int MODE, int C, int NB, int FL>
__global__ __attribute__((amdgpu_flat_work_group_size(1, RingCfg<MODE, C, NB, FL>::THREADS),
                          amdgpu_waves_per_eu(RingCfg<MODE, C, NB, FL>::MINW))) void conv_ring_kernel(
    RingArgs a) {
  using K = RingCfg<MODE, C, NB, FL>;
  using RA = typename K::RA;
  using RB = typename K::RB;
  constexpr bool FAM = K::FAM, HEAD = K::HEAD, S2 = K::S2, RES = K::RES, SC = K::SC;
  constexpr int HA = K::HA, NT = K::NT, GPW = K::GPW;
  const ConvOp& op = a.op;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* Wl = smem;
  unsigned char* ringA = smem + K::WBYTES;
  unsigned char* ringB = ringA + RA::BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int wrow = wave & 3;                                  // output row of the step
  const int g0 = (wave >> 2) * GPW;                           // first pixel group of the wave
  const bool dma_wave = wave < 4;                             // waves 0-3 issue the ring DMA
  unsigned char* epi = ringA + RA::BYTES + (K::FAM ? RB::BYTES : 0) + wave * K::EW;
  const int fr = lane & 15, fg = lane >> 4;
  const int wswz = ((fr >> 2) & 1) << 1;
  const int H = op.Ho, W = op.Wo;
  const ConvSeg& sa = op.seg[0];
  const int Hin = sa.Hin, Win = sa.Win;
  // XCD-contiguous unit order: block -> v (units v, v + grid, ...)
  const int per_xcd = gridDim.x >> 3;
  const int v0 = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  const int nu = v0 < a.nunits ? (a.nunits - 1 - v0) / (int)gridDim.x + 1 : 0;
  const int KT = nu * a.steps;  // steps of this block

  f16x8_r wr[K::WREG ? K::NSL : 1][NT];
  if constexpr (K::WREG) {
    // lane (fr, fg) of fragment (slice, nt): W[nt*16 + fr][slice*32 + fg*8 .. +7]
#pragma unroll
    for (int sl = 0; sl < K::NSL; ++sl)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        wr[sl][nt] = *(const f16x8_r*)((const half_t*)op.W + (size_t)ring_chm<K::PAIR>(nt, fr) * op.Kpad + sl * 32 + fg * 8);
  } else {
    ring_load_filter<NB, K::THREADS, K::PAIR>(Wl, (const half_t*)op.W, op.Kpad, K::NSL, tid);
  }
  f16x8_r wsc[SC ? NT : 1];  // shortcut segment (k rows NSL*32 ..)
  if constexpr (SC) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      wsc[nt] = *(const f16x8_r*)((const half_t*)op.W + (size_t)ring_chm<K::PAIR>(nt, fr) * op.Kpad + K::NSL * 32 + fg * 8);
  }
  const half_t* srcA = (const half_t*)sa.src + sa.coff;
  const half_t* srcB = FAM ? (const half_t*)op.seg[2].src + op.seg[2].coff : nullptr;
  const int csA = sa.cs, csB = FAM ? op.seg[2].cs : 0;
  const half_t* zero = (const half_t*)g_ring_zero;
  const half_t* ninf = (const half_t*)g_ring_ninf;
  RingLanes<RA> la;
  RingLanes<RB> lb;
  la.init(lane, Win, csA);
  if constexpr (FAM) lb.init(lane, Win, csB);

  // unit j of this block -> (image b, first output row y0, strip origin x0)
  auto unit_of = [&](int j, int& b, int& y0, int& x0) {
    const int u = v0 + j * (int)gridDim.x;
    const int sx = u % a.nstrips, r = u / a.nstrips;
    b = r / a.nseg;
    y0 = (r % a.nseg) * a.rs;
    x0 = sx * K::TW;
  };
  // step cursors (wave-uniform): the compute cursor is at step kk, the DMA
  // cursor two steps ahead
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
  // DMA of the rows step dc.s of its unit first needs, into ring group (k+1) & 3
  auto issue = [&](int k) {
    const bool live = dc.j < nu;
    const int grp = (k + 1) & 3;
    if ((FL & kRingAblDma) && k >= 2) {
    } else if (!dma_wave) {
    } else if constexpr (S2) {
      la.issue(srcA, csA, dc.b, Hin, Win, 2 * (dc.y0 + 4 * dc.s), 2 * dc.x0 - 1, live, zero, ringA, grp, wave);
    } else {
      la.issue(srcA, csA, dc.b, Hin, Win, dc.y0 + 4 * dc.s + HA, dc.x0 - HA, live, zero, ringA, grp, wave);
      if constexpr (FAM)
        lb.issue(srcB, csB, dc.b, Hin, Win, dc.y0 + 4 * dc.s + 1, dc.x0 - 1, live, ninf, ringB, grp, wave);
    }
    advance(dc);
  };

  __syncthreads();  // filter in LDS (ordinary loads, waited for by hipcc)
  issue(0);
  issue(1);

  f32x4_r bias4[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) bias4[nt][i] = op.bias ? op.bias[K::PAIR ? ring_ch(nt, fg * 4 + i) : nt * 16 + fg * 4 + i] : 0.f;
  float hw2[NT][4];
  if constexpr (HEAD) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) hw2[nt][i] = op.head_w[ring_chm<K::PAIR>(nt, fg * 4 + i)];
  }
  float p2s[K::OUT2 ? NT : 1][4], p2h[K::OUT2 ? NT : 1][4];
  if constexpr (K::OUT2) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        p2s[nt][i] = op.pre2_scale[ring_chm<K::PAIR>(nt, fg * 4 + i)];
        p2h[nt][i] = op.pre2_shift[ring_chm<K::PAIR>(nt, fg * 4 + i)];
      }
  }
  const int abase = fg * RA::PLANE + fr * 16;  // chunk plane fg, pixel fr of a ring row
  const int bbase = fg * RB::PLANE + fr * 16;
  // lane parts of the epilogue addresses (pixel g*16 + fr of the row, channels fg*4..)
  const int ocs = op.out_cs, rcs = RES ? op.res2_cs : 0;
  static_assert(K::THREADS <= 512 && NT <= 4, "sink: 128 bytes per thread");
  int oloff[GPW];
#pragma unroll
  for (int g = 0; g < GPW; ++g) oloff[g] = ((g0 + g) * 16 + fr) * ocs + fg * (K::PAIR ? 8 : 4);
  const size_t HWs = (size_t)H * W;
  const ConvSeg& ss = op.seg[SC ? 1 : 0];
  const half_t* scsrc = (const half_t*)ss.src + ss.coff;
  const int sccs = ss.cs, scH = ss.Hin, scW = ss.Win;

  float pool[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) pool[nt][i] = 0.f;
  bool flushed = false;

  for (int kk = 0; kk < KT; ++kk) {
    // (A) DMA(kk) has landed (younger: stores(kk-2), loads(kk-1), DMA(kk+1), stores(kk-1))
    // (+ the previous step's pool atomics when it ended a FAM unit)
    if (dma_wave) {
      if (kk == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::W0) : "memory");
      else if (kk == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::W1) : "memory");
      else if (flushed) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::WF) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::WK) : "memory");
    } else {
      // no ring DMA: only this wave's landing-zone reads must be behind the barrier
      if (kk == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (kk == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::W1B) : "memory");
      else if (flushed) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::WFB) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::WKB) : "memory");
    }
    __builtin_amdgcn_s_barrier();
    flushed = false;
    const int s = cc.s, b = cc.b, x0 = cc.x0;
    const int yend = min(H, cc.y0 + a.rs);
    const int y = cc.y0 + 4 * s + wrow;
    const bool rowok = s >= 0 && y < yend;
    const size_t prow = (size_t)(b * H + (rowok ? y : 0)) * W + x0;  // first pixel of this wave's output row

    // epilogue / shortcut inputs of this wave's output row -> its LDS landing
    // zone (LDS-DMA: no registers in flight, nothing for hipcc to reorder);
    // waited for after the MFMAs with vmcnt(G) (only DMA(kk+2) is younger)
    const int xw = x0 + g0 * 16;  // first output pixel of the wave
    bool ovalid[GPW];
#pragma unroll
    for (int g = 0; g < GPW; ++g) ovalid[g] = rowok && xw + g * 16 + fr < W;
    if constexpr (RES) {
      // EPX px x NB channels, pixel-major; the 16-byte chunks of landing pixel
      // l are XOR-permuted by ring_res_swz(l) so the epilogue's 8-byte reads
      // (16 pixels x 2 channel quads per 32-lane group) hit 32 distinct bank
      // pairs (the plain layout was 4-8-way: 56% of this kernel's LDS cycles)
      constexpr int CPP = NB / 8;  // 16-byte chunks per pixel
#pragma unroll
      for (int i = 0; i < K::E; ++i) {
        const int q = i * 64 + lane, l = q / CPP, px = g0 * 16 + l;
        const bool ok = rowok && x0 + px < W;
        const half_t* p =
            ok ? (const half_t*)op.res2 + (prow + px) * rcs + ((q % CPP) ^ ring_res_swz<CPP>(l)) * 8 : zero;
        __builtin_amdgcn_global_load_lds(p, (lds_void_ptr_r)(epi + i * 1024), 16, 0, 0);
      }
    }
    if constexpr (SC) {
      // the 1x1 stride-2 shortcut's source pixels (2y, 2x) of the row, 32 channels
#pragma unroll
      for (int i = 0; i < K::E; ++i) {
        const int q = i * 64 + lane, px = g0 * 16 + (q >> 2);
        const bool ok = rowok && x0 + px < W;
        const half_t* p = ok ? scsrc + ((size_t)(b * scH + 2 * y) * scW + 2 * (x0 + px)) * sccs + (q & 3) * 8 : zero;
        __builtin_amdgcn_global_load_lds(p, (lds_void_ptr_r)(epi + i * 1024), 16, 0, 0);
      }
    }
    if constexpr (HEAD) {
      // network input: 3 channel rows of the wave's pixels (NCHW), 16-byte chunks
      const int ppc = op.x_f16 ? 8 : 4;   // pixels per chunk
      const int cpr = K::EPX / ppc;       // chunks per channel row
      if (lane < 3 * cpr) {
        const int c = lane / cpr, k = lane % cpr;
        const bool ok = rowok && xw + k * ppc < W;
        const size_t e = (size_t)b * 2 * HWs + prow + g0 * 16 + c * HWs + k * ppc;  // (b*3 + c)*HW + y*W + x
        const void* p = !ok ? (const void*)zero
                            : op.x_f16 ? (const void*)((const half_t*)op.x_nchw + e) : (const void*)(op.x_nchw + e);
        __builtin_amdgcn_global_load_lds(p, (lds_void_ptr_r)epi, 16, 0, 0);  // lane -> epi + 16 * lane
      }
    }
    issue(kk + 2);

    // ---- MFMAs: D[n][px] = bias[n] + sum_k W[n][k] * X[px][k] -----------------
    f32x4_r acc[NT][GPW];
    // plain programs: the bias is the C operand of each tile's first MFMA (no
    // per-step copies into the accumulators); FAM / DMA-only steps start from it here
    if (FAM || s < 0) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int g = 0; g < GPW; ++g) acc[nt][g] = bias4[nt];
    }
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
      if constexpr (!FAM) {
        // chunk c = (tap row r, 32-channel slice ks): 3 taps x NG pixel groups
        // of X fragments (+ the 3 x NT filter fragments when the filter is in LDS)
        constexpr int NCH = 3 * K::KS;
        constexpr int NW = K::WREG ? 1 : 3;
        constexpr int NX = 3 * GPW;
        // ring row of tap row r: stride 1 -> input row y + r - 1; stride 2 -> 2y + r - 1
        auto rowA = [&](int r) {
          if constexpr (S2) return ((8 * kk + 8 + 2 * wrow - 1 + r) & (RA::RR - 1)) * (RA::RW * 16);
          else return ((4 * kk + 4 + wrow - HA + r - 1) & (RA::RR - 1)) * (RA::RW * 16);
        };
        // ring column of tap sc, pixel group g (lane pixel fr added by abase)
        auto colA = [&](int sc, int g) {
          if constexpr (S2) return sc == 1 ? RA::HALF : sc / 2;
          else return (g0 + g) * 16 + sc;
        };
        f16x8_r bx[2][NX], bw[2][NW][NT];
        auto ld = [&](int c, f16x8_r (&x)[NX], f16x8_r (&w)[NW][NT]) {
          const int r = c / K::KS, ks = c % K::KS;
          const unsigned char* xr = ringA + abase + rowA(r) + ks * 4 * RA::PLANE;
#pragma unroll
          for (int sc = 0; sc < 3; ++sc)
#pragma unroll
            for (int g = 0; g < GPW; ++g) x[sc * GPW + g] = *(const f16x8_r*)(xr + colA(sc, g) * 16);
          if constexpr (!K::WREG) {
#pragma unroll
            for (int sc = 0; sc < 3; ++sc) ring_filter_frags<NT, NB>(Wl, (r * 3 + sc) * K::KS + ks, fr, fg, wswz, w[sc]);
          }
        };
        auto mm = [&](int c, const f16x8_r (&x)[NX], const f16x8_r (&w)[NW][NT]) {
          const int r = c / K::KS, ks = c % K::KS;
#pragma unroll
          for (int sc = 0; sc < 3; ++sc)
#pragma unroll
            for (int g = 0; g < GPW; ++g)
#pragma unroll
              for (int nt = 0; nt < NT; ++nt) {
                f16x8_r wf;
                if constexpr (K::WREG) wf = wr[(r * 3 + sc) * K::KS + ks][nt];
                else wf = w[sc][nt];
                if constexpr ((FL & kRingAblMma) != 0) {
                  if (c == 0 && sc == 0) acc[nt][g] = bias4[nt] + (f32x4_r)__builtin_bit_cast(f32x4_r, x[sc * GPW + g]);
                } else {
                  acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf, x[sc * GPW + g],
                                                                      c == 0 && sc == 0 ? bias4[nt] : acc[nt][g], 0, 0, 0);
                }
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
        // h3 (3x3, d1): slices 0..8, planes 0-3; h4 (3x3, d2): slices 9..17,
        // planes 4-7; then x (1x1, slice 18) and maxpool3(x) (1x1, slice 19)
        // from the x ring.  Chunk = one ring row (3 taps x 2 pixel groups).
        static_assert(K::WREG, "FAM keeps its filter in registers");
        auto rowA = [&](int dy) { return ((4 * kk + 4 + wrow - HA + dy) & (RA::RR - 1)) * (RA::RW * 16); };
        auto rowB = [&](int dy) { return ((4 * kk + 4 + wrow - 1 + dy) & (RB::RR - 1)) * (RB::RW * 16); };
        constexpr int NB6 = 3 * GPW;  // fragments per chunk
        auto ld_h = [&](int c, f16x8_r (&buf)[NB6]) {
          const int seg = c / 3, r = c % 3, d = seg + 1;
          const unsigned char* xr = ringA + abase + seg * 4 * RA::PLANE + rowA((r - 1) * d);
#pragma unroll
          for (int sc = 0; sc < 3; ++sc)
#pragma unroll
            for (int g = 0; g < GPW; ++g)
              buf[sc * GPW + g] = *(const f16x8_r*)(xr + ((g0 + g) * 16 + 2 + (sc - 1) * d) * 16);
        };
        auto ld_x = [&](int dr, f16x8_r (&buf)[NB6]) {
          const unsigned char* xr = ringB + bbase + rowB(dr - 1);
#pragma unroll
          for (int ds = 0; ds < 3; ++ds)
#pragma unroll
            for (int g = 0; g < GPW; ++g) buf[ds * GPW + g] = *(const f16x8_r*)(xr + ((g0 + g) * 16 + ds) * 16);
        };
        auto mm_h = [&](int c, const f16x8_r (&buf)[NB6]) {
          const int seg = c / 3, r = c % 3;
#pragma unroll
          for (int sc = 0; sc < 3; ++sc)
#pragma unroll
            for (int g = 0; g < GPW; ++g)
#pragma unroll
              for (int nt = 0; nt < NT; ++nt)
                acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[seg * 9 + r * 3 + sc][nt], buf[sc * GPW + g],
                                                                    acc[nt][g], 0, 0, 0);
        };
        f16x8_r ctr[GPW], mx[GPW];
        auto mp = [&](int dr, const f16x8_r (&buf)[NB6]) {
#pragma unroll
          for (int ds = 0; ds < 3; ++ds)
#pragma unroll
            for (int g = 0; g < GPW; ++g) {
              const f16x8_r v = buf[ds * GPW + g];
              if (dr == 0 && ds == 0) mx[g] = v;
              else mx[g] = __builtin_elementwise_max(mx[g], v);
              if (dr == 1 && ds == 1) ctr[g] = v;
            }
        };
        f16x8_r b0[NB6], b1[NB6];
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
        for (int g = 0; g < GPW; ++g)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[18][nt], ctr[g], acc[nt][g], 0, 0, 0);
            acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[19][nt], mx[g], acc[nt][g], 0, 0, 0);
          }
      }
    }
#undef RING_LDS_DONE
#undef RING_FENCE

    // (B) this step's epilogue inputs have landed (only DMA(kk+2) is younger)
    if (dma_wave) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::G) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (SC) {
      if (s >= 0) {
#pragma unroll
        for (int g = 0; g < GPW; ++g) {
          const f16x8_r xf = *(const f16x8_r*)(epi + (g * 16 + fr) * 64 + fg * 16);
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wsc[nt], xf, acc[nt][g], 0, 0, 0);
        }
      }
    }

    // ---- epilogue ---------------------------------------------------------------
    if constexpr (HEAD) {
      // r = sum_n relu(v_n) * w2_n ; illu = sigmoid(mean_c(x) + r + b2)
#pragma unroll
      for (int g = 0; g < GPW; ++g) {
        float part = 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) part += fmaxf(acc[nt][g][i], 0.f) * hw2[nt][i];
        part += __shfl_xor(part, 16);
        part += __shfl_xor(part, 32);
        const int xp = g * 16 + fr;
        float x0f, x1f, x2f;
        if (op.x_f16) {
          const half_t* xl = (const half_t*)epi;
          x0f = (float)xl[xp];
          x1f = (float)xl[K::EPX + xp];
          x2f = (float)xl[2 * K::EPX + xp];
        } else {
          const float* xl = (const float*)epi;
          x0f = xl[xp];
          x1f = xl[K::EPX + xp];
          x2f = xl[2 * K::EPX + xp];
        }
        const float z = (x0f + x1f + x2f) / 3.f + (part + op.head_b);
        const float il = 1.f / (1.f + expf(-z));
        float* dst = (ovalid[g] && fg == 0) ? op.illu + prow + (g0 + g) * 16 + fr : (float*)(g_ring_sink + tid);
        *dst = il;
      }
    } else {
#pragma unroll
      for (int g = 0; g < GPW; ++g) {
        // one pointer per pixel group (the sink for invalid outputs), channel tiles at immediates
        half_t* dg = ovalid[g] ? (half_t*)op.out + prow * ocs + op.out_coff + oloff[g]
                               : (half_t*)(g_ring_sink + tid * 16);
        if constexpr (K::PAIR) {
#pragma unroll
        for (int p = 0; p < NT / 2; ++p) {
          // fragments 2p, 2p + 1: channels 32p + 8fg .. + 7 of pixel fr (ring_ch)
          float v[8];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = acc[2 * p][g][i];
            v[4 + i] = acc[2 * p + 1][g][i];
          }
          if constexpr (K::RELU && RES) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], 0.f);
          }
          if constexpr (RES) {
            const int k = 4 * p + fg;  // logical 16-byte chunk of this lane's 8 channels
            const f16x8_r rr = *(const f16x8_r*)(epi + (g * 16 + fr) * NB * 2 + ((k ^ ring_res_swz<NB / 8>(fr)) * 16));
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] += (float)rr[i];
          }
          f16x8_r o;
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = (half_t)v[i];
          if constexpr (K::RELU && !RES) {
            // relu after the RNE rounding (the same values: rounding is monotone and
            // keeps the sign) as a signed 16-bit max per pair: every negative half,
            // -0 included, becomes +0 -- 4 instructions per 8 channels instead of 16
            // (inline asm: written as vector code, hipcc split the packed conversions
            // into per-element ones + permutes to feed an element-wise max)
            uint4 w = __builtin_bit_cast(uint4, o);
            asm("v_pk_max_i16 %0, %1, 0" : "=v"(w.x) : "v"(w.x));
            asm("v_pk_max_i16 %0, %1, 0" : "=v"(w.y) : "v"(w.y));
            asm("v_pk_max_i16 %0, %1, 0" : "=v"(w.z) : "v"(w.z));
            asm("v_pk_max_i16 %0, %1, 0" : "=v"(w.w) : "v"(w.w));
            o = __builtin_bit_cast(f16x8_r, w);
          }
          if constexpr (K::OUT32) {
            // (float)(fp16 result) + res32, zeroed where mask16 <= 0 (the order
            // of direct_epilogue); the fp16 copy is the fp32 value stored
            f32x4_r o32a, o32b;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              o32a[i] = (float)o[i];
              o32b[i] = (float)o[4 + i];
            }
            if constexpr (K::R32) {
              if (ovalid[g]) {
                const float* r32 =
                    op.res32 + prow * op.res32_cs + (size_t)((g0 + g) * 16 + fr) * op.res32_cs + fg * 8 + p * 32;
                o32a += *(const f32x4_r*)r32;
                o32b += *(const f32x4_r*)(r32 + 4);
              }
            }
            if (op.mask16 && ovalid[g]) {
              const half_t* mk = (const half_t*)op.mask16 + prow * op.mask16_cs +
                                 (size_t)((g0 + g) * 16 + fr) * op.mask16_cs + fg * 8 + p * 32;
              const f16x8_r mv = *(const f16x8_r*)mk;
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                o32a[i] = (float)mv[i] > 0.f ? o32a[i] : 0.f;
                o32b[i] = (float)mv[4 + i] > 0.f ? o32b[i] : 0.f;
              }
            }
            float* d32 = ovalid[g] ? op.out32 + prow * op.out32_cs + op.out32_coff +
                                         (size_t)((g0 + g) * 16 + fr) * op.out32_cs + fg * 8
                                   : g_ring_sink32 + tid * 64;
            if (!op.skip32) {
              *(f32x4_r*)(d32 + p * 32) = o32a;
              *(f32x4_r*)(d32 + p * 32 + 4) = o32b;
            }
            if (op.out32_h16) {
              f16x8_r h;
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                h[i] = (half_t)o32a[i];
                h[4 + i] = (half_t)o32b[i];
              }
              half_t* d16 = ovalid[g] ? (half_t*)op.out32_h16 + prow * op.out32_h16_cs +
                                            (size_t)((g0 + g) * 16 + fr) * op.out32_h16_cs + fg * 8
                                      : (half_t*)(g_ring_sink + tid * 16);
              *(uint4*)(d16 + p * 32) = __builtin_bit_cast(uint4, h);
            }
          } else {
            *(uint4*)(dg + p * 32) = __builtin_bit_cast(uint4, o);
          }
          if constexpr (K::OUT2) {
            f16x8_r q;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              q[i] = (half_t)fmaxf(__builtin_fmaf((float)o[i], p2s[2 * p][i], p2h[2 * p][i]), 0.f);
              q[4 + i] = (half_t)fmaxf(__builtin_fmaf((float)o[4 + i], p2s[2 * p + 1][i], p2h[2 * p + 1][i]), 0.f);
            }
            half_t* d2 = ovalid[g] ? (half_t*)op.out2 + prow * ocs + oloff[g] : (half_t*)(g_ring_sink + tid * 16);
            *(uint4*)(d2 + p * 32) = __builtin_bit_cast(uint4, q);
          }
        }
        } else {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = acc[nt][g][i];
            if constexpr (K::RELU && RES) v[i] = fmaxf(v[i], 0.f);
          }
          if constexpr (RES) {
            const int k = nt * 2 + (fg >> 1);  // logical 16-byte chunk of this lane's 4 channels
            const f16x4_r rr = *(const f16x4_r*)(epi + (g * 16 + fr) * NB * 2 + ((k ^ ring_res_swz<NB / 8>(fr)) * 16) +
                                                 (fg & 1) * 8);
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] += (float)rr[i];
          }
          f16x4_r o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = (half_t)v[i];
          if constexpr (K::RELU && !RES) {
            // relu after the RNE rounding, as a signed 16-bit max per pair (see above)
            uint2 w = __builtin_bit_cast(uint2, o);
            asm("v_pk_max_i16 %0, %1, 0" : "=v"(w.x) : "v"(w.x));
            asm("v_pk_max_i16 %0, %1, 0" : "=v"(w.y) : "v"(w.y));
            o = __builtin_bit_cast(f16x4_r, w);
          }
          if constexpr (FAM) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (ovalid[g]) pool[nt][i] += (float)o[i];
          }
          if constexpr (K::OUT32) {
            f32x4_r o32;
#pragma unroll
            for (int i = 0; i < 4; ++i) o32[i] = (float)o[i];
            if constexpr (K::R32) {
              if (ovalid[g])
                o32 += *(const f32x4_r*)(op.res32 + prow * op.res32_cs + (size_t)((g0 + g) * 16 + fr) * op.res32_cs +
                                         fg * 4 + nt * 16);
            }
            if (op.mask16 && ovalid[g]) {
              const half_t* mk = (const half_t*)op.mask16 + prow * op.mask16_cs +
                                 (size_t)((g0 + g) * 16 + fr) * op.mask16_cs + fg * 4 + nt * 16;
              const uint2 mw = *(const uint2*)mk;
              const f16x4_r mv = __builtin_bit_cast(f16x4_r, mw);
#pragma unroll
              for (int i = 0; i < 4; ++i) o32[i] = (float)mv[i] > 0.f ? o32[i] : 0.f;
            }
            float* d32 = ovalid[g] ? op.out32 + prow * op.out32_cs + op.out32_coff +
                                         (size_t)((g0 + g) * 16 + fr) * op.out32_cs + fg * 4
                                   : g_ring_sink32 + tid * 64;
            if (!op.skip32) *(f32x4_r*)(d32 + nt * 16) = o32;
            if (op.out32_h16) {
              const f16x4_r h = {(half_t)o32[0], (half_t)o32[1], (half_t)o32[2], (half_t)o32[3]};
              half_t* d16 = ovalid[g] ? (half_t*)op.out32_h16 + prow * op.out32_h16_cs +
                                            (size_t)((g0 + g) * 16 + fr) * op.out32_h16_cs + fg * 4
                                      : (half_t*)(g_ring_sink + tid * 16);
              *(uint2*)(d16 + nt * 16) = __builtin_bit_cast(uint2, h);
            }
          } else {
            *(uint2*)(dg + nt * 16) = __builtin_bit_cast(uint2, o);
          }
          if constexpr (K::OUT2) {
            f16x4_r q;
#pragma unroll
            for (int i = 0; i < 4; ++i) q[i] = (half_t)fmaxf(__builtin_fmaf((float)o[i], p2s[nt][i], p2h[nt][i]), 0.f);
            half_t* d2 = ovalid[g] ? (half_t*)op.out2 + prow * ocs + oloff[g] : (half_t*)(g_ring_sink + tid * 16);
            *(uint2*)(d2 + nt * 16) = __builtin_bit_cast(uint2, q);
          }
        }
        }
      }
    }
    // FAM: per-image channel sums, flushed at the end of every unit (a unit is one image)
    if constexpr (FAM) {
      if (op.pool && s == a.steps - 2) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v = pool[nt][i];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if (fr == 0) pool_add(op.pool, (size_t)b * op.N + nt * 16 + fg * 4 + i, v);
            pool[nt][i] = 0.f;
          }
        flushed = true;
      }
    }
    advance(cc);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// fp32 form (the configs[1] graph): the same ring / step / DMA structure for the
// 32-channel stride-1 3x3 convs at 512^2 (UpBlock dec1 convs, residual head,
// FAM branch3/4 first convs), on v_mfma_f32_16x16x4_f32.  A 16-byte chunk holds
// 4 channels, so a 32-channel slice is 8 chunk planes; each MFMA contracts 4
// channels and the slice's 8 MFMAs use the k order "lane group fg takes
// channels fg*8 .. fg*8+7" for both operands (any permutation of k shared by A
// and B leaves the sum unchanged): a lane reads its pixel's 8 channels as two
// conflict-free ds_read_b128 (planes 2fg, 2fg+1) per tap and feeds 8 MFMAs.
// fp32 MFMA time (32 cycles per 16x16x4) bounds these layers, not HBM.
// ---------------------------------------------------------------------------
// fp32 landing zone: rows of CPP 16-byte chunks read by ds_read_b128 lane
// groups {fr 0-3, 12-15 | fg 0} + {fr 4-11 | fg 1}: (l >> 1) & 7 for 8-chunk
// rows (the aligned-row swizzle of the wide kernels), l & 15 for 16-chunk rows
template <int CPP>
__device__ __forceinline__ int ring32_res_swz(int l) {
  if constexpr (CPP == 8) return (l >> 1) & 7;
  else return l & 15;
}

template <int MODE, int NB, int FL>
struct Ring32Cfg {
  static constexpr bool HEAD = MODE == kRingHead;
  static constexpr bool RES = FL & kRingRes, RELU = (FL & kRingRelu) != 0;
  static constexpr bool RESPRE = (FL & kRingResPre) != 0, POOL = (FL & kRingPool) != 0;
  static constexpr int DIL = (FL & kRingDil2) ? 2 : 1, HA = DIL;  // ring halo = the taps' reach
  static constexpr bool XP = (FL & kRingXPool) != 0;
  static constexpr int C = 32, NT = NB / 16, NG = 2;
  using RA = Ring<8, 32 + 2 * HA, 4>;               // 32 fp32 channels = 8 chunk planes
  using RB = Ring<8, 34, 4>;                        // kRingXPool: x, 1-pixel -inf halo
  static constexpr int NSL = XP ? 11 : 9;           // K slices of 32 channels
  // filter in registers: 9 (11) slices x NT tiles x 8 floats = 144 (176) / 288
  // VGPRs (one wave per SIMD: 32 -> 64 fits in 504 registers without spills;
  // the residual variant does not)
  static constexpr bool WREG = NT == 2 || (NT == 4 && !RES);
  static constexpr int WBYTES = WREG ? 0 : 9 * NB * 32 * 4;  // [tap][n][32 k] fp32
  static constexpr int EW = RES ? 32 * NB * 4 : HEAD ? 512 : 0;
  static constexpr int E = RES ? NB / 8 : HEAD ? 1 : 0;
  static constexpr int LDS = WBYTES + RA::BYTES + (XP ? RB::BYTES : 0) + 4 * EW;
  static constexpr int G = RA::G + (XP ? RB::G : 0);
  static constexpr int S = HEAD ? NG : NG * NT;
  static constexpr int W0 = G, W1 = E + G + S, WK = 2 * S + E + G, WF = WK + (POOL ? 4 * NT : 0);
  static_assert(WF <= 63, "vmcnt immediate");
  static_assert(!RESPRE || RES, "kRingResPre qualifies kRingRes");
  static_assert(!(HEAD && (POOL || DIL == 2)), "head: plain 3x3");
  static_assert(!XP || (WREG && DIL == 1 && !RES && !HEAD), "x / maxpool slices: the FAM h3 part");
};

template <int MODE, int NB, int FL>
__global__ __launch_bounds__(256) void conv_ring32_kernel(RingArgs a) {
  using K = Ring32Cfg<MODE, NB, FL>;
  using RA = typename K::RA;
  constexpr bool HEAD = K::HEAD, RES = K::RES;
  constexpr int NT = K::NT, NG = K::NG, HA = K::HA, DIL = K::DIL;
  using RB = typename K::RB;
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const ConvOp& op = a.op;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* Wl = smem;
  unsigned char* ringA = smem + K::WBYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  unsigned char* ringB = ringA + RA::BYTES;
  unsigned char* epi = ringA + RA::BYTES + (K::XP ? RB::BYTES : 0) + wave * K::EW;
  const int H = op.Ho, W = op.Wo;
  const ConvSeg& sa = op.seg[0];
  const int per_xcd = gridDim.x >> 3;
  const int v0 = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  const int nu = v0 < a.nunits ? (a.nunits - 1 - v0) / (int)gridDim.x + 1 : 0;
  const int KT = nu * a.steps;

  // filter: lane (fr = n within tile, fg) holds W[nt*16 + fr][tap*32 + fg*8 .. +7]
  f32x4 wr[K::WREG ? K::NSL : 1][NT][2];
  if constexpr (K::WREG) {
#pragma unroll
    for (int t = 0; t < K::NSL; ++t)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          wr[t][nt][h] = *(const f32x4*)((const float*)op.W + (size_t)(nt * 16 + fr) * op.Kpad + t * 32 + fg * 8 + h * 4);
  } else {
    // LDS [tap][n][32 floats], the 8-float run of lane group fg at 32*fg bytes (+ h*16)
    for (int i = tid; i < 9 * NB * 8; i += 256) {
      const int c4 = i & 7, n = (i >> 3) % NB, t = (i >> 3) / NB;
      *(f32x4*)(Wl + (size_t)i * 16) = *(const f32x4*)((const float*)op.W + (size_t)n * op.Kpad + t * 32 + c4 * 4);
    }
  }
  const half_t* srcA = (const half_t*)((const float*)sa.src + sa.coff);  // element offsets in halves below
  const int csA = sa.cs * 2;                                           // pixel stride in halves
  const half_t* zero = (const half_t*)g_ring_zero;
  RingLanes<RA> la;
  la.init(lane, sa.Win, csA);
  const ConvSeg& sx = op.seg[K::XP ? 1 : 0];
  const half_t* srcB = (const half_t*)((const float*)sx.src + sx.coff);
  const int csB = sx.cs * 2;
  const half_t* ninf = (const half_t*)g_ring_ninf32;
  RingLanes<RB> lb;
  if constexpr (K::XP) lb.init(lane, sx.Win, csB);

  auto unit_of = [&](int j, int& b, int& y0, int& x0) {
    const int u = v0 + j * (int)gridDim.x;
    const int sx = u % a.nstrips, r = u / a.nstrips;
    b = r / a.nseg;
    y0 = (r % a.nseg) * a.rs;
    x0 = sx * 32;
  };
  const int S = a.steps - 1;
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
  // RingLanes addresses half_t elements: an fp32 chunk c (4 channels) is at
  // half offset 8c, i.e. plane c <-> chunk c of the pixel
  auto issue = [&](int k) {
    const bool live = dc.j < nu;
    la.issue(srcA, csA, dc.b, sa.Hin, sa.Win, dc.y0 + 4 * dc.s + HA, dc.x0 - HA, live, zero, ringA, (k + 1) & 3, wave);
    if constexpr (K::XP)
      lb.issue(srcB, csB, dc.b, sx.Hin, sx.Win, dc.y0 + 4 * dc.s + 1, dc.x0 - 1, live, ninf, ringB, (k + 1) & 3, wave);
    advance(dc);
  };

  __syncthreads();
  issue(0);
  issue(1);

  float bv[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[nt][i] = op.bias ? op.bias[nt * 16 + fg * 4 + i] : 0.f;
  float hw2[NT][4];
  if constexpr (HEAD) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) hw2[nt][i] = op.head_w[nt * 16 + fg * 4 + i];
  }
  const int abase = 2 * fg * RA::PLANE + fr * 16;  // planes 2fg, 2fg+1 (channels fg*8 .. +7)
  const int ocs = op.out_cs, rcs = RES ? (K::RESPRE ? op.res1_cs : op.res2_cs) : 0;
  const float* resp = RES ? (const float*)(K::RESPRE ? op.res1 : op.res2) : nullptr;
  const size_t HWs = (size_t)H * W;
  float pool[K::POOL ? NT : 1][4];
#pragma unroll
  for (int nt = 0; nt < (K::POOL ? NT : 1); ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) pool[nt][i] = 0.f;
  bool flushed = false;

  for (int kk = 0; kk < KT; ++kk) {
    // (the previous step's pool atomics, when it ended a unit, are younger than DMA(kk) too)
    if (kk == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::W0) : "memory");
    else if (kk == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::W1) : "memory");
    else if (K::POOL && flushed) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::WF) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::WK) : "memory");
    __builtin_amdgcn_s_barrier();
    flushed = false;
    const int s = cc.s, b = cc.b, x0 = cc.x0;
    const int yend = min(H, cc.y0 + a.rs);
    const int y = cc.y0 + 4 * s + wave;
    const bool rowok = s >= 0 && y < yend;
    const size_t prow = (size_t)(b * H + (rowok ? y : 0)) * W + x0;
    bool ovalid[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) ovalid[g] = rowok && x0 + g * 16 + fr < W;
    if constexpr (RES) {
      // 32 px x NB fp32 channels, pixel-major, chunks XOR-permuted per pixel
      // (conflict-free 16-byte epilogue reads)
      constexpr int CPP = NB / 4;
#pragma unroll
      for (int i = 0; i < K::E; ++i) {
        const int q = i * 64 + lane, px = q / CPP;
        const bool ok = rowok && x0 + px < W;
        const void* p = ok ? (const void*)(resp + (prow + px) * rcs + ((q % CPP) ^ ring32_res_swz<CPP>(px)) * 4)
                           : (const void*)zero;
        __builtin_amdgcn_global_load_lds(p, (lds_void_ptr_r)(epi + i * 1024), 16, 0, 0);
      }
    }
    if constexpr (HEAD) {
      const int ppc = op.x_f16 ? 8 : 4, cpr = 32 / ppc;
      if (lane < 3 * cpr) {
        const int c = lane / cpr, k = lane % cpr;
        const bool ok = rowok && x0 + k * ppc < W;
        const size_t e = (size_t)b * 2 * HWs + prow + c * HWs + k * ppc;
        const void* p = !ok ? (const void*)zero
                            : op.x_f16 ? (const void*)((const half_t*)op.x_nchw + e) : (const void*)(op.x_nchw + e);
        __builtin_amdgcn_global_load_lds(p, (lds_void_ptr_r)epi, 16, 0, 0);
      }
    }
    issue(kk + 2);

    f32x4 acc[NT][NG];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int g = 0; g < NG; ++g) acc[nt][g] = f32x4{bv[nt][0], bv[nt][1], bv[nt][2], bv[nt][3]};
#define RING_FENCE __builtin_amdgcn_sched_barrier(0)
#define RING_LDS_DONE                                                               \
  do {                                                                              \
    RING_FENCE;                                                                     \
    __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0); vmcnt / expcnt untouched */ \
    RING_FENCE;                                                                     \
  } while (0)
    if (s >= 0) {
      // chunk = one tap row r: 3 taps x 2 groups x 2 halves of X (+ 3 x NT x 2 of W from LDS)
      // ring row of tap row r (input row y + (r - 1) * DIL); ring column of tap sc below
      auto rowA = [&](int r) { return ((4 * kk + 4 + wave - HA + (r - 1) * DIL) & 15) * (RA::RW * 16); };
      constexpr int NW = K::WREG ? 1 : 3;
      f32x4 bx[2][3][NG][2], bw[2][NW][NT][2];
      auto ld = [&](int r, f32x4 (&x)[3][NG][2], f32x4 (&w)[NW][NT][2]) {
        const unsigned char* xr = ringA + abase + rowA(r);
#pragma unroll
        for (int sc = 0; sc < 3; ++sc)
#pragma unroll
          for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int h = 0; h < 2; ++h)
              x[sc][g][h] = *(const f32x4*)(xr + h * RA::PLANE + (g * 16 + HA + (sc - 1) * DIL) * 16);
        if constexpr (!K::WREG) {
#pragma unroll
          for (int sc = 0; sc < 3; ++sc)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
              for (int h = 0; h < 2; ++h)
                w[sc][nt][h] = *(const f32x4*)(Wl + ((size_t)((r * 3 + sc) * NB + nt * 16 + fr) * 32 + fg * 8 + h * 4) * 4);
        }
      };
      auto mm = [&](int r, const f32x4 (&x)[3][NG][2], const f32x4 (&w)[NW][NT][2]) {
#pragma unroll
        for (int sc = 0; sc < 3; ++sc)
#pragma unroll
          for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int g = 0; g < NG; ++g)
#pragma unroll
              for (int nt = 0; nt < NT; ++nt) {
                const float wv = K::WREG ? wr[r * 3 + sc][nt][j >> 2][j & 3] : w[K::WREG ? 0 : sc][nt][j >> 2][j & 3];
                acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv, x[sc][g][j >> 2][j & 3], acc[nt][g], 0, 0, 0);
              }
      };
      ld(0, bx[0], bw[0]);
      ld(1, bx[1], bw[1]);
      RING_LDS_DONE;
      mm(0, bx[0], bw[0]);
      RING_FENCE;
      ld(2, bx[0], bw[0]);
      RING_FENCE;
      mm(1, bx[1], bw[1]);
      RING_LDS_DONE;
      if constexpr (K::XP) {
        // x rows y-1..y+1 of the x ring -> centre and 3x3 max per pixel group and channel half
        const int bbase = 2 * fg * RB::PLANE + fr * 16;
        auto rowB = [&](int dy) { return ((4 * kk + 4 + wave - 1 + dy) & 15) * (RB::RW * 16); };
        f32x4 xr3[3][NG][2];
#pragma unroll
        for (int sc = 0; sc < 3; ++sc)
#pragma unroll
          for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int h = 0; h < 2; ++h)
              xr3[sc][g][h] = *(const f32x4*)(ringB + bbase + rowB(-1) + h * RB::PLANE + (g * 16 + sc) * 16);
        RING_FENCE;
        mm(2, bx[0], bw[0]);
        RING_LDS_DONE;
        f32x4 ctr[NG][2], mx[NG][2];
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            mx[g][h] = __builtin_elementwise_max(__builtin_elementwise_max(xr3[0][g][h], xr3[1][g][h]), xr3[2][g][h]);
#pragma unroll
        for (int dr = 1; dr < 3; ++dr) {
#pragma unroll
          for (int sc = 0; sc < 3; ++sc)
#pragma unroll
            for (int g = 0; g < NG; ++g)
#pragma unroll
              for (int h = 0; h < 2; ++h)
                xr3[sc][g][h] = *(const f32x4*)(ringB + bbase + rowB(dr - 1) + h * RB::PLANE + (g * 16 + sc) * 16);
          RING_LDS_DONE;
#pragma unroll
          for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              mx[g][h] = __builtin_elementwise_max(
                  mx[g][h], __builtin_elementwise_max(__builtin_elementwise_max(xr3[0][g][h], xr3[1][g][h]), xr3[2][g][h]));
              if (dr == 1) ctr[g][h] = xr3[1][g][h];
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
              acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[9][nt][j >> 2][j & 3], ctr[g][j >> 2][j & 3],
                                                                acc[nt][g], 0, 0, 0);
              acc[nt][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[10][nt][j >> 2][j & 3], mx[g][j >> 2][j & 3],
                                                                acc[nt][g], 0, 0, 0);
            }
      } else {
        mm(2, bx[0], bw[0]);
      }
    }
#undef RING_LDS_DONE
#undef RING_FENCE

    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::G) : "memory");
    if constexpr (HEAD) {
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        float part = 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) part += fmaxf(acc[nt][g][i], 0.f) * hw2[nt][i];
        part += __shfl_xor(part, 16);
        part += __shfl_xor(part, 32);
        const int xp = g * 16 + fr;
        float x0f, x1f, x2f;
        if (op.x_f16) {
          const half_t* xl = (const half_t*)epi;
          x0f = (float)xl[xp];
          x1f = (float)xl[32 + xp];
          x2f = (float)xl[64 + xp];
        } else {
          const float* xl = (const float*)epi;
          x0f = xl[xp];
          x1f = xl[32 + xp];
          x2f = xl[64 + xp];
        }
        const float z = (x0f + x1f + x2f) / 3.f + (part + op.head_b);
        const float il = 1.f / (1.f + expf(-z));
        float* dst = (ovalid[g] && fg == 0) ? op.illu + prow + g * 16 + fr : (float*)(g_ring_sink + tid);
        *dst = il;
      }
    } else {
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        float* dg = ovalid[g] ? (float*)op.out + prow * ocs + op.out_coff + (g * 16 + fr) * ocs + fg * 4
                              : (float*)(g_ring_sink + tid * 16);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          f32x4 v = acc[nt][g];
          if constexpr (RES && K::RESPRE)
            v += *(const f32x4*)(epi + (g * 16 + fr) * NB * 4 + (((nt * 4 + fg) ^ ring32_res_swz<NB / 4>(fr)) * 16));
          if constexpr (K::RELU) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.f);
          }
          if constexpr (RES && !K::RESPRE)
            v += *(const f32x4*)(epi + (g * 16 + fr) * NB * 4 + (((nt * 4 + fg) ^ ring32_res_swz<NB / 4>(fr)) * 16));
          if constexpr (K::POOL) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (ovalid[g]) pool[nt][i] += v[i];
          }
          *(f32x4*)(dg + nt * 16) = v;
        }
      }
    }
    // per-image channel sums, flushed at the last compute step of every unit
    // (a unit lies in one image): one no-return atomic per (tile, channel quad)
    if constexpr (K::POOL) {
      if (s == a.steps - 2) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v = pool[nt][i];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if (fr == 0) pool_add(op.pool, (size_t)cc.b * op.N + nt * 16 + fg * 4 + i, v);
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

// row bands: minimise the makespan ceil(units / grid) * steps per unit
static void ring_bands(RingArgs& a, const ConvOp& op, int grid) {
  const int per_band = op.B * a.nstrips;
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
}

template <int MODE, int C, int NB, int FL>
static int launch_ring_cfg(const ConvOp& op, hipStream_t st) {
  using K = RingCfg<MODE, C, NB, FL>;
  auto kern = conv_ring_kernel<MODE, C, NB, FL>;
  static int occ = 0;
  if (!occ) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS);
    if (e != hipSuccess) return (int)e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)kern, K::THREADS, K::LDS);
    if (e != hipSuccess) return (int)e;
    if (occ < 1) occ = 1;
  }
  RingArgs a;
  a.op = op;
  a.nstrips = cdiv(op.Wo, K::TW);
  const int grid = ring_cus() * occ;  // a multiple of 8 (XCD-contiguous unit order)
  ring_bands(a, op, grid);
  int g = std::min(grid, cdiv(a.nunits, 8) * 8);
  g = std::max(8, g / 8 * 8);
  hipLaunchKernelGGL(kern, dim3(g), dim3(K::THREADS), K::LDS, st, a);
  return (int)hipGetLastError();
}

template <int MODE, int NB, int FL>
static int launch_ring32_cfg(const ConvOp& op, hipStream_t st) {
  using K = Ring32Cfg<MODE, NB, FL>;
  auto kern = conv_ring32_kernel<MODE, NB, FL>;
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
  a.nstrips = cdiv(op.Wo, 32);
  ring_bands(a, op, ring_cus() * occ);
  int g = std::min(ring_cus() * occ, cdiv(a.nunits, 8) * 8);
  g = std::max(8, g / 8 * 8);
  hipLaunchKernelGGL(kern, dim3(g), dim3(256), K::LDS, st, a);
  return (int)hipGetLastError();
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

// plain 3x3 segment reading C channels at 16-byte granularity
static bool ring_seg_ok(const ConvSeg& s) {
  return s.kh == 3 && s.kw == 3 && s.dil == 1 && s.pad == 1 && s.pre == kPreNone && s.kbase == 0 &&
         (s.C == 32 || s.C == 64) && s.cs % 8 == 0 && s.coff % 8 == 0 && (uintptr_t)s.src % 16 == 0;
}

template <int MODE, int C, int NB, int FL>
static int ring_relu(const ConvOp& op, hipStream_t st) {
  // timing ablations of the plain 32/64-channel programs (UPR_RING_ABL = 1 no DMA, 2 no MFMA)
  static const int abl = [] { const char* e = getenv("UPR_RING_ABL"); return e ? atoi(e) : 0; }();
  if constexpr (MODE == kRingConv && (FL & ~(kRingWide | kRingOcc3)) == 0) {
    if (abl == 1 && op.relu) return launch_ring_cfg<MODE, C, NB, FL | kRingRelu | kRingAblDma>(op, st);
    if (abl == 2 && op.relu) return launch_ring_cfg<MODE, C, NB, FL | kRingRelu | kRingAblMma>(op, st);
  }
  return op.relu ? launch_ring_cfg<MODE, C, NB, FL | kRingRelu>(op, st) : launch_ring_cfg<MODE, C, NB, FL>(op, st);
}

// fp16 only; kErrUnsupported for every op this kernel does not take
int launch_conv_ring(const ConvOp& op, hipStream_t st) {
  if (op.Ho < 4 || op.Wo < 16) return kErrUnsupported;
  if (op.out2 && op.nseg != 2) return kErrUnsupported;  // fused PreAct output: enc1.conv2 program only
  if (op.out32) {
    // fp32 output (training autocast convs): plain single-segment programs without
    // fp16 residuals; an fp32 res32 (an accumulated input gradient) is added in the epilogue
    if (op.res1 || op.res2 || op.out2 || op.nseg != 1 || op.store != kStoreNHWC) return kErrUnsupported;
    if (op.res32 && ((uintptr_t)op.res32 % 16 || op.res32_cs % 4)) return kErrUnsupported;
    if (op.img_bias || op.pool || op.scale || op.Kpad % 8 || (uintptr_t)op.out32 % 16 || op.out32_cs % 4 ||
        op.out32_coff % 4)
      return kErrUnsupported;
    const ConvSeg& s = op.seg[0];
    if (!ring_seg_ok(s)) return kErrUnsupported;
    if (s.stride == 2) {
      if (s.C != 32 || op.N != 64 || s.Hin != 2 * op.Ho || s.Win != 2 * op.Wo) return kErrUnsupported;
      return ring_relu<kRingS2, 32, 64, kRingOut32>(op, st);
    }
    if (s.stride != 1 || s.Hin != op.Ho || s.Win != op.Wo) return kErrUnsupported;
    if (op.res32) {
      // (32-pixel strips: the 64-pixel program with the res32 loads spilled)
      if (s.C == 32 && op.N == 32) return ring_relu<kRingConv, 32, 32, kRingOut32 | kRingR32>(op, st);
      return kErrUnsupported;
    }
    if (s.C == 32 && op.N == 32)
      return op.Wo >= 48 ? ring_relu<kRingConv, 32, 32, kRingWide | kRingOut32>(op, st)
                                        : ring_relu<kRingConv, 32, 32, kRingOut32>(op, st);
    if (s.C == 32 && op.N == 64) return ring_relu<kRingConv, 32, 64, kRingOut32>(op, st);
    if (s.C == 64 && op.N == 64) return ring_relu<kRingConv, 64, 64, kRingOut32>(op, st);
    return kErrUnsupported;
  }
  if (ring_fam_program(op)) return launch_ring_cfg<kRingFam, 32, 32, 0>(op, st);
  if (op.res1 || op.img_bias || op.pool || op.scale || op.Kpad % 8) return kErrUnsupported;
  const ConvSeg& s = op.seg[0];
  if (!ring_seg_ok(s)) return kErrUnsupported;
  if (op.store == kStoreHeadIllu) {
    if (op.nseg != 1 || s.stride != 1 || s.Hin != op.Ho || s.Win != op.Wo) return kErrUnsupported;
    if (op.N != 32 || s.C != 32 || op.res2 || op.illu_f16 || op.Wo % 8) return kErrUnsupported;
    return launch_ring_cfg<kRingHead, 32, 32, kRingWide>(op, st);
  }
  if (op.store != kStoreNHWC || op.out_cs % 4 || op.out_coff % 4) return kErrUnsupported;
  if (op.res2 && op.res2_cs % 4) return kErrUnsupported;
  const bool res = op.res2 != nullptr;
  if (s.stride == 2) {
    // enc1.conv1: 3x3 s2, 32 -> 64
    if (op.nseg != 1 || res || s.C != 32 || op.N != 64) return kErrUnsupported;
    if (s.Hin != 2 * op.Ho || s.Win != 2 * op.Wo) return kErrUnsupported;
    return ring_relu<kRingS2, 32, 64, 0>(op, st);
  }
  if (s.stride != 1 || s.Hin != op.Ho || s.Win != op.Wo) return kErrUnsupported;
  if (op.nseg == 2) {
    // enc1.conv2 + projecting shortcut: 3x3 64 -> 64 and a 1x1 s2 segment over 32 channels
    const ConvSeg& q = op.seg[1];
    if (s.C != 64 || op.N != 64 || res) return kErrUnsupported;
    if (q.kh != 1 || q.kw != 1 || q.stride != 2 || q.pad != 0 || q.pre != kPreNone || q.C != 32 || q.kbase != 576)
      return kErrUnsupported;
    if (q.Hin != 2 * op.Ho || q.Win != 2 * op.Wo || q.cs % 8 || q.coff % 8 || (uintptr_t)q.src % 16 || op.Kpad != 608)
      return kErrUnsupported;
    if (op.out2) return ring_relu<kRingConv, 64, 64, kRingSc | kRingOut2>(op, st);
    return ring_relu<kRingConv, 64, 64, kRingSc>(op, st);
  }
  if (op.nseg != 1) return kErrUnsupported;
  if (s.C == 32 && op.N == 32) {
    // 64-pixel strips for the plain conv only: with the residual landing zone
    // (4 KB per wave) they measured slower (dec1.conv.3 0.301 -> 0.308 ms)
    if (res) return ring_relu<kRingConv, 32, 32, kRingRes>(op, st);
    if (op.Wo >= 48) return ring_relu<kRingConv, 32, 32, kRingWide>(op, st);
    return ring_relu<kRingConv, 32, 32, kRingOcc3>(op, st);
  }
  // (64-pixel strips do not fit here: a 32 -> 64 filter in registers spills, the
  // 64 -> 64 ring + LDS filter needs 209 KB)
  if (s.C == 32 && op.N == 64) return res ? ring_relu<kRingConv, 32, 64, kRingRes>(op, st) : ring_relu<kRingConv, 32, 64, 0>(op, st);
  if (s.C == 64 && op.N == 64) return res ? ring_relu<kRingConv, 64, 64, kRingRes>(op, st) : ring_relu<kRingConv, 64, 64, 0>(op, st);
  return kErrUnsupported;
}

template <int MODE, int NB, int FL>
static int ring32_relu(const ConvOp& op, hipStream_t st) {
  return op.relu ? launch_ring32_cfg<MODE, NB, FL | kRingRelu>(op, st) : launch_ring32_cfg<MODE, NB, FL>(op, st);
}

// fp32: stride-1 3x3 over 32 channels (-> 32 / 64, head), and the split
// EnhancedFAM fusion's 3x3 parts (N 32: dilation 1 or 2, a pre-ReLU residual,
// per-image pool sums); kErrUnsupported otherwise
int launch_conv_ring32(const ConvOp& op, hipStream_t st) {
  if (op.Ho < 4 || op.Wo < 16) return kErrUnsupported;
  const ConvSeg& s = op.seg[0];
  if (op.nseg == 3) {
    // FAM fusion, h3 + x + maxpool3(x) part: conv(h3) + W1 x + W2 maxpool3(x) + bias (no ReLU)
    const ConvSeg& x1 = op.seg[1];
    const ConvSeg& x2 = op.seg[2];
    if (op.Kpad != 352 || op.N != 32 || op.store != kStoreNHWC || op.relu || op.pool || op.res1 || op.res2 ||
        op.img_bias || op.scale || op.out_cs % 4 || op.out_coff % 4)
      return kErrUnsupported;
    if (!ring_seg_ok(s) || s.C != 32 || s.stride != 1 || s.Hin != op.Ho || s.Win != op.Wo || s.cs % 4 || s.coff % 4)
      return kErrUnsupported;
    for (const ConvSeg* q : {&x1, &x2})
      if (q->kh != 1 || q->kw != 1 || q->stride != 1 || q->pad != 0 || q->C != 32 || q->Hin != op.Ho ||
          q->Win != op.Wo || q->src != x1.src || q->cs != x1.cs || q->coff != x1.coff)
        return kErrUnsupported;
    if (x1.pre != kPreNone || x2.pre != kPreMaxPool3 || x1.kbase != 288 || x2.kbase != 320 || x1.cs % 4 ||
        x1.coff % 4 || (uintptr_t)x1.src % 16)
      return kErrUnsupported;
    return launch_ring32_cfg<kRingConv, 32, kRingXPool>(op, st);
  }
  if (op.nseg != 1) return kErrUnsupported;
  if (op.img_bias || op.scale || op.Kpad != 288 || (op.res1 && op.res2)) return kErrUnsupported;
  if (s.C != 32 || s.stride != 1 || s.Hin != op.Ho || s.Win != op.Wo || s.cs % 4 || s.coff % 4) return kErrUnsupported;
  if (s.kh == 3 && s.kw == 3 && s.dil == 2 && s.pad == 2 && s.pre == kPreNone && s.kbase == 0 && s.cs % 8 == 0 &&
      s.coff % 8 == 0 && (uintptr_t)s.src % 16 == 0) {
    // FAM fusion, h4 part: relu(conv_d2(h4) + res1) (+ pool sums)
    if (op.store != kStoreNHWC || op.N != 32 || op.res2 || !op.res1 || !op.relu || op.res1_cs % 4 || op.out_cs % 4 ||
        op.out_coff % 4)
      return kErrUnsupported;
    return op.pool ? launch_ring32_cfg<kRingConv, 32, kRingDil2 | kRingRes | kRingResPre | kRingRelu | kRingPool>(op, st)
                   : launch_ring32_cfg<kRingConv, 32, kRingDil2 | kRingRes | kRingResPre | kRingRelu>(op, st);
  }
  if (!ring_seg_ok(s)) return kErrUnsupported;
  if (op.res1) {
    // FAM fusion, h3 part: conv(h3) + res1 (no ReLU)
    if (op.store != kStoreNHWC || op.N != 32 || op.relu || op.pool || op.res1_cs % 4 || op.out_cs % 4 || op.out_coff % 4)
      return kErrUnsupported;
    return launch_ring32_cfg<kRingConv, 32, kRingRes | kRingResPre>(op, st);
  }
  if (op.pool) return kErrUnsupported;
  if (op.store == kStoreHeadIllu) {
    if (op.N != 32 || op.res2 || op.illu_f16 || op.Wo % 8) return kErrUnsupported;
    return launch_ring32_cfg<kRingHead, 32, 0>(op, st);
  }
  if (op.store != kStoreNHWC || op.out_cs % 4 || op.out_coff % 4) return kErrUnsupported;
  if (op.res2 && op.res2_cs % 4) return kErrUnsupported;
  const bool res = op.res2 != nullptr;
  if (op.N == 32) return res ? ring32_relu<kRingConv, 32, kRingRes>(op, st) : ring32_relu<kRingConv, 32, 0>(op, st);
  if (op.N == 64) return res ? ring32_relu<kRingConv, 64, kRingRes>(op, st) : ring32_relu<kRingConv, 64, 0>(op, st);
  return kErrUnsupported;
}

}  // namespace upr
