// Halo-tiled direct convolution for gfx950 (stride-1 3x3 / 1x1 segments, plus
// the 1x1 stride-2 ResBlock shortcut and the EnhancedFAM max-pool branch).
//
// The generic implicit-GEMM kernel (conv.hip) re-reads the A operand once per
// filter tap.  Here a block owns a TH x 32 output-pixel tile of one image and
// stages, per K step (= one segment x 32-channel chunk), the input REGION the
// tile needs (tile + (k-1)*dil halo) into LDS once; every tap then reads its A
// fragments from LDS at shifted offsets.  The step's weights for all taps sit
// next to it (staged once per block when the whole K is one step).
//
// * Step kinds (compile-time region geometry, so every index division is by a
//   constant):
//     1x1        region = tile
//     3x3        region = tile + 1-pixel halo
//     3x3 d2     region = tile + 2-pixel halo
//     pair       EnhancedFAM branch1 + branch2 (models/model.py:29-32,66-69):
//                x (1x1) and maxpool3x3(x) (1x1) from ONE region with a 1-pixel
//                -inf halo — tap 0 reads the centre, tap 1 the 3x3 max
//     1x1 s2     ResBlock projecting shortcut (model.py:114-118): region =
//                every other input pixel of the tile's 2x footprint
// * An op's segments form a PROGRAM: up to three phases of one kind each
//   (e.g. FAM fusion = [3x3, 3x3 d2, pair]; ResBlock conv2 = [3x3, 1x1 s2]);
//   the kernel is instantiated per program, so each phase is straight-line
//   code and only one kind's registers are live at a time.
// * Blocks loop over tiles (persistent grid, sized to co-resident blocks).
//   The NEXT step's region (possibly of the next tile) is loaded into
//   registers while the current step's MFMAs run; the pre-activation
//   prologue (BN + ReLU) is applied when the registers are written to LDS.
// * LDS pixel / weight-row strides make the 16-byte fragment reads of the MFMA
//   operands bank-conflict free (fp32: 10 chunks per row with the
//   k-permutation {g, g+4}; fp16: 6 chunks per row).
// * Epilogue goes through LDS: residual chunks are requested before the last
//   step's MFMAs, and every global store is a full 16-byte chunk of
//   consecutive channels (NHWC rows are contiguous; the ConvTranspose 2x2
//   pixel shuffle keeps each chunk inside one output pixel).
//
// MFMA fragments: lane (r = lane&15, g = lane>>4) owns 8 channels of pixel /
// weight row r: fp16 [8g, 8g+8) -> one v_mfma_f32_16x16x32_f16;
// fp32 [4g, 4g+4) u [16+4g, 16+4g+4) -> 8 x v_mfma_f32_16x16x4_f32 (exact fp32).
// The same channel permutation is applied to A and B, so the sum is unchanged.
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "upr_common.h"

namespace upr {

typedef float f32x4_h __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8_h __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float hto_f(float v) { return v; }
__device__ __forceinline__ float hto_f(half_t v) { return (float)v; }
template <typename T> __device__ __forceinline__ T hfrom_f(float v);
template <> __device__ __forceinline__ float hfrom_f<float>(float v) { return v; }
template <> __device__ __forceinline__ half_t hfrom_f<half_t>(float v) { return (half_t)v; }

constexpr int HALO_TW = 32;
constexpr int HALO_MAXSTEPS = 64;

// ---- step kinds and programs ------------------------------------------------
enum HaloKind : int { kK1x1 = 0, kK3x3 = 1, kK3x3D2 = 2, kKPair = 3, kK1x1S2 = 4, kK3x3S2 = 5 };

// Region geometry per kind, for a TH x 32 output tile whose origin is (oy0, ox0):
//   region pixel (hy, hx), hy < kind_hh, hx < kind_hw, reads input
//   (S*oy0 - PAD + SS*hy, S*ox0 - PAD + SS*hx) and sits at LDS pixel
//   hy*kind_lw + hx, or, for 3x3 s2, column-parity de-interleaved at
//   hy*66 + (hx&1)*33 + (hx>>1) so that a tap's 16 A rows (output columns
//   px..px+15 -> input columns 2px+c) are 16 CONSECUTIVE LDS pixels.
constexpr int kind_ext(int k) { return k == kK3x3 || k == kKPair ? 2 : (k == kK3x3D2 ? 4 : 0); }
constexpr int kind_hh(int k, int th) { return k == kK3x3S2 ? 2 * th + 1 : th + kind_ext(k); }
constexpr int kind_hw(int k) { return k == kK3x3S2 ? 2 * HALO_TW + 1 : HALO_TW + kind_ext(k); }
constexpr int kind_lw(int k) { return k == kK3x3S2 ? 2 * HALO_TW + 2 : kind_hw(k); }
constexpr int kind_s(int k) { return k == kK1x1S2 || k == kK3x3S2 ? 2 : 1; }
constexpr int kind_ss(int k) { return k == kK1x1S2 ? 2 : 1; }
constexpr int kind_pad(int k) { return k == kK3x3S2 ? 1 : kind_ext(k) / 2; }
constexpr int kind_taps(int k) { return k == kK3x3 || k == kK3x3D2 || k == kK3x3S2 ? 9 : (k == kKPair ? 2 : 1); }
constexpr int kind_lds_pix(int k, int hy, int hx) {
  return k == kK3x3S2 ? hy * kind_lw(k) + (hx & 1) * (HALO_TW + 1) + (hx >> 1) : hy * kind_lw(k) + hx;
}
constexpr int cmax3(int a, int b, int c) { return a > b ? (a > c ? a : c) : (b > c ? b : c); }
// program = up to 3 phases, kind+1 per 3-bit digit (0 terminates)
constexpr int prog1(int a) { return a + 1; }
constexpr int prog2(int a, int b) { return (a + 1) | (b + 1) << 3; }
constexpr int prog3(int a, int b, int c) { return (a + 1) | (b + 1) << 3 | (c + 1) << 6; }
constexpr int prog_len(int p) { return p == 0 ? 0 : 1 + prog_len(p >> 3); }
constexpr int prog_kind(int p, int i) { return ((p >> (3 * i)) & 7) - 1; }

// host-built step table: step -> (segment, 32-channel chunk); phase p = steps [end[p-1], end[p])
struct HaloSteps {
  int n;
  int phase_end[3];
  int wtaps;  // taps over all steps (weights of the whole program = wtaps x NB rows)
  int res;    // 1: the whole program's weights stay resident in LDS (set per launch)
  unsigned char si[HALO_MAXSTEPS];
  unsigned char cq[HALO_MAXSTEPS];
  unsigned short wtap0[HALO_MAXSTEPS];  // first tap of each step in the resident weight image
};

// The whole kernel argument.  The kernel reads it through the kernarg segment
// pointer: indexing op.seg[] / hs.si[] with a runtime step then compiles to
// scalar loads, instead of the compiler copying the by-value argument to
// scratch to make it addressable.
struct HaloArgs {
  ConvOp op;
  HaloSteps hs;
  int tiles_x, tiles_y, ntiles, region_bytes;
  // experiments (UPR_HALO_SCHED="flags,n"; timing only, results wrong for 4..64):
  // 1 setprio / 2 start stagger (n x s_sleep(127)) for the grid's 2nd half,
  // 4 no staging, 8 no epilogue, 16 no LDS stores, 32 no prefetch loads, 64 no post-staging barrier
  int sched;
};

template <typename T, int NB, int TH>
struct HaloCfg {
  static constexpr int EPC = 16 / sizeof(T);   // elements per 16-byte chunk
  static constexpr int CCH = 32 / EPC;         // chunks per 32-channel slice
  static constexpr int PSTR = sizeof(T) == 4 ? 40 : 48;  // row stride (elements): 10 / 6 chunks
  static constexpr int CSTR = NB + 4;          // fp32 epilogue staging stride
  static constexpr int EPI_BYTES = TH * HALO_TW * CSTR * 4;
  static constexpr int CHN = NB / EPC;         // epilogue chunks per pixel
  static constexpr int PPP = 256 / CHN;        // epilogue pixels per pass
  static constexpr int PASSES = TH * HALO_TW / PPP;
  static constexpr int pf_of(int k) { return (kind_hh(k, TH) * kind_hw(k) * CCH + 255) / 256; }
  static constexpr int region_of(int k) { return kind_hh(k, TH) * kind_lw(k) * PSTR * (int)sizeof(T); }
};

template <typename T, int NB, int TH, int PROG>
struct ProgCfg {
  static constexpr int NPH = prog_len(PROG);
  static constexpr int K0 = prog_kind(PROG, 0);
  static constexpr int K1 = NPH > 1 ? prog_kind(PROG, 1) : K0;
  static constexpr int K2 = NPH > 2 ? prog_kind(PROG, 2) : K0;
  using C = HaloCfg<T, NB, TH>;
  static constexpr int PF = cmax3(C::pf_of(K0), C::pf_of(K1), C::pf_of(K2));
  static constexpr int REGION = cmax3(C::region_of(K0), C::region_of(K1), C::region_of(K2));
  static constexpr int MAXTAPS = cmax3(kind_taps(K0), kind_taps(K1), kind_taps(K2));
  static constexpr int PW = (MAXTAPS * NB * HaloCfg<T, NB, TH>::CCH + 255) / 256;  // weight chunks per thread
};

// Weight rows in LDS are unpadded (32 channels) with the 16-byte chunk index
// XOR-swizzled by the row: fp16 c ^ ((row >> 1) & 3), fp32 c ^ (row & 7).  B
// fragment reads start at rows that are multiples of 16, so the swizzle is a
// per-lane constant (of fr); reads and the staging writes are bank-conflict
// free (checked against the ds_read_b128 / ds_write_b128 lane groups).
template <typename T>
__device__ __forceinline__ int bswz(int row) { return sizeof(T) == 2 ? ((row >> 1) & 3) : (row & 7); }

// Region of one step -> registers.  Every kind writes EVERY pf[] entry at a
// constant index: when code paths write different subsets, the compiler merges
// their stores through a phi'd address and demotes pf[] to scratch (each
// prefetch then waits on vmcnt(0)).
template <typename T, int NB, int TH, int KIND, int PFN>
__device__ __forceinline__ void halo_load(uint4 (&pf)[PFN], const ConvSeg& sg, int b, int oy0, int ox0, int c0,
                                          int tid) {
  using C = HaloCfg<T, NB, TH>;
  constexpr int HW = kind_hw(KIND), HH = kind_hh(KIND, TH), NCH = HH * HW * C::CCH;
  constexpr int PAD = kind_pad(KIND), S = kind_s(KIND), SS = kind_ss(KIND);
  constexpr unsigned FILL = KIND != kKPair ? 0u : (sizeof(T) == 2 ? 0xFC00FC00u : 0xFF800000u);  // -inf
  // opaque copy of tid: stops the per-entry offsets (tile-invariant) from being
  // hoisted out of the tile loop and held in registers for every step kind
  asm volatile("" : "+v"(tid));
  // wave-uniform 64-bit base of the region's top-left input pixel (may point
  // before the image; only in-bounds offsets are dereferenced) + per-lane
  // 32-bit byte offsets: the loads use the SGPR-base form, no 64-bit VALU math
  const int iy0 = S * oy0 - PAD, ix0 = S * ox0 - PAD;
  const char* rb = (const char*)((const T*)sg.src + (size_t)b * sg.Hin * sg.Win * sg.cs + sg.coff + c0) +
                   ((long long)iy0 * sg.Win + ix0) * sg.cs * (long long)sizeof(T);
  const unsigned rstride = (unsigned)(SS * sg.Win * sg.cs * (int)sizeof(T));  // bytes per region row
  const unsigned pstride = (unsigned)(SS * sg.cs * (int)sizeof(T));           // bytes per region column
  // interior tiles (uniform): the whole region is inside the image, no bounds checks
  const bool interior = iy0 >= 0 && iy0 + SS * (HH - 1) < sg.Hin && ix0 >= 0 && ix0 + SS * (HW - 1) < sg.Win;
#pragma unroll
  for (int j = 0; j < PFN; ++j) {
    const unsigned q = (unsigned)tid + j * 256u;
    uint4 v = make_uint4(FILL, FILL, FILL, FILL);
    if (j * 256 < NCH) {
      const unsigned px = q / C::CCH, ch = q % C::CCH;
      const unsigned hy = px / HW, hx = px % HW;
      const unsigned off = hy * rstride + hx * pstride + ch * 16u;
      bool ok = (j + 1) * 256 <= NCH || q < (unsigned)NCH;
      if (!interior) {
        const int iy = iy0 + SS * (int)hy, ix = ix0 + SS * (int)hx;
        ok = ok && iy >= 0 && iy < sg.Hin && ix >= 0 && ix < sg.Win;
      }
      if (ok) v = *(const uint4*)(rb + off);
    }
    pf[j] = v;
  }
}

template <typename T, int NB, int TH, int KIND, int PFN>
__device__ __forceinline__ void halo_store(const uint4 (&pf)[PFN], const ConvSeg& sg, int oy0, int ox0, int c0,
                                           int tid, T* halo) {
  using C = HaloCfg<T, NB, TH>;
  constexpr int HW = kind_hw(KIND), HH = kind_hh(KIND, TH), NCH = HH * HW * C::CCH;
  constexpr int PAD = kind_pad(KIND), S = kind_s(KIND), SS = kind_ss(KIND);
  const bool aff = KIND != kKPair && sg.pre == kPreAffineRelu;
  asm volatile("" : "+v"(tid));  // see halo_load
#pragma unroll
  for (int j = 0; j < PFN; ++j) {
    const unsigned q = (unsigned)tid + j * 256u;
    if (j * 256 < NCH && ((j + 1) * 256 <= NCH || q < (unsigned)NCH)) {
      const unsigned px = q / C::CCH, ch = q % C::CCH;
      uint4 v = pf[j];
      const unsigned hy = px / HW, hx = px % HW;
      if (aff) {
        const int iy = S * oy0 - PAD + SS * (int)hy, ix = S * ox0 - PAD + SS * (int)hx;
        if (iy >= 0 && iy < sg.Hin && ix >= 0 && ix < sg.Win) {  // zero padding stays zero
          const int cb = c0 + ch * C::EPC;
          T* vv = (T*)&v;
#pragma unroll
          for (int e = 0; e < C::EPC; ++e)
            vv[e] = hfrom_f<T>(fmaxf(hto_f(vv[e]) * sg.pre_scale[cb + e] + sg.pre_shift[cb + e], 0.f));
        }
      }
      *(uint4*)(halo + kind_lds_pix(KIND, (int)hy, (int)hx) * C::PSTR + ch * C::EPC) = v;
    }
  }
}

// Weights of one step (all taps x NB rows x 32 channels) -> registers; same
// every-entry rule as halo_load.  Pair: tap t is segment si + t (both 1x1).
template <typename T, int NB, int TH, int KIND, int PWN>
__device__ __forceinline__ void wts_load(uint4 (&pw)[PWN], const ConvOp& op, int si, int c0, int n0, int tid) {
  using C = HaloCfg<T, NB, TH>;
  constexpr int NBQ = kind_taps(KIND) * NB * C::CCH;
  asm volatile("" : "+v"(tid));  // see halo_load
  // uniform base (row n0, this segment's k offset, channel chunk c0) + 32-bit offsets
  const ConvSeg& s0 = op.seg[si];
  const char* wb = (const char*)((const T*)op.W + (size_t)n0 * op.Kpad + s0.kbase + c0);
  const unsigned rowb = (unsigned)(op.Kpad * (int)sizeof(T));
  const unsigned tapb = KIND == kKPair ? (unsigned)((op.seg[si + 1].kbase - s0.kbase) * (int)sizeof(T))
                                       : (unsigned)(s0.C * (int)sizeof(T));
#pragma unroll
  for (int j = 0; j < PWN; ++j) {
    const unsigned q = (unsigned)tid + j * 256u;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (j * 256 < NBQ && ((j + 1) * 256 <= NBQ || q < (unsigned)NBQ)) {
      const unsigned row = q / C::CCH, ch = q % C::CCH;  // row = tap*NB + n
      const unsigned tap = row / NB, n = row % NB;
      v = *(const uint4*)(wb + (n * rowb + tap * tapb + ch * 16u));
    }
    pw[j] = v;
  }
}

template <typename T, int NB, int TH, int KIND, int PWN>
__device__ __forceinline__ void wts_store(const uint4 (&pw)[PWN], int tid, T* Bs) {
  using C = HaloCfg<T, NB, TH>;
  constexpr int NBQ = kind_taps(KIND) * NB * C::CCH;
  asm volatile("" : "+v"(tid));
#pragma unroll
  for (int j = 0; j < PWN; ++j) {
    const unsigned q = (unsigned)tid + j * 256u;
    if (j * 256 < NBQ && ((j + 1) * 256 <= NBQ || q < (unsigned)NBQ)) {
      const unsigned row = q / C::CCH, ch = q % C::CCH;
      *(uint4*)(Bs + row * 32 + (ch ^ (unsigned)bswz<T>((int)row)) * C::EPC) = pw[j];
    }
  }
}

// A fragments of one M tile (16 pixels starting at region pixel `pix`)
template <typename T, int PSTR>
struct Frag;
template <int PSTR>
struct Frag<half_t, PSTR> {
  f16x8_h v;
  __device__ __forceinline__ void ld(const half_t* s, int pix, int fg) { v = *(const f16x8_h*)(s + pix * PSTR + fg * 8); }
  // weight row (row = 16-aligned base + fr) of the swizzled B image
  __device__ __forceinline__ void ldb(const half_t* s, int row, int fr, int fg) {
    v = *(const f16x8_h*)(s + row * 32 + ((fg ^ bswz<half_t>(fr)) * 8));
  }
  __device__ __forceinline__ void max_with(const Frag& o) { v = __builtin_elementwise_max(v, o.v); }
};
template <int PSTR>
struct Frag<float, PSTR> {
  f32x4_h v[2];
  __device__ __forceinline__ void ld(const float* s, int pix, int fg) {
    const float* p = s + pix * PSTR + fg * 4;
    v[0] = *(const f32x4_h*)p;
    v[1] = *(const f32x4_h*)(p + 16);
  }
  __device__ __forceinline__ void ldb(const float* s, int row, int fr, int fg) {
    v[0] = *(const f32x4_h*)(s + row * 32 + ((fg ^ bswz<float>(fr)) * 4));
    v[1] = *(const f32x4_h*)(s + row * 32 + (((fg + 4) ^ bswz<float>(fr)) * 4));
  }
  __device__ __forceinline__ void max_with(const Frag& o) {
    v[0] = __builtin_elementwise_max(v[0], o.v[0]);
    v[1] = __builtin_elementwise_max(v[1], o.v[1]);
  }
};

template <int MT, int NT, int PSTR>
__device__ __forceinline__ void frag_mma(f32x4_h (&acc)[MT][NT], const Frag<half_t, PSTR> (&af)[MT],
                                         const Frag<half_t, PSTR> (&bf)[NT]) {
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i].v, bf[j].v, acc[i][j], 0, 0, 0);
}
template <int MT, int NT, int PSTR>
__device__ __forceinline__ void frag_mma(f32x4_h (&acc)[MT][NT], const Frag<float, PSTR> (&af)[MT],
                                         const Frag<float, PSTR> (&bf)[NT]) {
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i].v[e >> 2][e & 3], bf[j].v[e >> 2][e & 3], acc[i][j],
                                                        0, 0, 0);
}

// all taps of one step
template <typename T, int NB, int TH, int KIND>
__device__ __forceinline__ void halo_taps(f32x4_h (&acc)[TH / 2][NB / 16], const T* halo, const T* Bs, int wave,
                                          int fr, int fg) {
  using C = HaloCfg<T, NB, TH>;
  constexpr int PSTR = C::PSTR;
  constexpr int RPW = TH / 4;
  constexpr int MT = 2 * RPW;
  constexpr int NT = NB / 16;
  constexpr int LW = kind_lw(KIND);
  using F = Frag<T, PSTR>;
  // LDS pixel of tap (r, c) for output row wave*RPW + (i>>1), column (i&1)*16 + fr
  auto pix = [&](int i, int r, int c) {
    const int orow = wave * RPW + (i >> 1), ocol = (i & 1) * 16 + fr;
    if constexpr (KIND == kK3x3S2)
      return (2 * orow + r) * LW + (c & 1) * (HALO_TW + 1) + (c >> 1) + ocol;
    else
      return (orow + r) * LW + ocol + c;
  };
  if constexpr (KIND == kKPair) {
    F bf[NT], af[MT];
#pragma unroll
    for (int j = 0; j < NT; ++j) bf[j].ldb(Bs, j * 16 + fr, fr, fg);
#pragma unroll
    for (int i = 0; i < MT; ++i) af[i].ld(halo, pix(i, 1, 1), fg);
    frag_mma<MT, NT, PSTR>(acc, af, bf);
#pragma unroll
    for (int j = 0; j < NT; ++j) bf[j].ldb(Bs, NB + j * 16 + fr, fr, fg);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t == 4) continue;  // centre already in af[i]
        F o;
        o.ld(halo, pix(i, t / 3, t % 3), fg);
        af[i].max_with(o);
      }
    }
    frag_mma<MT, NT, PSTR>(acc, af, bf);
  } else {
    constexpr int K = kind_taps(KIND) == 9 ? 3 : 1;
    constexpr int D = KIND == kK3x3D2 ? 2 : 1;
    // two fragment sets: tap t+1's reads are in flight while tap t's MFMAs issue
    F bf[2][NT], af[2][MT];
    auto rd = [&](int tap, F (&a)[MT], F (&b)[NT]) {
      const int r = tap / K, c = tap % K;
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j].ldb(Bs, tap * NB + j * 16 + fr, fr, fg);
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i].ld(halo, pix(i, r * D, c * D), fg);
    };
    // Pinned interleave (sched_group_barrier; masks MFMA 0x8, DS_READ 0x100):
    // each of the next tap's NR reads goes out beside one of this tap's NM MFMAs.
    constexpr int NR = (MT + NT) * (sizeof(T) == 4 ? 2 : 1);
    constexpr int NM = MT * NT * (sizeof(T) == 4 ? 8 : 1);
    constexpr int NI = NR < NM ? NR : NM;
    rd(0, af[0], bf[0]);
    __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
    for (int tap = 0; tap < K * K; ++tap) {
      if (tap + 1 < K * K) rd(tap + 1, af[(tap + 1) & 1], bf[(tap + 1) & 1]);
      frag_mma<MT, NT, PSTR>(acc, af[tap & 1], bf[tap & 1]);
      if (tap + 1 < K * K) {
#pragma unroll
        for (int k = 0; k < NI; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if constexpr (NR > NI) __builtin_amdgcn_sched_group_barrier(0x100, NR - NI, 0);
        if constexpr (NM > NI) __builtin_amdgcn_sched_group_barrier(0x8, NM - NI, 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x8, NM, 0);
      }
    }
  }
}

template <int V>
using IC = std::integral_constant<int, V>;

// OCC = waves per SIMD the register allocation must allow (= co-resident
// 256-thread blocks per CU): at 2 a second block's MFMAs overlap this block's
// staging / epilogue.
template <typename T, int NB, int TH, int OCC, int PROG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void conv_halo_kernel(
    HaloArgs args) {
  const HaloArgs& A = *(const HaloArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  const ConvOp& op = A.op;
  const HaloSteps& hs = A.hs;
  const int tiles_x = A.tiles_x, tiles_y = A.tiles_y, ntiles = A.ntiles, region_bytes = A.region_bytes;
  using C = HaloCfg<T, NB, TH>;
  using P = ProgCfg<T, NB, TH, PROG>;
  constexpr int EPC = C::EPC;
  constexpr int TW = HALO_TW;
  constexpr int RPW = TH / 4;  // tile rows per wave
  constexpr int MT = 2 * RPW;  // 16-pixel M tiles per wave
  constexpr int NT = NB / 16;  // 16-channel N tiles
  constexpr int CHN = C::CHN, PPP = C::PPP, PASSES = C::PASSES;
  // dynamic LDS sized per op on the host: [region | epilogue staging] then weights
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* halo = (T*)smem;
  float* Cs = (float*)smem;
  T* Bs = (T*)(smem + region_bytes);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int nblk_n = op.N / NB;
  const int HWo = op.Ho * op.Wo;
  // at most one residual per op (launch_conv_halo checks): added before (res1) or after (res2) the ReLU
  const T* resp = (const T*)(op.res1 ? op.res1 : op.res2);
  const int res_cs = op.res1 ? op.res1_cs : op.res2_cs;
  const bool res_pre = op.res1 != nullptr;
  const int nsteps = hs.n;
  // weights resident for the whole kernel: the host found LDS room for every
  // step's weights (hs.res), and the block's N slice never changes (tile t has
  // nb = t % nblk_n and the block strides by the grid size, a multiple of
  // nblk_n — launch_halo_cfg guarantees it)
  const bool b_keep = hs.res && gridDim.x % nblk_n == 0;

  auto tile_coords = [&](int tile, int& b, int& oy0, int& ox0, int& n0) {
    int t = tile;
    const int nb = t % nblk_n; t /= nblk_n;
    const int tx = t % tiles_x; t /= tiles_x;
    const int ty = t % tiles_y; t /= tiles_y;
    b = t; oy0 = ty * TH; ox0 = tx * TW; n0 = nb * NB;
  };
  // the next step's region and (unless resident) weights, in registers
  uint4 pf[P::PF];
  uint4 pw[P::PW];
  auto load = [&](auto kc, int step, int tile) {
    constexpr int K = decltype(kc)::value;
    int b, oy0, ox0, n0;
    tile_coords(tile, b, oy0, ox0, n0);
    halo_load<T, NB, TH, K>(pf, op.seg[hs.si[step]], b, oy0, ox0, hs.cq[step] * 32, tid);
    if (!b_keep) wts_load<T, NB, TH, K>(pw, op, hs.si[step], hs.cq[step] * 32, n0, tid);
  };

  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  if (A.sched && blockIdx.x >= gridDim.x / 2) {
    if (A.sched & 1) __builtin_amdgcn_s_setprio(1);
    if (A.sched & 2)
      for (int i = 0; i < (A.sched >> 8); ++i) __builtin_amdgcn_s_sleep(127);
  }
  if (b_keep) {  // every step's weights, staged once per block
    int b, oy0, ox0, n0;
    tile_coords(tile, b, oy0, ox0, n0);
    auto stage_phase = [&](auto kc, int s0, int s1) {
      constexpr int K = decltype(kc)::value;
      for (int st = s0; st < s1; ++st) {
        wts_load<T, NB, TH, K>(pw, op, hs.si[st], hs.cq[st] * 32, n0, tid);
        wts_store<T, NB, TH, K>(pw, tid, Bs + hs.wtap0[st] * NB * 32);
      }
    };
    stage_phase(IC<P::K0>{}, 0, hs.phase_end[0]);
    if constexpr (P::NPH > 1) stage_phase(IC<P::K1>{}, hs.phase_end[0], hs.phase_end[1]);
    if constexpr (P::NPH > 2) stage_phase(IC<P::K2>{}, hs.phase_end[1], hs.phase_end[2]);
  }
  load(IC<P::K0>{}, 0, tile);

  for (; tile < ntiles; tile += gridDim.x) {
    int b, oy0, ox0, n0;
    tile_coords(tile, b, oy0, ox0, n0);

    f32x4_h acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_h{0.f, 0.f, 0.f, 0.f};

    const int ch = tid % CHN;
    const int nb0 = ch * EPC;  // first channel (within the block slice) of this thread in the epilogue
    const bool tile_full = oy0 + TH <= op.Ho && ox0 + TW <= op.Wo;  // uniform: no per-pixel validity checks
    uint4 rr[PASSES];
    float xs[sizeof(T) == 4 ? PASSES : 1][3];  // fp32 residual head: network-input pixels of this tile, prefetched
    int step = 0;
    // one phase: steps [step, pend) of kind K; the step after the phase is of kind KN
    auto phase = [&](auto kc, auto knc, int pend) {
      constexpr int K = decltype(kc)::value;
      // resident weight image of this phase's steps: consecutive, taps(K)*NB rows apart
      const T* bstep = Bs + (b_keep && step < pend ? hs.wtap0[step] * NB * 32 : 0);
      for (; step < pend; ++step, bstep += b_keep ? kind_taps(K) * NB * 32 : 0) {
        const int si = hs.si[step], c0 = hs.cq[step] * 32;
        const ConvSeg& sg = op.seg[si];
        __syncthreads();  // LDS free (previous step's MFMAs / previous tile's epilogue)
        if (!(A.sched & (4 | 16))) {
          halo_store<T, NB, TH, K>(pf, sg, oy0, ox0, c0, tid, halo);
          if (!b_keep) wts_store<T, NB, TH, K>(pw, tid, Bs);
        }
        if (!(A.sched & 64)) __syncthreads();
        {
          // next step: this tile's, or the first of the block's next tile
          int ns = step + 1, nt = tile;
          if (ns == nsteps) { ns = 0; nt = tile + (int)gridDim.x; }
          // the step after a phase is the next phase's first (kind KN) or, after
          // the last phase, the next tile's first (KN == K0): at most 2 call sites
          if (nt < ntiles && !(A.sched & (4 | 32))) {
            if constexpr (K == decltype(knc)::value)
              load(kc, ns, nt);
            else if (ns > 0 && ns < pend)
              load(kc, ns, nt);
            else
              load(knc, ns, nt);
          }
        }
        if (step == nsteps - 1 && resp) {
          // residual chunks of this tile, requested before the last step's MFMAs
          const char* rb = (const char*)(resp + (((size_t)b * op.Ho + oy0) * op.Wo + ox0) * res_cs + n0);
          const unsigned rrow = (unsigned)(op.Wo * res_cs * (int)sizeof(T)), rcol = (unsigned)(res_cs * (int)sizeof(T));
#pragma unroll
          for (int ps = 0; ps < PASSES; ++ps) {
            const unsigned p = (unsigned)tid / CHN + ps * PPP;
            const unsigned off = (p / TW) * rrow + (p % TW) * rcol + (unsigned)nb0 * sizeof(T);
            const bool ok = tile_full || (oy0 + (int)(p / TW) < op.Ho && ox0 + (int)(p % TW) < op.Wo);
            rr[ps] = ok ? *(const uint4*)(rb + off) : make_uint4(0, 0, 0, 0);
          }
        }
        // fp32 (2 blocks/CU) exposes the epilogue's x-read latency; fp16's head runs
        // 3 blocks/CU, where the early loads only cost (measured)
        if constexpr (sizeof(T) == 4) if (step == nsteps - 1 && op.store == kStoreHeadIllu) {
#pragma unroll
          for (int ps = 0; ps < PASSES; ++ps) {
            const int p = tid / CHN + ps * PPP;
            const int oy = oy0 + p / TW, ox = ox0 + p % TW;
            const bool ok = tile_full || (oy < op.Ho && ox < op.Wo);
            const size_t pp = (size_t)b * 3 * HWo + (size_t)oy * op.Wo + ox;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              float xv = 0.f;
              if (ok) xv = op.x_f16 ? (float)((const half_t*)op.x_nchw)[pp + (size_t)c * HWo] : op.x_nchw[pp + (size_t)c * HWo];
              xs[ps][c] = xv;
            }
          }
        }
        halo_taps<T, NB, TH, K>(acc, halo, bstep, wave, fr, fg);
      }
    };
    phase(IC<P::K0>{}, IC<P::K1>{}, hs.phase_end[0]);
    if constexpr (P::NPH > 1) phase(IC<P::K1>{}, IC<P::K2>{}, hs.phase_end[1]);
    if constexpr (P::NPH > 2) phase(IC<P::K2>{}, IC<P::K0>{}, hs.phase_end[2]);

    // ---- epilogue ------------------------------------------------------------
    if (A.sched & 8) {  // experiment: no epilogue (keeps acc alive)
      float z = 0.f;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) z += acc[i][j][0];
      if (z == 12345.f) ((float*)op.out)[tid] = z;
      continue;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int py = wave * RPW + (i >> 1), px0 = (i & 1) * 16 + fg * 4;
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) Cs[(py * TW + px0 + e) * C::CSTR + j * 16 + fr] = acc[i][j][e];
    }
    __syncthreads();

    float bias_v[EPC];
    if (op.bias) {
      const f32x4_h* bp = (const f32x4_h*)(op.bias + n0 + nb0);
#pragma unroll
      for (int e = 0; e < EPC; e += 4) {
        const f32x4_h t4 = bp[e / 4];
        bias_v[e] = t4[0]; bias_v[e + 1] = t4[1]; bias_v[e + 2] = t4[2]; bias_v[e + 3] = t4[3];
      }
    } else {
#pragma unroll
      for (int e = 0; e < EPC; ++e) bias_v[e] = 0.f;
    }
    float psum[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) psum[e] = 0.f;
    // residual-head 1x1 weights in registers: read once, not per pass (the illu
    // stores may alias them as far as the compiler knows)
    float hw_v[EPC];
    if (op.store == kStoreHeadIllu) {
#pragma unroll
      for (int e = 0; e < EPC; ++e) hw_v[e] = op.head_w[nb0 + e];
    }
    T* out = (T*)op.out;
    // uniform tile base + 32-bit per-lane byte offsets (NHWC store)
    char* ob = (char*)(out + (((size_t)b * op.Ho + oy0) * op.Wo + ox0) * op.out_cs + op.out_coff + n0);
    const unsigned orow = (unsigned)(op.Wo * op.out_cs * (int)sizeof(T)), ocol = (unsigned)(op.out_cs * (int)sizeof(T));
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const int p = tid / CHN + ps * PPP;
      const int oy = oy0 + p / TW, ox = ox0 + p % TW;
      const bool valid = tile_full || (oy < op.Ho && ox < op.Wo);
      const size_t m = ((size_t)b * op.Ho + oy) * op.Wo + ox;
      float v[EPC];
      {
        const f32x4_h* cp = (const f32x4_h*)(Cs + p * C::CSTR + nb0);
#pragma unroll
        for (int e = 0; e < EPC; e += 4) {
          const f32x4_h t4 = cp[e / 4];
          v[e] = t4[0] + bias_v[e]; v[e + 1] = t4[1] + bias_v[e + 1];
          v[e + 2] = t4[2] + bias_v[e + 2]; v[e + 3] = t4[3] + bias_v[e + 3];
        }
      }
      if (op.store == kStoreHeadIllu) {
        // residual head (models/model.py:324-328, :351-358); NB == N == 32
        float part = 0.f;
#pragma unroll
        for (int e = 0; e < EPC; ++e) part += fmaxf(v[e], 0.f) * hw_v[e];
#pragma unroll
        for (int s = 1; s < CHN; s <<= 1) part += __shfl_xor(part, s);
        if (ch == 0 && valid) {
          float x0, x1, x2;
          if constexpr (sizeof(T) == 4) {
            x0 = xs[ps][0]; x1 = xs[ps][1]; x2 = xs[ps][2];
          } else {
            const size_t pp = (size_t)oy * op.Wo + ox;
            if (op.x_f16) {
              const half_t* x = (const half_t*)op.x_nchw + (size_t)b * 3 * HWo + pp;
              x0 = (float)x[0]; x1 = (float)x[HWo]; x2 = (float)x[2 * HWo];
            } else {
              const float* x = op.x_nchw + (size_t)b * 3 * HWo + pp;
              x0 = x[0]; x1 = x[HWo]; x2 = x[2 * HWo];
            }
          }
          const float z = (x0 + x1 + x2) / 3.f + (part + op.head_b);
          const float il = 1.f / (1.f + expf(-z));
          if (op.illu_f16) ((half_t*)op.illu)[m] = (half_t)il;
          else op.illu[m] = il;
        }
        continue;
      }
      if (!valid) continue;
      if (op.img_bias) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] += op.img_bias[b * op.N + n0 + nb0 + e];
      }
      if (resp && res_pre) {
        const T* rv = (const T*)&rr[ps];
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] += hto_f(rv[e]);
      }
      if (op.relu) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (resp && !res_pre) {
        const T* rv = (const T*)&rr[ps];
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] += hto_f(rv[e]);
      }
      uint4 o;
      T* ov = (T*)&o;
#pragma unroll
      for (int e = 0; e < EPC; ++e) ov[e] = hfrom_f<T>(v[e]);
      if constexpr (sizeof(T) == 2) {
        if (op.out32) {
          // fp32 output of the fp16 conv (training autocast): the fp16-rounded
          // value (+ res32, fp32), NHWC only (launch_conv_halo checks)
          float* d32 = op.out32 + m * op.out32_cs + op.out32_coff + n0 + nb0;
          const float* r32 = op.res32 ? op.res32 + m * op.res32_cs + n0 + nb0 : nullptr;
#pragma unroll
          for (int e = 0; e < EPC; e += 4) {
            f32x4_h w4 = {hto_f(ov[e]), hto_f(ov[e + 1]), hto_f(ov[e + 2]), hto_f(ov[e + 3])};
            if (r32) w4 += *(const f32x4_h*)(r32 + e);
            if (op.mask16) {
              typedef _Float16 h4m __attribute__((ext_vector_type(4)));
              const h4m mk = *(const h4m*)((const half_t*)op.mask16 + m * op.mask16_cs + n0 + nb0 + e);
#pragma unroll
              for (int q = 0; q < 4; ++q) w4[q] = (float)mk[q] > 0.f ? w4[q] : 0.f;
            }
            if (!op.skip32) *(f32x4_h*)(d32 + e) = w4;
            if (op.out32_h16) {
              typedef _Float16 h4h __attribute__((ext_vector_type(4)));
              *(h4h*)((half_t*)op.out32_h16 + m * op.out32_h16_cs + n0 + nb0 + e) =
                  h4h{(half_t)w4[0], (half_t)w4[1], (half_t)w4[2], (half_t)w4[3]};
            }
          }
          continue;
        }
      }
      if (op.store == kStoreConvT2x2) {
        // ConvTranspose2d(2, 2) pixel shuffle (model.py:167): n = (dy*2+dx)*Cout + co
        const int cout = op.N >> 2;
        const int n = n0 + nb0, q = n / cout, co = n - q * cout;
        const size_t opix = ((size_t)b * 2 * op.Ho + 2 * oy + (q >> 1)) * (2 * op.Wo) + 2 * ox + (q & 1);
        *(uint4*)(out + opix * op.out_cs + op.out_coff + co) = o;
      } else {
        *(uint4*)(ob + ((unsigned)(p / TW) * orow + (unsigned)(p % TW) * ocol + (unsigned)nb0 * sizeof(T))) = o;
      }
#pragma unroll
      for (int e = 0; e < EPC; ++e) psum[e] += hto_f(ov[e]);
    }
    if (op.pool) {
      // per-channel tile sums -> one atomic per channel
      __syncthreads();
#pragma unroll
      for (int e = 0; e < EPC; ++e) Cs[tid * (EPC + 1) + e] = psum[e];
      __syncthreads();
      if (tid < NB) {
        const int cch = tid / EPC, e = tid % EPC;
        float s = 0.f;
        for (int q = cch; q < 256; q += CHN) s += Cs[q * (EPC + 1) + e];
        pool_add(op.pool, (size_t)b * op.N + n0 + tid, s);
      }
    }
  }
}

// ---- host side ------------------------------------------------------------------

template <typename T, int NB, int TH, int OCC, int PROG>
static int launch_halo_cfg(const ConvOp& op, const HaloSteps& hs, hipStream_t st) {
  const int tiles_x = cdiv(op.Wo, HALO_TW), tiles_y = cdiv(op.Ho, TH);
  const int ntiles = op.B * tiles_x * tiles_y * (op.N / NB);
  using C = HaloCfg<T, NB, TH>;
  using P = ProgCfg<T, NB, TH, PROG>;
  // LDS: region (largest over the program's kinds; the epilogue staging reuses
  // it) + weights: one step's (largest tap count) staged per step, or every
  // step's resident for the whole kernel when that costs no co-resident block
  constexpr int region = ((P::REGION > C::EPI_BYTES ? P::REGION : C::EPI_BYTES) + 15) / 16 * 16;
  constexpr int row_bytes = 32 * (int)sizeof(T);  // unpadded, swizzled weight rows
  constexpr int lds_step = region + P::MAXTAPS * NB * row_bytes;
  static_assert(lds_step <= 160 * 1024, "halo LDS budget");
  const int lds_res = region + hs.wtaps * NB * row_bytes;
  static bool attr_set = false;
  static int reg_cap = 0;  // co-resident blocks per CU allowed by registers
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)conv_halo_kernel<T, NB, TH, OCC, PROG>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&reg_cap, (const void*)conv_halo_kernel<T, NB, TH, OCC, PROG>,
                                                     256, 0) != hipSuccess || reg_cap < 1)
      reg_cap = 1;
    attr_set = true;
  }
  auto blocks = [&](int l) { const int c = (160 * 1024) / l; return c < reg_cap ? c : reg_cap; };
  const bool res = lds_res <= 160 * 1024 && blocks(lds_res) >= blocks(lds_step);
  const int lds = res ? lds_res : lds_step;
  // Persistent grid = blocks that are actually co-resident (registers AND LDS);
  // an oversized grid leaves a second, partial wave of blocks (tail).  Speed only.
  int per_cu = blocks(lds);
  if (per_cu < 1) per_cu = 1;
  int grid = 256 * per_cu;
  if (grid > ntiles) grid = ntiles;
  grid -= grid % (op.N / NB);  // a whole number of N slices per grid stride (resident weights)
  HaloArgs args;
  args.op = op;
  args.hs = hs;
  args.hs.res = res ? 1 : 0;
  args.tiles_x = tiles_x;
  args.tiles_y = tiles_y;
  args.ntiles = ntiles;
  args.region_bytes = region;
  args.sched = 0;
  hipLaunchKernelGGL((conv_halo_kernel<T, NB, TH, OCC, PROG>), dim3(grid), dim3(256), lds, st, args);
  return (int)hipGetLastError();
}

template <typename T, int NB, int PROG>
static int launch_halo_prog(const ConvOp& op, const HaloSteps& hs, int th, int occ, hipStream_t st) {
  // stride-2 3x3: a (2*TH+1) x 65 region; only 4-row tiles fit LDS (one block per CU)
  if constexpr (PROG == prog1(kK3x3S2)) {
    (void)th;
    (void)occ;
    return launch_halo_cfg<T, NB, 4, 1, PROG>(op, hs, st);
  } else {
    if (th == 4)
      return occ >= 3 ? launch_halo_cfg<T, NB, 4, 3, PROG>(op, hs, st) : launch_halo_cfg<T, NB, 4, 2, PROG>(op, hs, st);
    return occ >= 2 ? launch_halo_cfg<T, NB, 8, 2, PROG>(op, hs, st) : launch_halo_cfg<T, NB, 8, 1, PROG>(op, hs, st);
  }
}

// the programs instantiated (any other segment mix runs on the generic kernel)
constexpr int kProg3x3 = prog1(kK3x3);
constexpr int kProg1x1 = prog1(kK1x1);
constexpr int kProgD2 = prog1(kK3x3D2);
constexpr int kProgFam = prog3(kK3x3, kK3x3D2, kKPair);  // EnhancedFAM fusion GEMM
constexpr int kProgResS2 = prog2(kK3x3, kK1x1S2);        // ResBlock conv2 + projecting shortcut
constexpr int kProgS2 = prog1(kK3x3S2);                   // ResBlock conv1 (stride 2)

template <typename T, int NB>
static int launch_halo_nb(const ConvOp& op, const HaloSteps& hs, int prog, int th, int occ, hipStream_t st) {
  switch (prog) {
    case kProg3x3: return launch_halo_prog<T, NB, kProg3x3>(op, hs, th, occ, st);
    case kProg1x1: return launch_halo_prog<T, NB, kProg1x1>(op, hs, th, occ, st);
    case kProgD2: return launch_halo_prog<T, NB, kProgD2>(op, hs, th, occ, st);
    case kProgFam: return launch_halo_prog<T, NB, kProgFam>(op, hs, th, occ, st);
    case kProgResS2: return launch_halo_prog<T, NB, kProgResS2>(op, hs, th, occ, st);
    case kProgS2: return launch_halo_prog<T, NB, kProgS2>(op, hs, th, occ, st);
    default: return kErrUnsupported;
  }
}

// Segment kind of the halo kernel, or -1.  `pair` = segment s+1 is the max-pool
// twin of s (same source slice), consumed together.
static int seg_kind(const ConvOp& op, int s, int Ho, int Wo, bool& pair) {
  const ConvSeg& g = op.seg[s];
  pair = false;
  if (g.C % 32 || g.kh != g.kw) return -1;
  if (g.stride == 2) {
    if ((g.Hin - 1) / 2 + 1 != Ho || (g.Win - 1) / 2 + 1 != Wo) return -1;
    if (g.kh == 3 && g.pad == 1 && g.dil == 1) return kK3x3S2;
    if (g.kh != 1 || g.pad != 0 || g.pre != kPreNone) return -1;
    return kK1x1S2;
  }
  if (g.stride != 1 || g.Hin != Ho || g.Win != Wo) return -1;
  if (g.kh == 3) {
    if (g.dil == 1 && g.pad == 1) return kK3x3;
    if (g.dil == 2 && g.pad == 2) return kK3x3D2;
    return -1;
  }
  if (g.kh != 1 || g.pad != 0) return -1;
  if (g.pre == kPreMaxPool3) return -1;  // only as the twin of a plain 1x1
  if (s + 1 < op.nseg) {
    const ConvSeg& h = op.seg[s + 1];
    if (h.pre == kPreMaxPool3 && g.pre == kPreNone && h.kh == 1 && h.kw == 1 && h.stride == 1 && h.pad == 0 &&
        h.src == g.src && h.C == g.C && h.cs == g.cs && h.coff == g.coff && h.Hin == g.Hin && h.Win == g.Win) {
      pair = true;
      return kKPair;
    }
  }
  return kK1x1;
}

// Tile rows / occupancy per program, from per-layer sweeps of the whole forward
// on MI355X (tools/layer_sweep.sh + tools/layer_table.py, bs 32, 512^2):
//   fp32: 4-row tiles at 2 blocks/CU; 8-row tiles for the 1x1 (ConvT) and the
//         FAM fusion program (1 block/CU, all 20 taps of weights resident)
//   fp16: 4-row tiles at 2 blocks/CU for N >= 64 (64-wide N blocks) and the FAM
//         fusion (weights resident); 8-row tiles at 2 blocks/CU for N = 32 and
//         1x1; the residual head 4-row at 3 blocks/CU
// UPR_HALO="<th>,<occ>" overrides (experiments).
static void halo_choice(int dtype, int prog, int store, int N, int& th, int& occ) {
  if (dtype == kF16) {
    th = N >= 64 || prog == kProgFam ? 4 : 8;
    occ = 2;
    if (store == kStoreHeadIllu) { th = 4; occ = 3; }
  } else {
    th = 4;
    occ = 2;
    if (prog == kProg1x1) th = 8;
    if (prog == kProgFam) { th = 8; occ = 1; }
  }
  if (prog == kProgS2) { th = 4; occ = 1; }
}

// Returns kErrUnsupported when the op is not a halo-kernel shape (caller falls back).
int launch_conv_halo(const ConvOp& op, int dtype, hipStream_t st) {
  if (op.Wo < 24 || op.Ho < 8) return kErrUnsupported;
  if (op.out32) {
    // fp32 output (training autocast convs): fp16 kernel, plain NHWC store, no pool / residual-before-ReLU
    if (dtype != kF16 || op.out || op.store != kStoreNHWC || op.pool || op.res1 || op.res2 || op.img_bias ||
        (uintptr_t)op.out32 % 16 || op.out32_cs % 4 || op.out32_coff % 4 || op.N % 4 ||
        (op.res32 && ((uintptr_t)op.res32 % 16 || op.res32_cs % 4)))
      return kErrUnsupported;
  }
  const int elt = dtype == kF16 ? 2 : 4;
  if (op.out && ((op.out_cs * elt) % 16 || (op.out_coff * elt) % 16)) return kErrUnsupported;
  if (op.res1 && (op.res1_cs * elt) % 16) return kErrUnsupported;
  if (op.res2 && (op.res2_cs * elt) % 16) return kErrUnsupported;
  if (op.res1 && op.res2) return kErrUnsupported;
  if (op.store == kStoreHeadIllu && op.N != 32) return kErrUnsupported;
  if (op.store == kStoreConvT2x2 && ((op.N / 4) % 16 || op.pool)) return kErrUnsupported;
  if (op.bias && ((uintptr_t)op.bias % 16)) return kErrUnsupported;
  if (op.scale) return kErrUnsupported;  // the graph folds every scale into the weights
  // step table + program
  HaloSteps hs;
  hs.n = 0;
  hs.wtaps = 0;
  hs.res = 0;
  int kinds[3], nph = 0;
  for (int s = 0; s < op.nseg; ++s) {
    bool pair = false;
    const int k = seg_kind(op, s, op.Ho, op.Wo, pair);
    if (k < 0) return kErrUnsupported;
    if (nph == 0 || kinds[nph - 1] != k) {
      if (nph == 3) return kErrUnsupported;
      if (nph > 0) hs.phase_end[nph - 1] = hs.n;
      kinds[nph++] = k;
    }
    for (int cq = 0; cq < op.seg[s].C / 32; ++cq) {
      if (hs.n == HALO_MAXSTEPS) return kErrUnsupported;
      hs.si[hs.n] = (unsigned char)s;
      hs.cq[hs.n] = (unsigned char)cq;
      hs.wtap0[hs.n] = (unsigned short)hs.wtaps;
      hs.wtaps += kind_taps(k);
      ++hs.n;
    }
    if (pair) ++s;
  }
  if (nph == 0) return kErrUnsupported;
  // stride-2 3x3 only pays for fp16 with few steps (one block per CU; measured)
  if (nph == 1 && kinds[0] == kK3x3S2 && (dtype != kF16 || hs.n > 2)) return kErrUnsupported;
  hs.phase_end[nph - 1] = hs.n;
  for (int p = nph; p < 3; ++p) hs.phase_end[p] = hs.n;
  const int prog = nph == 1 ? prog1(kinds[0]) : (nph == 2 ? prog2(kinds[0], kinds[1]) : prog3(kinds[0], kinds[1], kinds[2]));
  int th, occ;
  halo_choice(dtype, prog, op.store, op.N, th, occ);
  if (dtype == kF16) {
    if (op.N == 32) return launch_halo_nb<half_t, 32>(op, hs, prog, th, occ, st);
    if (op.N % 64 == 0) return launch_halo_nb<half_t, 64>(op, hs, prog, th, occ, st);
  } else {
    if (op.N % 32 == 0) return launch_halo_nb<float, 32>(op, hs, prog, th, occ, st);
  }
  return kErrUnsupported;
}

}  // namespace upr
