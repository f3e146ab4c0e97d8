// conv_hw2_kernel: the fp16 3x3 convs over 256 channels at W 64 (the
// bottleneck ResBlock / PreActResBlock convs and the ASPP dilated branches,
// models/model.py:100-178, :181-251) as TWO independent 256-thread blocks per
// CU, each with <= 80 KiB of LDS.
//
// Why: conv_hwide4_kernel runs one 512-thread block per CU (160 KiB: an 8-row
// ring of 64-channel rows + three 32 KiB B stages).  Its 8 waves meet at one
// barrier per K step, so the two waves of a SIMD stall together (PMC: wait_any
// 0.39-0.40, MFMA busy ~0.65 of the wave lifetime), and nothing overlaps a
// tile's prologue DMA or its epilogue burst.  Here the CU holds two blocks
// whose barriers are unrelated: one wave per SIMD from each, so while one
// block drains its counted DMA wait or its epilogue the other's MFMAs issue.
//
// * Tile: 4 output rows x 64 pixels x 128 channels (the two N halves of a
//   pixel tile are adjacent block ids: their shared A region is an L2 hit);
//   4 waves as 2 (column halves of 32 px) x 2 (64-channel halves): each wave
//   8 x 4 fragments of v_mfma_f32_16x16x32_f16 = 128 accumulators, the
//   per-wave fragment economy of hwide4 (12 ds_read_b128 per 32 MFMAs).
// * K walks 32-channel SLICES (one MFMA K per step): an input row of one slice
//   is 64 px x 64 B = 4 KiB, so the row ring fits the 80 KiB budget with room
//   for B stages of one (slice, tap) each (128 rows x 64 B = 8 KiB).  Two steps
//   form a macro step with one barrier (64 K per barrier, as hwide4).
// * Every DMA is a compile-time item (Hw2Sched): region row u goes into ring
//   row u % RR, B step s into stage s % NBS, each issued right after the
//   barrier that ends its slot's previous reader; the counted vmcnt before
//   each barrier waits for exactly the items the next macro step reads.
// * 64-byte LDS rows: the 16-byte k-group g of row p sits at slot
//   g ^ 2((p >> 2) & 1) -- conflict-free for ds_read_b128 at every start
//   offset of a 16-row fragment (the lane groups {0-3,12-15,20-27}, ... see
//   MI355X_MICROARCH.md §LDS: each group's 16 lanes cover 4 pixel residues
//   mod 4 x 4 distinct slots), so tap shifts and dilations need no table.
// * Epilogue: hwide4's direct store (operand-swapped MFMAs, B rows in
//   hw4_perm32 order, 16-byte stores from registers, residual prefetch).
// Same arithmetic as hwide4 up to the K summation order (fp32 accumulation).
#include "wide_common.h"

namespace upr {

// 32 KiB of zeros: the source of out-of-image region rows (a lane reads at its
// offset: < 16 pixels x 1024 channels x 2 B)
__device__ __attribute__((aligned(256))) uint4 g_hw2_zero[2048];

__host__ __device__ constexpr int h2_swz(int p) { return ((p >> 2) & 1) << 1; }

constexpr int kHw2Row = 64 * 64;     // one ring row: 64 pixels x 32 channels x 2 B
constexpr int kHw2Stage = 128 * 64;  // one B stage: 128 weight rows x 32 K x 2 B

// Compile-time DMA schedule.  Steps S = 0 .. T - 1 (T = 9 NSL), macro step
// M = S / 2; barrier b (b = -1 .. NM - 2) precedes macro step b + 1 (b = -1:
// the prologue barrier); items of barrier b are issued right after it, items
// of "barrier -2" before the prologue barrier.  Items: B step s (2 pieces per
// wave) and region row (unit) u (1 piece per wave).
//   non-DL: unit u = (slice u / 6, region row u % 6) = input row oy0 - 1 + u % 6;
//           step S = (slice S / 9, tap S % 9) reads units 6c + ty .. + 3
//   DL:     unit u = (region u / 4, row u % 4); region k = (tap row k / NSL,
//           slice k % NSL) = input rows oy0 + (ty - 1) d + 0..3; step S =
//           (region S / 3, tap column S % 3) reads units 4k .. 4k + 3
template <int NSL, bool DL, int RR, int NBS>
struct Hw2Sched {
  static constexpr int T = 9 * NSL;
  static constexpr int NM = T / 2;
  static constexpr int NU = DL ? 12 * NSL : 6 * NSL;
  static constexpr int NI = T + NU;
  static constexpr int mac(int s) { return s / 2; }
  static constexpr int u_fr(int u) {
    return DL ? 3 * (u / 4) : 9 * (u / 6) + 3 * (u % 6 > 3 ? u % 6 - 3 : 0);
  }
  static constexpr int u_lr(int u) { return DL ? 3 * (u / 4) + 2 : 9 * (u / 6) + 3 * (u % 6 < 2 ? u % 6 : 2) + 2; }
  int kind[NI] = {}, idx[NI] = {}, bar[NI] = {}, fr[NI] = {};
  int start[NM + 2] = {};  // items of barrier b: [start[b + 2], start[b + 3])
  int wait[NM] = {};       // vmcnt before barrier b: wait[b + 1]
  bool ok = true;
  constexpr Hw2Sched() {
    int n = 0;
    for (int s = 0; s < T; ++s) {
      kind[n] = 0; idx[n] = s; fr[n] = s;
      bar[n] = s >= NBS ? mac(s - NBS) : -2;
      ++n;
    }
    for (int u = 0; u < NU; ++u) {
      kind[n] = 1; idx[n] = u; fr[n] = u_fr(u);
      bar[n] = u >= RR ? mac(u_lr(u - RR)) : -2;
      ++n;
    }
    // stable sort by (bar, fr)
    for (int i = 1; i < NI; ++i) {
      int j = i;
      while (j > 0 && (bar[j - 1] > bar[j] || (bar[j - 1] == bar[j] && fr[j - 1] > fr[j]))) {
        int t = 0;
        t = kind[j]; kind[j] = kind[j - 1]; kind[j - 1] = t;
        t = idx[j]; idx[j] = idx[j - 1]; idx[j - 1] = t;
        t = bar[j]; bar[j] = bar[j - 1]; bar[j - 1] = t;
        t = fr[j]; fr[j] = fr[j - 1]; fr[j - 1] = t;
        --j;
      }
    }
    for (int i = 0; i < NI; ++i)
      if (bar[i] > mac(fr[i]) - 2 || bar[i] > NM - 2) ok = false;  // must land before a wait precedes its reader
    for (int j = 0; j < NM + 2; ++j) {
      int k = 0;
      while (k < NI && bar[k] < j - 2) ++k;
      start[j] = k;
    }
    for (int b = -1; b <= NM - 2; ++b) {
      const int issued = start[b + 2];
      int total = 0, pos = 0;
      for (int i = 0; i < issued; ++i) {
        total += kind[i] == 0 ? 2 : 1;
        if (mac(fr[i]) <= b + 1) pos = total;
      }
      for (int i = issued; i < NI; ++i)
        if (mac(fr[i]) <= b + 1) ok = false;
      const int w = total - pos;
      wait[b + 1] = w > 63 ? 63 : w;
    }
  }
};

template <int NSL, bool DL, int RR, int NBS>
constexpr Hw2Sched<NSL, DL, RR, NBS> kHw2Sched{};

// NSL: 32-channel slices of the input (Cin / 32).  DL: dilated (pad = dil).
// NR: no residual operand (no prefetch registers).  RR: ring rows, NBS: B
// stages (RR * 4 KiB + NBS * 8 KiB <= 80 KiB).
// IL: the DMA items of a barrier are issued spread over the next step's MFMA
// rows (one item after each of the first rows) instead of in one burst right
// after the barrier, so the waves of a CU do not all queue LDS-DMA issue at once
template <int NSL, bool DL, bool NR, int RR, int NBS, int IL>
__global__ __launch_bounds__(256, 2) void conv_hw2_kernel(ConvOp op) {
  constexpr int W = 64, TR = 4, BM = TR * W, BN = 128;
  constexpr int WAVES_M = 2, CW = W / WAVES_M, FPR = CW / 16;
  constexpr int WM = TR * FPR, WN = BN / 2 / 16;  // 8 x 4 fragments per wave
  constexpr int RB = NBS * kHw2Stage;             // ring base (the B stages first: small ds_read offsets)
  using SC = Hw2Sched<NSL, DL, RR, NBS>;
#define SCV kHw2Sched<NSL, DL, RR, NBS>
  static_assert(SCV.ok, "DMA schedule: every item must be issued a macro step before the wait its reader needs");
  static_assert(RB + RR * kHw2Row <= 81920, "two blocks per CU");
  static_assert(SC::T % 2 == 0, "whole macro steps");
  constexpr int Cin = NSL * 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WAVES_M;
  const int wn = wave / WAVES_M;

  const int HW = op.Ho * W;
  const int M = op.B * HW;
  const int mtiles = M / BM;
  const int ntiles = op.N / BN;
  const int L = wide_xcd_remap(blockIdx.x, mtiles * ntiles);
  const int ntile = L % ntiles;
  const int mtile = L / ntiles;
  const int m0 = mtile * BM;
  const int n0 = ntile * BN;
  const int img = m0 / HW;
  const int oy0 = (m0 - img * HW) / W;
  const ConvSeg& sg = op.seg[0];
  const int cs = sg.cs, H = op.Ho;
  const int dil = DL ? sg.dil : 1;

  // region row: wave w DMAs pixels 16w .. 16w + 15 (lane = pixel, k-group slot)
  const int qp = lane >> 2;
  const unsigned voff_a = (unsigned)((qp * cs + (((lane & 3) ^ h2_swz(qp)) * 8)) * 2);
  const unsigned char* abase =
      (const unsigned char*)((const half_t*)sg.src + sg.coff + ((size_t)img * HW + (size_t)wave * 16) * cs);
  const size_t row_bytes = (size_t)W * cs * 2;
  auto issue_unit = [&](auto U_) {
    constexpr int u = decltype(U_)::value;
    constexpr int r = DL ? u % 4 : u % 6;
    constexpr int ty = DL ? (u / 4) / NSL : 0;
    constexpr int c = DL ? (u / 4) % NSL : u / 6;
    const int iy = DL ? oy0 + (ty - 1) * dil + r : oy0 - 1 + r;
    const bool in = (unsigned)iy < (unsigned)H;
    const unsigned char* ub = in ? abase + (size_t)iy * row_bytes + c * 64 : (const unsigned char*)g_hw2_zero;
    glds16_s(ub, voff_a, smem + RB + (u % RR) * kHw2Row + wave * 1024);
  };
  // B: wave w DMAs stage rows 32w .. 32w + 31 (one hw4_perm32 group), row R
  // holding weight row n0 + hw4_perm32(R)
  unsigned voff_b[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    voff_b[j] = (unsigned)((hw4_perm32(16 * j + qp) * op.Kpad + (((lane & 3) ^ h2_swz(qp)) * 8)) * 2);
  const unsigned char* bbase =
      (const unsigned char*)((const half_t*)op.W + (size_t)(n0 + wave * 32) * op.Kpad + sg.kbase);
  auto issue_b = [&](auto S_) {
    constexpr int s = decltype(S_)::value;
    constexpr int kb = DL ? (((s / 3) / NSL) * 3 + s % 3) * Cin + ((s / 3) % NSL) * 32 : (s % 9) * Cin + (s / 9) * 32;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      glds16_s(bbase + (size_t)kb * 2, voff_b[j], smem + (s % NBS) * kHw2Stage + wave * 2048 + j * 1024);
  };
  auto issue_items = [&](auto B_, auto E_) {
    constexpr int b0 = decltype(B_)::value, e0 = decltype(E_)::value;
    static_for<e0 - b0>([&](auto I_) {
      constexpr int i = b0 + decltype(I_)::value;
      if constexpr (SCV.kind[i] == 0)
        issue_b(std::integral_constant<int, SCV.idx[i]>{});
      else
        issue_unit(std::integral_constant<int, SCV.idx[i]>{});
    });
  };

  f32x4_w acc[WM][WN];
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = f32x4_w{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15;
  const int fg = lane >> 4;
  // A fragment lane offsets: pixel p of the ring row at p * 64 + slot; lanes
  // whose tap column leaves the image row read through a base far beyond the
  // block's LDS (out-of-range LDS reads return zero) with the bank bits of an
  // in-row pixel of the same residue
  constexpr int kLdsVoid = 1 << 30;
  auto lofs = [&](int p) {
    return (unsigned)p < (unsigned)W ? p * 64 + ((fg ^ h2_swz(p)) * 16)
                                     : kLdsVoid + (p & 15) * 64 + ((fg ^ h2_swz(p & 15)) * 16);
  };
  int aofs[3][FPR];
#pragma unroll
  for (int tx = 0; tx < 3; ++tx)
#pragma unroll
    for (int f = 0; f < FPR; ++f) aofs[tx][f] = lofs(CW * wm + f * 16 + fr + (tx - 1) * dil);
  const int bofs = (wn * 64 + fr) * 64 + ((fg ^ h2_swz(fr)) * 16);

  auto rd_b = [&](auto S_, f16x8_w (&bf)[WN]) {
    constexpr int S = decltype(S_)::value;
#pragma unroll
    for (int b = 0; b < WN; ++b) bf[b] = *(const f16x8_w*)(smem + bofs + (S % NBS) * kHw2Stage + b * 1024);
  };
  auto rd_a = [&](auto S_, auto A_) -> f16x8_w {
    constexpr int S = decltype(S_)::value, a = decltype(A_)::value;
    constexpr int tx = DL ? S % 3 : (S % 9) % 3;
    constexpr int u = DL ? 4 * (S / 3) + a / FPR : 6 * (S / 9) + (S % 9) / 3 + a / FPR;
    constexpr int off = RB + (u % RR) * kHw2Row;
    int ao = aofs[tx][a % FPR];
    // ds_read's immediate offset is 16 bits: a ring row at >= 64 KiB takes
    // its base in the address register (added per read: a hoisted base per
    // row stays live across the unrolled loop and spills)
    if constexpr (off >= 65536) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(ao) : "n"(off & ~0xffff));
    return *(const f16x8_w*)(smem + ao + (off & 0xffff));
  };
  f16x8_w af[WM], b0[WN], b1[WN];
  f16x8_w rv0[WM];  // pair-0 residual rows (hw4_res_load)
  // MFMAs of step S (af, bf); af rolls to step S2's fragments as each row's MFMAs issue
  // (items [IB, IE) issued after the rows: item j after row j * WM / n)
  auto mm_roll = [&](auto S2_, const f16x8_w (&bf)[WN], bool roll, auto IB_, auto IE_) {
    constexpr int ib = decltype(IB_)::value, n = decltype(IE_)::value - ib;
    static_for<WM>([&](auto A_) {
      constexpr int a = decltype(A_)::value;
#pragma unroll
      for (int b = 0; b < WN; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[b], af[a], acc[a][b], 0, 0, 0);
      if (roll) af[a] = rd_a(S2_, A_);
      static_for<n>([&](auto J_) {
        constexpr int j = decltype(J_)::value;
        if constexpr ((j * WM) / n == a)
          issue_items(std::integral_constant<int, ib + j>{}, std::integral_constant<int, ib + j + 1>{});
      });
    });
  };
  using INone = std::integral_constant<int, 0>;
  using I0 = std::integral_constant<int, 0>;
  // prologue: the "barrier -2" items, wait for macro step 0's, barrier, barrier -1's items
  issue_items(std::integral_constant<int, SCV.start[0]>{}, std::integral_constant<int, SCV.start[1]>{});
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SCV.wait[0]) : "memory");
  __builtin_amdgcn_s_barrier();
  issue_items(std::integral_constant<int, SCV.start[1]>{}, std::integral_constant<int, SCV.start[2]>{});
  rd_b(I0{}, b0);
  static_for<WM>([&](auto A_) { af[decltype(A_)::value] = rd_a(I0{}, A_); });
  static_for<SC::NM>([&](auto M_) {
    constexpr int Mi = decltype(M_)::value;
    constexpr int s0 = 2 * Mi, s1 = 2 * Mi + 1;
    rd_b(std::integral_constant<int, s1>{}, b1);
    mm_roll(std::integral_constant<int, s1>{}, b0, true, INone{}, INone{});
    if constexpr (Mi + 1 < SC::NM) {
      // RAW: the items macro step Mi + 1 reads have landed (own DMAs; everyone's
      // after the barrier).  WAR: own fragment reads of macro step Mi retired.
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(SCV.wait[Mi + 1]) : "memory");
      __builtin_amdgcn_s_barrier();
      using IB = std::integral_constant<int, SCV.start[Mi + 2]>;
      using IE = std::integral_constant<int, SCV.start[Mi + 3]>;
      if constexpr (!IL) issue_items(IB{}, IE{});
      rd_b(std::integral_constant<int, s0 + 2>{}, b0);
      if constexpr (IL) {
        mm_roll(std::integral_constant<int, s0 + 2>{}, b1, true, IB{}, IE{});
      } else {
        mm_roll(std::integral_constant<int, s0 + 2>{}, b1, true, INone{}, INone{});
      }
      // (after the items: the counted waits above only ever count DMAs)
      if constexpr (!NR && Mi == SC::NM - 2) hw4_res_load<WM, WN, WAVES_M, W>(op, rv0, m0, n0, wm, wn, lane);
    } else {
      mm_roll(std::integral_constant<int, s1>{}, b1, false, INone{}, INone{});
    }
  });
  if (op.pool) {
    // the pool partials reuse LDS: every wave's reads are done
    __syncthreads();
  }
  hw4_direct_epilogue<BN, WM, WN, WAVES_M, W, !NR>(op, acc, m0, n0, wm, wn, lane, rv0, smem);
#undef SCV
}

template <int NSL, bool DL, bool NR, int RR, int NBS, int IL>
static int launch_hw2_k(const ConvOp& op, hipStream_t st) {
  constexpr int LDS = NBS * kHw2Stage + RR * kHw2Row;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute((const void*)conv_hw2_kernel<NSL, DL, NR, RR, NBS, IL>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  const int grid = (op.B * op.Ho * 64 / 256) * (op.N / 128);
  hipLaunchKernelGGL((conv_hw2_kernel<NSL, DL, NR, RR, NBS, IL>), dim3(grid), dim3(256), LDS, st, op);
  return (int)hipGetLastError();
}

template <bool DL, bool NR>
static int launch_hw2_v(const ConvOp& op, hipStream_t st, int v) {
  // (ring rows, B stages, spread issue): 1 = (10, 5), 2 = (8, 6), 3 = (12, 4); 4..6 the same, spread
  switch (v) {
    case 2: return launch_hw2_k<8, DL, NR, 8, 6, 0>(op, st);
    case 3: return launch_hw2_k<8, DL, NR, 12, 4, 0>(op, st);
    case 4: return launch_hw2_k<8, DL, NR, 10, 5, 1>(op, st);
    case 5: return launch_hw2_k<8, DL, NR, 8, 6, 1>(op, st);
    case 6: return launch_hw2_k<8, DL, NR, 12, 4, 1>(op, st);
    default: return launch_hw2_k<8, DL, NR, 10, 5, 0>(op, st);
  }
}

// 3x3 stride-1 convs over 256 input channels at W 64, N % 128 == 0, pad 1
// (dilation 1) or pad = dilation (the ASPP branches); kErrUnsupported otherwise.
// UPR_HW2: 0 = off (hwide4 takes these), 1..3 = schedule variant (A/B)
int launch_conv_hw2(const ConvOp& op, hipStream_t st) {
  static const int mode = [] { const char* e = getenv("UPR_HW2"); return e ? atoi(e) : 1; }();
  if (mode == 0) return kErrUnsupported;
  if (op.nseg != 1 || op.store != kStoreNHWC || !hw4_ds_ok(op)) return kErrUnsupported;
  const ConvSeg& s = op.seg[0];
  if (s.kh != 3 || s.kw != 3 || s.stride != 1 || s.pre != kPreNone || s.kbase != 0) return kErrUnsupported;
  if (s.pad != s.dil || s.dil < 1 || s.dil >= 64) return kErrUnsupported;
  if (s.C != 256 || s.Hin != op.Ho || s.Win != op.Wo || op.Wo != 64 || op.Ho % 4 || op.N % 128) return kErrUnsupported;
  if (op.Kpad != 9 * s.C || op.Kpad % 8 || (uintptr_t)op.W % 16) return kErrUnsupported;
  if (s.cs % 8 || s.coff % 8 || s.cs > 1024 || (uintptr_t)s.src % 16) return kErrUnsupported;
  const bool nr = !op.res1 && !op.res2;
  if (s.dil > 1) return nr ? launch_hw2_v<true, true>(op, st, mode) : launch_hw2_v<true, false>(op, st, mode);
  return nr ? launch_hw2_v<false, true>(op, st, mode) : launch_hw2_v<false, false>(op, st, mode);
}

}  // namespace upr
