// Streaming ConvTranspose2d(k=2, s=2) for the fp16 UpBlock up-convs (dec1.up
// 64 -> 32, dec2.up 128 -> 64, dec3.up 256 -> 128; models/model.py:254-274).
// Each input pixel produces a 2x2 block of output pixels: a GEMM with K = Cin and N = 4*Cout (n = (dy*2+dx)*Cout + co, the
// graph's packing) and a pixel-shuffle store.  K is one to four 64-deep steps,
// so a tile GEMM (conv_wide) spends its time in per-tile prologue / epilogue;
// this kernel streams instead:
//   * a wave owns a 128-wide slice of N for the block's lifetime, its filter
//     fragments (A operand, 16 n x 32 k each) and bias resident in registers;
//     N / 128 waves share a 16-pixel group (one of a row's 16-pixel runs);
//   * the pixels are the B operand, read straight from HBM into registers
//     (lane = pixel fr, channels 8fg..8fg+7 of each 32-channel slice: 16-byte
//     loads) two groups ahead of the MFMAs;
//   * results go through a per-wave LDS tile [output row][32 output pixels]
//     [Cout] (pixels padded by 16 bytes; 16-byte aligned for the reads, 2-way
//     conflicts on the 8-byte writes) so every global store is a 16-byte chunk
//     of a contiguous 1 KB run of the output.
// HBM-bound: (Cin + 4 Cout) * 2 bytes per input pixel.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "upr_common.h"

namespace upr {

typedef _Float16 t2h8 __attribute__((ext_vector_type(8)));
typedef _Float16 t2h4 __attribute__((ext_vector_type(4)));
typedef float t2f4 __attribute__((ext_vector_type(4)));

template <int KC, int COUT>
struct ConvT2Cfg {
  static constexpr int N = 4 * COUT;
  static constexpr int NSPLIT = N / 128;     // waves per pixel group
  static constexpr int KS = KC / 32;         // 32-deep k slices
  static constexpr int NT = 8;               // 16-wide n tiles per wave
  static constexpr int TEAMS = 4 / NSPLIT;   // pixel groups in flight per 4-wave block
  static constexpr int QPW = COUT >= 128 ? 1 : 128 / COUT;  // (dy, dx) quads per wave
  static constexpr int ROWS = QPW >= 2 ? QPW / 2 : 1;        // output rows per wave
  static constexpr int XS = QPW >= 2 ? 32 : 16;  // staged output pixels per row (both dx / one dx)
  static constexpr int RSTR = COUT + 8;      // LDS stride (halves) of one output pixel
  static constexpr int LDSW = ROWS * XS * RSTR * 2;  // bytes per wave
  static constexpr int OCC = KC >= 256 ? 1 : 2;      // blocks per CU the registers allow
  static_assert(N % 128 == 0 && COUT % 32 == 0 && (QPW == 1 || QPW % 2 == 0), "Cout 32 / 64 / 128");
};

template <int KC, int COUT>
__global__ __launch_bounds__(256, (KC >= 256 ? 1 : 2)) void conv_t2_kernel(ConvOp op, int ngroups) {
  using K = ConvT2Cfg<KC, COUT>;
  __shared__ __attribute__((aligned(16))) unsigned char stage[4 * K::LDSW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int ns = wave % K::NSPLIT, team = wave / K::NSPLIT;
  unsigned char* st = stage + wave * K::LDSW;
  const ConvSeg& sg = op.seg[0];
  const half_t* src = (const half_t*)sg.src + sg.coff;
  const int cs = sg.cs;
  const int H = op.Ho, W = op.Wo, gpr = W / 16;  // groups per input row

  // filter fragments: lane (fr, fg) of (nt, ks) = W[ns*128 + nt*16 + fr][ks*32 + fg*8 .. +7]
  t2h8 wf[K::NT][K::KS];
  t2f4 bias[K::NT];
#pragma unroll
  for (int nt = 0; nt < K::NT; ++nt) {
    const int n = ns * 128 + nt * 16;
#pragma unroll
    for (int ks = 0; ks < K::KS; ++ks)
      wf[nt][ks] = *(const t2h8*)((const half_t*)op.W + (size_t)(n + fr) * op.Kpad + ks * 32 + fg * 8);
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[nt][r] = op.bias ? op.bias[n + fg * 4 + r] : 0.f;
  }

  // groups of this team: g0, g0 + stride, ...
  const int stride = gridDim.x * K::TEAMS;
  int g = blockIdx.x * K::TEAMS + team;
  auto load = [&](int gg, t2h8 (&x)[K::KS]) {
    if (gg < ngroups) {
      const half_t* p = src + ((size_t)gg * 16 + fr) * cs + fg * 8;
#pragma unroll
      for (int ks = 0; ks < K::KS; ++ks) x[ks] = *(const t2h8*)(p + ks * 32);
    }
  };
  t2h8 x0[K::KS], x1[K::KS], x2[K::KS];
  load(g, x0);
  load(g + stride, x1);
  for (; g < ngroups; g += stride) {
    load(g + 2 * stride, x2);
    t2f4 acc[K::NT];
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt) acc[nt] = bias[nt];
#pragma unroll
    for (int ks = 0; ks < K::KS; ++ks)
#pragma unroll
      for (int nt = 0; nt < K::NT; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nt][ks], x0[ks], acc[nt], 0, 0, 0);
    // lane holds n = ns*128 + nt*16 + 4fg + r (r = 0..3) of pixel fr: quad q = n / COUT,
    // channels co..co+3 -> LDS [row dy - dy0][2 fr + dx (both dx) | fr (one dx)][co]
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt) {
      const int nl = nt * 16 + fg * 4;  // within the wave's slice
      const int ql = nl / COUT, co = nl % COUT;
      const int row = ql >> 1, xs = K::QPW >= 2 ? 2 * fr + (ql & 1) : fr;
      t2h4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[nt][r];
        if (op.relu) v = fmaxf(v, 0.f);
        o[r] = (half_t)v;
      }
      *(t2h4*)(st + ((row * K::XS + xs) * K::RSTR + co) * 2) = o;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // (b, y, x0) of the group; output rows 2y + dy0 + row, columns 2 x0 ..
    const int b = g / (H * gpr), rem = g - b * H * gpr, y = rem / gpr, xg = (rem - y * gpr) * 16;
    const int q0 = ns * K::QPW, dy0 = q0 >> 1;
    constexpr int CPP = COUT / 8;  // 16-byte chunks per output pixel
    constexpr int CHUNKS = K::ROWS * K::XS * CPP;
#pragma unroll
    for (int i = 0; i < CHUNKS / 64; ++i) {
      const int c = i * 64 + lane;
      const int row = c / (K::XS * CPP), xs = (c / CPP) % K::XS, part = c % CPP;
      const int xo = K::QPW >= 2 ? 2 * xg + xs : 2 * (xg + xs) + (q0 & 1);  // output column
      const t2h8 v = *(const t2h8*)(st + ((row * K::XS + xs) * K::RSTR + part * 8) * 2);
      half_t* dst = (half_t*)op.out + ((size_t)(b * 2 * H + 2 * y + dy0 + row) * (2 * W) + xo) * op.out_cs +
                    op.out_coff + part * 8;
      *(t2h8*)dst = v;
    }
    __builtin_amdgcn_wave_barrier();  // the LDS tile is rewritten next iteration
#pragma unroll
    for (int ks = 0; ks < K::KS; ++ks) {
      x0[ks] = x1[ks];
      x1[ks] = x2[ks];
    }
  }
}

// fp32 form (v_mfma_f32_16x16x4_f32): the same streaming / staging; the k
// order inside a pixel is permuted identically for both operands (lane group
// fg takes channels fg*KC/4 .. +KC/4-1, so a lane's pixel operand is KC/16
// 16-byte loads and its filter operand a contiguous run of one filter row).
// KC 64 (dec1.up) and 128 (dec2.up): the filter slice is KC/4 x 8 floats per
// lane (128 / 256 VGPRs).
template <int KC, int COUT>
__global__ __launch_bounds__(256, (KC >= 128 ? 1 : 2)) void conv_t2_f32_kernel(ConvOp op, int ngroups) {
  using K = ConvT2Cfg<KC, COUT>;
  constexpr int KJ = KC / 4;    // k steps of 4 (one MFMA each per n tile)
  constexpr int KQ = KJ / 4;    // 16-byte chunks of a lane's pixel operand
  constexpr int RSTR = COUT + 4;  // LDS stride (floats) of one output pixel (16-byte aligned)
  constexpr int LDSW = K::ROWS * K::XS * RSTR * 4;
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) unsigned char stage[4 * LDSW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int ns = wave % K::NSPLIT, team = wave / K::NSPLIT;
  unsigned char* st = stage + wave * LDSW;
  const ConvSeg& sg = op.seg[0];
  const float* src = (const float*)sg.src + sg.coff;
  const int cs = sg.cs;
  const int H = op.Ho, W = op.Wo, gpr = W / 16;

  f4 wf[K::NT][KQ];  // lane (fr, fg) of n tile nt: W[ns*128 + nt*16 + fr][fg*KJ .. +KJ-1]
  f4 bias[K::NT];
#pragma unroll
  for (int nt = 0; nt < K::NT; ++nt) {
    const int n = ns * 128 + nt * 16;
#pragma unroll
    for (int q = 0; q < KQ; ++q)
      wf[nt][q] = *(const f4*)((const float*)op.W + (size_t)(n + fr) * op.Kpad + fg * KJ + q * 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[nt][r] = op.bias ? op.bias[n + fg * 4 + r] : 0.f;
  }
  const int stride = gridDim.x * K::TEAMS;
  int g = blockIdx.x * K::TEAMS + team;
  auto load = [&](int gg, f4 (&x)[KQ]) {
    if (gg < ngroups) {
      const float* p = src + ((size_t)gg * 16 + fr) * cs + fg * KJ;
#pragma unroll
      for (int q = 0; q < KQ; ++q) x[q] = *(const f4*)(p + q * 4);
    }
  };
  f4 x0[KQ], x1[KQ];
  load(g, x0);
  for (; g < ngroups; g += stride) {
    load(g + stride, x1);
    f4 acc[K::NT];
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt) acc[nt] = bias[nt];
#pragma unroll
    for (int j = 0; j < KJ; ++j)
#pragma unroll
      for (int nt = 0; nt < K::NT; ++nt)
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[nt][j >> 2][j & 3], x0[j >> 2][j & 3], acc[nt], 0, 0, 0);
#pragma unroll
    for (int nt = 0; nt < K::NT; ++nt) {
      const int nl = nt * 16 + fg * 4;
      const int ql = nl / COUT, co = nl % COUT;
      const int row = ql >> 1, xs = K::QPW >= 2 ? 2 * fr + (ql & 1) : fr;
      f4 o = acc[nt];
      if (op.relu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = fmaxf(o[r], 0.f);
      }
      *(f4*)(st + ((row * K::XS + xs) * RSTR + co) * 4) = o;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int b = g / (H * gpr), rem = g - b * H * gpr, y = rem / gpr, xg = (rem - y * gpr) * 16;
    const int q0 = ns * K::QPW, dy0 = q0 >> 1;
    constexpr int CPP = COUT / 4;
    constexpr int CHUNKS = K::ROWS * K::XS * CPP;
#pragma unroll
    for (int i = 0; i < CHUNKS / 64; ++i) {
      const int c = i * 64 + lane;
      const int row = c / (K::XS * CPP), xs = (c / CPP) % K::XS, part = c % CPP;
      const int xo = K::QPW >= 2 ? 2 * xg + xs : 2 * (xg + xs) + (q0 & 1);
      const f4 v = *(const f4*)(st + ((row * K::XS + xs) * RSTR + part * 4) * 4);
      float* dst = (float*)op.out + ((size_t)(b * 2 * H + 2 * y + dy0 + row) * (2 * W) + xo) * op.out_cs +
                   op.out_coff + part * 4;
      *(f4*)dst = v;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < KQ; ++q) x0[q] = x1[q];
  }
}

template <int KC, int COUT>
static int launch_t2_f32(const ConvOp& op, hipStream_t st) {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)conv_t2_f32_kernel<KC, COUT>, 256, 0) !=
            hipSuccess ||
        occ < 1)
      occ = 1;
  }
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const int ngroups = op.B * op.Ho * (op.Wo / 16);
  const int teams = ConvT2Cfg<KC, COUT>::TEAMS;
  int grid = std::min(cus * occ, (ngroups + teams - 1) / teams);
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((conv_t2_f32_kernel<KC, COUT>), dim3(grid), dim3(256), 0, st, op, ngroups);
  return (int)hipGetLastError();
}

template <int KC, int COUT>
static int launch_t2(const ConvOp& op, hipStream_t st) {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)conv_t2_kernel<KC, COUT>, 256, 0) !=
            hipSuccess ||
        occ < 1)
      occ = 1;
  }
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const int ngroups = op.B * op.Ho * (op.Wo / 16);
  const int teams = ConvT2Cfg<KC, COUT>::TEAMS;
  int grid = std::min(cus * occ, (ngroups + teams - 1) / teams);
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((conv_t2_kernel<KC, COUT>), dim3(grid), dim3(256), 0, st, op, ngroups);
  return (int)hipGetLastError();
}

// ConvT 2x2 ops these kernels take; kErrUnsupported otherwise.
int launch_conv_t2(const ConvOp& op, int dtype, hipStream_t st) {
  if (op.store != kStoreConvT2x2 || op.nseg != 1) return kErrUnsupported;
  if (op.res1 || op.res2 || op.pool || op.img_bias || op.scale || op.out2 || op.out32) return kErrUnsupported;
  const ConvSeg& s = op.seg[0];
  if (s.kh != 1 || s.kw != 1 || s.stride != 1 || s.pad != 0 || s.pre != kPreNone || s.kbase != 0) return kErrUnsupported;
  if (s.Hin != op.Ho || s.Win != op.Wo || op.Wo % 16 || s.cs % 8 || s.coff % 8 || (uintptr_t)s.src % 16)
    return kErrUnsupported;
  if (op.out_cs % 8 || op.out_coff % 8 || (uintptr_t)op.out % 16 || (uintptr_t)op.W % 16 || op.Kpad % 8)
    return kErrUnsupported;
  if (dtype != kF16) {
    if (s.cs % 4 || s.coff % 4 || op.out_cs % 4 || op.out_coff % 4) return kErrUnsupported;
    if (s.C == 64 && op.N == 128) return launch_t2_f32<64, 32>(op, st);
    if (s.C == 128 && op.N == 256) return launch_t2_f32<128, 64>(op, st);
    return kErrUnsupported;
  }
  if (s.C == 64 && op.N == 128) return launch_t2<64, 32>(op, st);
  if (s.C == 128 && op.N == 256) return launch_t2<128, 64>(op, st);
  if (s.C == 256 && op.N == 512) return launch_t2<256, 128>(op, st);
  return kErrUnsupported;
}

}  // namespace upr
