// Streaming 1x1 convolution (fp16 operands, fp32 accumulate) for the narrow
// GEMMs of the training step: K = Cin and N = Cout both in {32, 64, 96, 128}
// at 256^2 / 512^2 -- the multi-scale head's fusion 96 -> 32 and the
// EnhancedFAM fusion 128 -> 32 (models/model.py:49, :413-414) and their input
// gradients 32 -> 96 / 32 -> 128, and the projecting shortcut's stride-2 input
// gradient (model.py:119-122).  A 64-deep tile GEMM spends these in prologue /
// epilogue (one or two K steps); here, as in conv_t2:
//   * a wave keeps the whole filter (N/16 x K/32 fragments) and the bias in
//     registers for the block's lifetime and walks 16-pixel groups;
//   * the pixels are the B operand, read straight from HBM into registers
//     (lane = pixel fr, channels 8 fg .. 8 fg + 7 of each 32-channel slice:
//     16-byte loads) one group ahead of the MFMAs;
//   * the MFMA operands are swapped (weights first), so a lane holds 4
//     consecutive output channels of one pixel: the epilogue stores 16 bytes
//     (fp32) / 8 bytes (fp16) per lane with no LDS staging.
// Epilogues: the fp16 `out` (bias, ReLU) and the training step's fp32 family
// (ConvOp::out32 / res32 / mask16 / out32_h16 / skip32: the fp16-rounded
// result widened to fp32, plus the accumulated gradient, ReLU-masked).
// out_s2: the 1x1 stride-2 input gradient -- input pixel (b, i, j) is written
// to output pixel (b, 2i, 2j) of a 2H x 2W map; the other pixels are left as
// they are (the caller accumulates into a gradient that already holds the
// rest), so the zero-upsampled operand of the generic path is never built.
// HBM-bound: (K * 2 + N * (4 + 2 [+ 4 residual])) bytes per pixel.
#include <algorithm>

#include "upr_common.h"

namespace upr {

typedef _Float16 pwh8 __attribute__((ext_vector_type(8)));
typedef _Float16 pwh4 __attribute__((ext_vector_type(4)));
typedef float pwf4 __attribute__((ext_vector_type(4)));

template <int KC, int NC, bool OUT32, bool S2>
__global__ __launch_bounds__(256, 2) void conv_pw_kernel(ConvOp op, int ngroups) {
  constexpr int KS = KC / 32, NT = NC / 16;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const ConvSeg& sg = op.seg[0];
  const half_t* src = (const half_t*)sg.src + sg.coff;
  const int cs = sg.cs;
  const int Win = sg.Win, HWin = sg.Hin * sg.Win;

  // filter fragment (nt, ks): lane (fr, fg) = W[nt*16 + fr][ks*32 + 8 fg .. +7]
  pwh8 wf[NT][KS];
  pwf4 bias[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[nt][ks] = *(const pwh8*)((const half_t*)op.W + (size_t)(nt * 16 + fr) * op.Kpad + ks * 32 + fg * 8);
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[nt][r] = op.bias ? op.bias[nt * 16 + fg * 4 + r] : 0.f;
  }
  // OUT32 with every fp32-family tensor dense ([pix][NC]): a wave's 16 pixels
  // are one contiguous 16 x NC run of each, so the epilogue stages the rounded
  // values in LDS and then reads, adds, masks and stores that run in 16-byte
  // lane pieces (1 KB per instruction) -- the direct form's 64-byte pieces at
  // an NC * 4-byte pixel stride held the 96-channel input gradient at ~3.5 TB/s
  constexpr int STG = OUT32 && !S2 ? 16 * NC : 4;
  __shared__ __attribute__((aligned(16))) float stg[4][STG];
  const bool dense = OUT32 && !S2 && op.out32_cs == NC && op.out32_coff == 0 && (!op.res32 || op.res32_cs == NC) &&
                     (!op.mask16 || op.mask16_cs == NC) && (!op.out32_h16 || op.out32_h16_cs == NC);
  const int stride = gridDim.x * 4;
  int g = blockIdx.x * 4 + wave;
  auto load = [&](int gg, pwh8 (&x)[KS]) {
    if (gg < ngroups) {
      const half_t* p = src + ((size_t)gg * 16 + fr) * cs + fg * 8;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) x[ks] = *(const pwh8*)(p + ks * 32);
    }
  };
  pwh8 x0[KS], x1[KS];
  load(g, x0);
  for (; g < ngroups; g += stride) {
    load(g + stride, x1);
    pwf4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = pwf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nt][ks], x0[ks], acc[nt], 0, 0, 0);
    // output pixel of this lane
    size_t m = (size_t)g * 16 + fr;
    if constexpr (S2) {
      // groups are whole 16-pixel runs of one input row (Win % 16 == 0)
      const int q0 = g * 16;
      const int b = q0 / HWin, rem = q0 - b * HWin, i = rem / Win, j = rem - i * Win + fr;
      m = ((size_t)(b * 2 * sg.Hin + 2 * i) * (2 * Win)) + 2 * j;
    }
    if constexpr (OUT32 && !S2) {
      if (dense) {
        float* sw = stg[wave];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          pwf4 t;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[nt][r] + bias[nt][r];
            if (op.relu) v = fmaxf(v, 0.f);
            t[r] = (float)(half_t)v;
          }
          *(pwf4*)(sw + fr * NC + nt * 16 + fg * 4) = t;
        }
        __builtin_amdgcn_wave_barrier();  // (one wave's LDS accesses execute in order)
        const size_t e0 = (size_t)g * 16 * NC;
#pragma unroll
        for (int i = 0; i < NC / 16; ++i) {
          const int e = (i * 64 + lane) * 4;
          pwf4 t = *(const pwf4*)(sw + e);
          const size_t me = e0 + e;
          if (op.res32) t += *(const pwf4*)(op.res32 + me);
          if (op.mask16) {
            const pwh4 mk = *(const pwh4*)((const half_t*)op.mask16 + me);
#pragma unroll
            for (int r = 0; r < 4; ++r) t[r] = (float)mk[r] > 0.f ? t[r] : 0.f;
          }
          if (!op.skip32) *(pwf4*)(op.out32 + me) = t;
          if (op.out32_h16)
            *(pwh4*)((half_t*)op.out32_h16 + me) = pwh4{(half_t)t[0], (half_t)t[1], (half_t)t[2], (half_t)t[3]};
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) x0[ks] = x1[ks];
        continue;
      }
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = nt * 16 + fg * 4;
      pwh4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[nt][r] + bias[nt][r];
        if (op.relu) v = fmaxf(v, 0.f);
        o[r] = (half_t)v;
      }
      if constexpr (OUT32) {
        pwf4 t;
#pragma unroll
        for (int r = 0; r < 4; ++r) t[r] = (float)o[r];
        if (op.res32) t += *(const pwf4*)(op.res32 + m * op.res32_cs + n);
        if (op.mask16) {
          const pwh4 mk = *(const pwh4*)((const half_t*)op.mask16 + m * op.mask16_cs + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) t[r] = (float)mk[r] > 0.f ? t[r] : 0.f;
        }
        if (!op.skip32) *(pwf4*)(op.out32 + m * op.out32_cs + op.out32_coff + n) = t;
        if (op.out32_h16)
          *(pwh4*)((half_t*)op.out32_h16 + m * op.out32_h16_cs + n) =
              pwh4{(half_t)t[0], (half_t)t[1], (half_t)t[2], (half_t)t[3]};
      } else {
        *(pwh4*)((half_t*)op.out + m * op.out_cs + op.out_coff + n) = o;
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) x0[ks] = x1[ks];
  }
}

template <int KC, int NC, bool OUT32, bool S2>
static int launch_pw(const ConvOp& op, hipStream_t st) {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)conv_pw_kernel<KC, NC, OUT32, S2>, 256, 0) !=
            hipSuccess ||
        occ < 1)
      occ = 1;
  }
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const long long npix = (long long)op.B * op.seg[0].Hin * op.seg[0].Win;
  const int ngroups = (int)(npix / 16);
  int grid = std::min(cus * occ, (ngroups + 3) / 4);
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((conv_pw_kernel<KC, NC, OUT32, S2>), dim3(grid), dim3(256), 0, st, op, ngroups);
  return (int)hipGetLastError();
}

template <int KC, bool OUT32, bool S2>
static int pw_n(const ConvOp& op, hipStream_t st) {
  switch (op.N) {
    case 32: return launch_pw<KC, 32, OUT32, S2>(op, st);
    case 64: return launch_pw<KC, 64, OUT32, S2>(op, st);
    case 96: return launch_pw<KC, 96, OUT32, S2>(op, st);
    case 128: return launch_pw<KC, 128, OUT32, S2>(op, st);
    default: return kErrUnsupported;
  }
}

template <bool OUT32, bool S2>
static int pw_k(const ConvOp& op, hipStream_t st) {
  switch (op.seg[0].C) {
    case 32: return pw_n<32, OUT32, S2>(op, st);
    case 64: return pw_n<64, OUT32, S2>(op, st);
    case 96: return pw_n<96, OUT32, S2>(op, st);
    case 128: return pw_n<128, OUT32, S2>(op, st);
    default: return kErrUnsupported;
  }
}

// ---------------------------------------------------------------------------
// Input gradient of a 3x3 stride-2 pad-1 conv (enc1.conv1, 32 -> 64 at 512^2:
// models/model.py:100-178) without the zero-upsampled operand.  As a stride-1
// conv over the zero-upsampled dy z (z(2i', 2j') = dy(i', j')) with the
// flipped filter wf, dx(r, c) = sum_{t'} z(r - 1 + t'y, c - 1 + t'x) wf(t');
// only the taps that land on even z positions contribute, so the four output
// phases (r, c) = (2i + py, 2j + px) are small convs over dy itself:
//   (0,0): wf(1,1) dy(i,j)
//   (0,1): wf(1,0) dy(i,j) + wf(1,2) dy(i,j+1)
//   (1,0): wf(0,1) dy(i,j) + wf(2,1) dy(i+1,j)
//   (1,1): wf(0,0) dy(i,j) + wf(0,2) dy(i,j+1) + wf(2,0) dy(i+1,j) + wf(2,2) dy(i+1,j+1)
// -- the 9 taps once each, no MFMA on zeros, no upsampled tensor in HBM.  A
// wave keeps the whole flipped filter (9 taps x N/16 x K/32 fragments) in
// registers and walks 16-pixel groups of dy rows, loading the four shifted
// pixel runs (zero past the image) and writing all four phases with the
// out32 epilogue family of conv_pw_kernel.
// ---------------------------------------------------------------------------
template <int KC, int NC>
__global__ __launch_bounds__(256) void conv_s2dg_kernel(ConvOp op, int ngroups) {
  constexpr int KS = KC / 32, NT = NC / 16;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const ConvSeg& sg = op.seg[0];
  const half_t* src = (const half_t*)sg.src;
  const int Hin = sg.Hin, Win = sg.Win, HWin = Hin * Win;

  // flipped tap (ty, tx) fragment (nt, ks): lane (fr, fg) = W[nt*16 + fr][(ty*3 + tx)*KC + ks*32 + 8 fg .. +7]
  pwh8 wf[9][NT][KS];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        wf[t][nt][ks] = *(const pwh8*)((const half_t*)op.W + (size_t)(nt * 16 + fr) * op.Kpad + t * KC + ks * 32 + fg * 8);
  const int stride = gridDim.x * 4;
  for (int g = blockIdx.x * 4 + wave; g < ngroups; g += stride) {
    const int q0 = g * 16;
    const int b = q0 / HWin, rem = q0 - b * HWin, i = rem / Win, j = rem - i * Win + fr;
    pwh8 x[4][KS];  // (di, dj) = (0,0), (0,1), (1,0), (1,1)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ii = i + (s >> 1), jj = j + (s & 1);
      const bool in = ii < Hin && jj < Win;
      const half_t* p = src + ((size_t)(b * Hin + ii) * Win + jj) * sg.cs + fg * 8;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) x[s][ks] = in ? *(const pwh8*)(p + ks * 32) : pwh8{};
    }
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int py = ph >> 1, px = ph & 1;
      pwf4 acc[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = pwf4{0.f, 0.f, 0.f, 0.f};
      // taps of the phase: (di, flipped ty) = py ? {(0, 0), (1, 2)} : {(0, 1)}; the same in x
#pragma unroll
      for (int a = 0; a < 1 + py; ++a) {
        const int di = a, ty = py ? 2 * a : 1;
#pragma unroll
        for (int c = 0; c < 1 + px; ++c) {
          const int dj = c, tx = px ? 2 * c : 1;
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
              acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ty * 3 + tx][nt][ks], x[di * 2 + dj][ks], acc[nt], 0, 0, 0);
        }
      }
      const size_t m = (size_t)(b * 2 * Hin + 2 * i + py) * (2 * Win) + 2 * j + px;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int n = nt * 16 + fg * 4;
        pwf4 t;
#pragma unroll
        for (int r = 0; r < 4; ++r) t[r] = (float)(half_t)acc[nt][r];
        if (op.res32) t += *(const pwf4*)(op.res32 + m * op.res32_cs + n);
        if (op.mask16) {
          const pwh4 mk = *(const pwh4*)((const half_t*)op.mask16 + m * op.mask16_cs + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) t[r] = (float)mk[r] > 0.f ? t[r] : 0.f;
        }
        if (!op.skip32) *(pwf4*)(op.out32 + m * op.out32_cs + op.out32_coff + n) = t;
        if (op.out32_h16)
          *(pwh4*)((half_t*)op.out32_h16 + m * op.out32_h16_cs + n) =
              pwh4{(half_t)t[0], (half_t)t[1], (half_t)t[2], (half_t)t[3]};
      }
    }
  }
}

// The same phase decomposition for wider convs (enc2.conv1: 128 -> 64 and
// enc3.conv1: 256 -> 128 input gradients; their filters do not fit the
// registers): a block owns an NC-channel slice of the output (grid.y), its
// flipped filter slice sits in LDS as per-lane 16-byte fragments
// [tap][nt][ks][lane], and a wave walks 16-pixel groups of dy rows, loading
// the four shifted runs of one 32-channel chunk at a time and issuing every
// phase's taps on it (accumulators of all four phases live together).  One
// fragment read per MFMA; dy is read once per slice.  (Those shapes zero-
// upsampled dy and ran the stride-1 conv over it: 4x the MFMAs and the
// upsampled tensor's traffic, 17x the shape's bound.)
template <int KC, int NC>
__global__ __launch_bounds__(256, 2) void conv_s2dg_lds_kernel(ConvOp op, int ngroups) {
  constexpr int KS = KC / 32, NT = NC / 16, NFRAG = 9 * NT * KS;
  extern __shared__ __attribute__((aligned(16))) unsigned char s2smem[];
  pwh8* wl = (pwh8*)s2smem;  // [9][NT][KS][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const ConvSeg& sg = op.seg[0];
  const half_t* src = (const half_t*)sg.src;
  const int Hin = sg.Hin, Win = sg.Win, HWin = Hin * Win;
  const int nbase = blockIdx.y * NC;
  for (int f = threadIdx.x; f < NFRAG * 64; f += 256) {
    const int ln = f & 63, rest = f >> 6;
    const int ks = rest % KS, nt = (rest / KS) % NT, t = rest / (KS * NT);
    wl[f] = *(const pwh8*)((const half_t*)op.W + (size_t)(nbase + nt * 16 + (ln & 15)) * op.Kpad + t * KC + ks * 32 +
                           (ln >> 4) * 8);
  }
  __syncthreads();
  const int stride = gridDim.x * 4;
  for (int g = blockIdx.x * 4 + wave; g < ngroups; g += stride) {
    const int q0 = g * 16;
    const int b = q0 / HWin, rem = q0 - b * HWin, i = rem / Win, j = rem - i * Win + fr;
    pwf4 acc[4][NT];
#pragma unroll
    for (int ph = 0; ph < 4; ++ph)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[ph][nt] = pwf4{0.f, 0.f, 0.f, 0.f};
    // (two chunks per pass: a fully unrolled chunk loop hoisted every chunk's loads and spilled)
#pragma unroll 2
    for (int ks = 0; ks < KS; ++ks) {
      pwh8 x[4];  // (di, dj) = (0,0), (0,1), (1,0), (1,1)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int ii = i + (s >> 1), jj = j + (s & 1);
        const bool in = ii < Hin && jj < Win;
        x[s] = in ? *(const pwh8*)(src + ((size_t)(b * Hin + ii) * Win + jj) * sg.cs + ks * 32 + fg * 8) : pwh8{};
      }
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        const int py = ph >> 1, px = ph & 1;
#pragma unroll
        for (int a = 0; a < 1 + py; ++a) {
          const int ty = py ? 2 * a : 1;
#pragma unroll
          for (int c = 0; c < 1 + px; ++c) {
            const int tx = px ? 2 * c : 1;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
              acc[ph][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[(((ty * 3 + tx) * NT + nt) * KS + ks) * 64 + lane],
                                                                   x[a * 2 + c], acc[ph][nt], 0, 0, 0);
          }
        }
      }
    }
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int py = ph >> 1, px = ph & 1;
      const size_t m = (size_t)(b * 2 * Hin + 2 * i + py) * (2 * Win) + 2 * j + px;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int n = nbase + nt * 16 + fg * 4;
        pwf4 t;
#pragma unroll
        for (int r = 0; r < 4; ++r) t[r] = (float)(half_t)acc[ph][nt][r];
        if (op.res32) t += *(const pwf4*)(op.res32 + m * op.res32_cs + n);
        if (op.mask16) {
          const pwh4 mk = *(const pwh4*)((const half_t*)op.mask16 + m * op.mask16_cs + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) t[r] = (float)mk[r] > 0.f ? t[r] : 0.f;
        }
        if (!op.skip32) *(pwf4*)(op.out32 + m * op.out32_cs + op.out32_coff + n) = t;
        if (op.out32_h16)
          *(pwh4*)((half_t*)op.out32_h16 + m * op.out32_h16_cs + n) =
              pwh4{(half_t)t[0], (half_t)t[1], (half_t)t[2], (half_t)t[3]};
      }
    }
  }
}

// the 3x3 stride-2 input gradients above (op: dy as a 1-segment 3x3 op over
// Hin x Win with the flipped filter, out32 family at 2 Hin x 2 Win): 64 -> 32
// with the filter in registers, 128 -> 64 and 256 -> 128 with LDS filter slices
int launch_conv_s2dg(const ConvOp& op, hipStream_t st, bool probe) {
  const ConvSeg& s = op.seg[0];
  if (op.nseg != 1 || op.store != kStoreNHWC || !op.out32 || op.bias || op.relu || op.res1 || op.res2 || op.pool ||
      op.img_bias || op.scale || op.out2)
    return kErrUnsupported;
  // (C, N): 64 -> 32 register-filter kernel; 128 -> 64 and 256 -> 128 LDS-filter kernel
  const int form = s.C == 64 && op.N == 32 ? 1 : s.C == 128 && op.N == 64 ? 2 : s.C == 256 && op.N == 128 ? 3 : 0;
  if (s.kh != 3 || s.kw != 3 || !form || s.kbase != 0 || s.pre != kPreNone) return kErrUnsupported;
  if (s.cs % 8 || (uintptr_t)s.src % 16 || op.Kpad % 8 || (uintptr_t)op.W % 16 || s.Win % 16) return kErrUnsupported;
  if ((uintptr_t)op.out32 % 16 || op.out32_cs % 4 || op.out32_coff % 4) return kErrUnsupported;
  if (op.res32 && ((uintptr_t)op.res32 % 16 || op.res32_cs % 4)) return kErrUnsupported;
  if (op.mask16 && ((uintptr_t)op.mask16 % 8 || op.mask16_cs % 4)) return kErrUnsupported;
  if (op.out32_h16 && ((uintptr_t)op.out32_h16 % 8 || op.out32_h16_cs % 4)) return kErrUnsupported;
  const long long npix = (long long)op.B * s.Hin * s.Win;
  if (npix >= (1ll << 31) / 4) return kErrUnsupported;
  if (probe) return kOk;
  const int ngroups = (int)(npix / 16);
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  int grid = std::min(cus * 2, (ngroups + 3) / 4);
  if (grid < 1) grid = 1;
  // (64 -> 32 as an LDS-filter slice measured slower than the register-filter kernel: 141.6 vs
  // 133.3 us, profiles/r5_s2dgrad_lds_ab.txt)
  if (form == 1) {
    hipLaunchKernelGGL((conv_s2dg_kernel<64, 32>), dim3(grid), dim3(256), 0, st, op, ngroups);
  } else {
    // LDS filter slices (73.7 KB each: two blocks per CU); the slices split the CUs
    auto go = [&](auto kern, int nc, int kc) {
      const size_t lds = (size_t)9 * nc * kc * 2;
      static bool attr[4] = {false, false, false, false};
      if (!attr[form]) {
        const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
        attr[form] = true;
      }
      const int slices = op.N / nc;
      const int gx = std::max(1, std::min((cus * 2 + slices - 1) / slices, (ngroups + 3) / 4));
      hipLaunchKernelGGL(kern, dim3(gx, slices), dim3(256), lds, st, op, ngroups);
      return 0;
    };
    const int rc = form == 2 ? go(conv_s2dg_lds_kernel<128, 32>, 32, 128) : go(conv_s2dg_lds_kernel<256, 16>, 16, 256);
    if (rc != 0) return rc;
  }
  return (int)hipGetLastError();
}

// fp16 1x1 stride-1 convs of the shapes above; kErrUnsupported otherwise
// (an out_s2 op must be taken here: no other kernel implements it)
int launch_conv_pw(const ConvOp& op, hipStream_t st, bool probe) {
  if (op.nseg != 1 || op.store != kStoreNHWC) return kErrUnsupported;
  const ConvSeg& s = op.seg[0];
  if (s.kh != 1 || s.kw != 1 || s.stride != 1 || s.pad != 0 || s.pre != kPreNone || s.kbase != 0) return kErrUnsupported;
  if (s.Hin != op.Ho || s.Win != op.Wo) return kErrUnsupported;
  if (s.C > 128 || s.C % 32 || op.N > 128 || op.N % 32) return kErrUnsupported;
  if (op.res1 || op.res2 || op.pool || op.img_bias || op.scale || op.out2) return kErrUnsupported;
  if (s.cs % 8 || s.coff % 8 || (uintptr_t)s.src % 16 || op.Kpad % 8 || (uintptr_t)op.W % 16) return kErrUnsupported;
  if (((long long)op.B * s.Hin * s.Win) % 16) return kErrUnsupported;
  if (op.out_s2 && (s.Win % 16 || !op.out32)) return kErrUnsupported;
  if (op.out32) {
    if ((uintptr_t)op.out32 % 16 || op.out32_cs % 4 || op.out32_coff % 4) return kErrUnsupported;
    if (op.res32 && ((uintptr_t)op.res32 % 16 || op.res32_cs % 4)) return kErrUnsupported;
    if (op.mask16 && ((uintptr_t)op.mask16 % 8 || op.mask16_cs % 4)) return kErrUnsupported;
    if (op.out32_h16 && ((uintptr_t)op.out32_h16 % 8 || op.out32_h16_cs % 4)) return kErrUnsupported;
    if (probe) return kOk;
    return op.out_s2 ? pw_k<true, true>(op, st) : pw_k<true, false>(op, st);
  }
  if ((uintptr_t)op.out % 8 || op.out_cs % 4 || op.out_coff % 4) return kErrUnsupported;
  if (probe) return kOk;
  return pw_k<false, false>(op, st);
}

}  // namespace upr
