// Wide-tile implicit-GEMM convolution for fp32 operands (exact fp32:
// v_mfma_f32_16x16x4_f32, fp32 accumulate) -- the fp32 graph's (configs[1],
// BASELINE.json headline) MFMA-bound convs with >= 64 output channels:
// encoder blocks incl. the stride-2 convs and the projecting shortcut K-segment,
// bottleneck ResBlocks, ASPP, decoder convs and the ConvTranspose GEMMs, and the
// EnhancedFAM cascaded first convs (models/model.py:11-97, 100-274).
//
// fp32 MFMA runs at 1/16 of the fp16 rate (64 FLOP/clk/SIMD), so a K step of
// 32 channels over a 256 x 128 (or 512 x 64) tile is 8192 MFMA cycles per SIMD:
// one barrier and one operand fetch per step cost little next to it, which is
// what the register-staged halo kernel (conv_halo.hip: 4 x 32 pixels x 32
// channels per block, ~2.4 VALU + 1.2 SALU per MFMA of staging address math)
// could not offer.  Structure (shared with the fp16 conv_wide.hip):
//
// * 512 threads = 8 waves, each a 64-pixel x 64-channel block of 16 x 16
//   accumulator tiles (WM = WN = 4, 64 accumulator registers).
// * Both operands global -> LDS by LDS-DMA (global_load_lds_dwordx4): 128-byte
//   rows (32 fp32 channels), lane-linear; the 16-byte chunk index XOR-swizzled
//   by (row >> 1) & 7 on the SOURCE address, un-swizzled on the fragment reads
//   (ds_read_b128 lane groups conflict free).  A rows are a per-lane gather
//   (output pixel shifted by the tap through stride / dilation / padding;
//   padded taps and rows past M read a 128-byte zero line); B rows are the
//   packed [N][Kpad] weights.
// * Fragments: lane (r = lane & 15, g = lane >> 4) reads chunk g (first half)
//   and chunk 4 + g (second half) of its row: 4 MFMAs per half per tile, MFMA
//   e takes channel 4*chunk + e of lane group g as its k-slot g.  A and B use
//   the same map, so the dot product is unchanged (exact fp32 fma chain).
// * Two LDS stages and the half-step software pipeline of conv_wide.hip: the
//   second half's fragments are read before the barrier that releases the next
//   stage, its MFMAs run after it; the next step's DMA flies meanwhile.
// * Epilogue through LDS in 64-row passes: bias / per-image bias / residual /
//   ReLU / residual, 2 x 16-byte stores per 8 channels, ConvTranspose pixel
//   shuffle, per-image pooled sums (ASPP global branch) with one atomic per
//   channel per tile.
//
// Segments must be plain (no pre-activation / max-pool prologue), C % 32 == 0.
#include <cstdlib>
#include <cstring>

#include "upr_common.h"

namespace upr {

typedef float f32x4_q __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_void_ptr_q;

__device__ __attribute__((aligned(128))) uint4 g_w32_zero[8];

constexpr int Q_BK = 32;  // fp32 channels per K step = one 128-byte LDS row

template <int BM, int BN>
struct Q32Cfg {
  static constexpr int WN = BN >= 64 ? 4 : BN / 16;  // 16-column tiles per wave
  static constexpr int WAVES_N = BN / (16 * WN);
  static constexpr int WAVES_M = 8 / WAVES_N;
  static constexpr int WM = BM / WAVES_M / 16;  // 16-row tiles per wave
  static constexpr int A_BYTES = BM * 128;
  static constexpr int B_BYTES = BN * 128;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int AI = BM / 64;            // A DMA instructions per wave per step (8 rows each)
  static constexpr int BJ = (BN / 8 + 7) / 8;   // B DMA instructions per wave per step (<= BN / 8 in all)
  static constexpr int CPR = BN / 8;            // epilogue: 8-channel chunks per row
  static constexpr int RPI = 512 / CPR;         // epilogue rows per iteration
  static constexpr int PH = RPI > 64 ? RPI : 64;  // epilogue rows per LDS pass
  static constexpr int EPI = PH * (BN + 4) * 4;
  static constexpr int LDS = 2 * STAGE > EPI ? 2 * STAGE : EPI;
  static_assert(WAVES_M * WAVES_N == 8 && WM >= 1 && BM % PH == 0, "tile");
};

__device__ __forceinline__ int q_xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return ((xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ void q_glds16(const void* g, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_void_ptr_q)lds, 16, 0, 0);
}

// (segment, tap, channel) cursor of the K loop, current segment's geometry in
// registers (reloaded only when the cursor crosses into the next segment)
template <int NR>
struct Q32Cursor {
  const ConvOp& op;
  const int (&rb)[NR];
  const int (&ry)[NR];
  const int (&rx)[NR];
  int seg, ty, tx, c0;
  const float* src;
  int Hin, Win, cs, stride, kw, kh, dil, pad, C, kbase;

  __device__ Q32Cursor(const ConvOp& o, const int (&b)[NR], const int (&y)[NR], const int (&x)[NR])
      : op(o), rb(b), ry(y), rx(x), seg(0), ty(0), tx(0), c0(0) {
    load();
  }
  __device__ __forceinline__ void load() {
    const ConvSeg& sg = op.seg[seg];
    src = (const float*)sg.src + sg.coff;
    Hin = sg.Hin; Win = sg.Win; cs = sg.cs; stride = sg.stride; kh = sg.kh; kw = sg.kw;
    dil = sg.dil; pad = sg.pad; C = sg.C; kbase = sg.kbase;
  }
  __device__ __forceinline__ const float* a_src(int i, const float* zero) const {
    const int iy = ry[i] * stride + ty * dil - pad;
    const int ix = rx[i] * stride + tx * dil - pad;
    if (rb[i] >= 0 && (unsigned)iy < (unsigned)Hin && (unsigned)ix < (unsigned)Win)
      return src + c0 + (size_t)((rb[i] * Hin + iy) * Win + ix) * cs;
    return zero;
  }
  __device__ __forceinline__ int kb() const { return kbase + (ty * kw + tx) * C + c0; }
  __device__ __forceinline__ void advance() {
    c0 += Q_BK;
    if (c0 >= C) {
      c0 = 0;
      if (++tx >= kw) {
        tx = 0;
        if (++ty >= kh) {
          ty = 0;
          if (++seg < op.nseg) load();
        }
      }
    }
  }
};

template <int BM, int BN>
__device__ __forceinline__ void q32_epilogue(const ConvOp& op, f32x4_q (&acc)[Q32Cfg<BM, BN>::WM][Q32Cfg<BM, BN>::WN],
                                             unsigned char* smem, int m0, int n0, int M, int HW) {
  using C = Q32Cfg<BM, BN>;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % C::WAVES_M;
  const int wn = wave / C::WAVES_M;
  const int fr = lane & 15;
  const int fg = lane >> 4;
  constexpr int EST = BN + 4;
  constexpr int CPR = C::CPR, RPI = C::RPI, PH = C::PH;
  constexpr int WN = C::WN;
  float* Es = (float*)smem;
  const int col8 = tid % CPR;
  const int nch = n0 + col8 * 8;
  float bi[8], psum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bi[e] = op.bias ? op.bias[nch + e] : 0.f;
    psum[e] = 0.f;
  }
  const bool one_image = (m0 / HW) == (min(m0 + BM, M) - 1) / HW;
  const bool convt = op.store == kStoreConvT2x2;
  const float* res1 = (const float*)op.res1;
  const float* res2 = (const float*)op.res2;
  float* out = (float*)op.out;
  // (image, y, x) of the finished row, carried by RPI per iteration (no
  // per-row integer divisions; see wide_epilogue)
  int img, py, px;
  {
    const int mfirst = m0 + tid / CPR;
    img = mfirst / HW;
    const int r = mfirst - img * HW;
    py = r / op.Wo;
    px = r - py * op.Wo;
  }
  const int cout4 = op.N >> 2;
  const int cq = convt ? nch / cout4 : 0;
  const int cco = convt ? nch - cq * cout4 : 0;
  __syncthreads();  // every wave is done with the last stage
#pragma unroll 1
  for (int p = 0; p < BM / PH; ++p) {
#pragma unroll
    for (int a = 0; a < C::WM; ++a) {
      const int t16 = wm * C::WM + a;  // 16-row tile index within the block tile
      if (t16 / (PH / 16) == p) {
#pragma unroll
        for (int b = 0; b < WN; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            Es[((t16 % (PH / 16)) * 16 + fg * 4 + i) * EST + wn * WN * 16 + b * 16 + fr] = acc[a][b][i];
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PH / RPI; ++it) {
      const int row = tid / CPR + it * RPI;
      const int m = m0 + p * PH + row;
      if (p + it > 0) {
        px += RPI;
        while (px >= op.Wo) {
          px -= op.Wo;
          if (++py >= op.Ho) { py = 0; ++img; }
        }
      }
      if (m < M) {
        const f32x4_q lo = *(const f32x4_q*)(Es + row * EST + col8 * 8);
        const f32x4_q hi = *(const f32x4_q*)(Es + row * EST + col8 * 8 + 4);
        float v[8] = {lo[0] + bi[0], lo[1] + bi[1], lo[2] + bi[2], lo[3] + bi[3],
                      hi[0] + bi[4], hi[1] + bi[5], hi[2] + bi[6], hi[3] + bi[7]};
        if (op.img_bias) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += op.img_bias[img * op.N + nch + e];
        }
        if (res1) {
          const f32x4_q* r = (const f32x4_q*)(res1 + (size_t)m * op.res1_cs + nch);
          const f32x4_q r0 = r[0], r1 = r[1];
          v[0] += r0[0]; v[1] += r0[1]; v[2] += r0[2]; v[3] += r0[3];
          v[4] += r1[0]; v[5] += r1[1]; v[6] += r1[2]; v[7] += r1[3];
        }
        if (op.relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (res2) {
          const f32x4_q* r = (const f32x4_q*)(res2 + (size_t)m * op.res2_cs + nch);
          const f32x4_q r0 = r[0], r1 = r[1];
          v[0] += r0[0]; v[1] += r0[1]; v[2] += r0[2]; v[3] += r0[3];
          v[4] += r1[0]; v[5] += r1[1]; v[6] += r1[2]; v[7] += r1[3];
        }
        size_t off;
        if (convt) {
          const size_t opix = ((size_t)img * 2 * op.Ho + 2 * py + (cq >> 1)) * (2 * op.Wo) + 2 * px + (cq & 1);
          off = opix * op.out_cs + op.out_coff + cco;
        } else {
          off = (size_t)m * op.out_cs + op.out_coff + nch;
        }
        f32x4_q* o = (f32x4_q*)(out + off);
        o[0] = f32x4_q{v[0], v[1], v[2], v[3]};
        o[1] = f32x4_q{v[4], v[5], v[6], v[7]};
        if (op.pool) {
          if (one_image) {
#pragma unroll
            for (int e = 0; e < 8; ++e) psum[e] += v[e];
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) pool_add(op.pool, (size_t)img * op.N + nch + e, v[e]);
          }
        }
      }
    }
    __syncthreads();
  }
  if (op.pool && one_image && !convt) {
#pragma unroll
    for (int e = 0; e < 8; ++e) Es[(tid / CPR) * BN + col8 * 8 + e] = psum[e];
    __syncthreads();
    if (tid < BN) {
      float t = 0.f;
      for (int g = 0; g < RPI; ++g) t += Es[g * BN + tid];
      pool_add(op.pool, (size_t)(m0 / HW) * op.N + n0 + tid, t);
    }
  }
}

// Direct-store epilogue (conv_wide32_kernel<DS = true>): the main loop ran the
// MFMAs with the operands swapped (weights first), so a lane's accumulator
// tile b holds 4 consecutive fp32 CHANNELS (16 bytes) of pixel fr: bias /
// per-image bias / residuals / ReLU in registers and one 16-byte store per
// (fragment, tile) -- no LDS parking passes or block barriers.  NHWC stores;
// the per-image pool needs every pixel of the block in one image (host check).
template <int BM, int BN>
__device__ __forceinline__ void q32_direct_epilogue(const ConvOp& op,
                                                    f32x4_q (&acc)[Q32Cfg<BM, BN>::WM][Q32Cfg<BM, BN>::WN],
                                                    unsigned char* smem, int m0, int n0, int M, int HW) {
  using C = Q32Cfg<BM, BN>;
  constexpr int WM = C::WM, WN = C::WN;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % C::WAVES_M;
  const int wn = wave / C::WAVES_M;
  const int fr = lane & 15;
  const int fg = lane >> 4;
  const int cb = n0 + wn * WN * 16 + fg * 4;  // channel of tile b: cb + 16b
  const int mb = m0 + wm * WM * 16 + fr;      // pixel of fragment a: mb + 16a
  const float* res1 = (const float*)op.res1;
  const float* res2 = (const float*)op.res2;
  float* out = (float*)op.out;
  const float* rp = res1 ? res1 : res2;
  const int rcs = res1 ? op.res1_cs : op.res2_cs;
  f32x4_q rv[WM][WN];
  if (rp) {
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
      for (int b = 0; b < WN; ++b)
        rv[a][b] = mb + 16 * a < M ? *(const f32x4_q*)(rp + (size_t)(mb + 16 * a) * rcs + cb + 16 * b) : f32x4_q{};
  }
  const int img0 = m0 / HW;
  float psum[WN][4];
#pragma unroll
  for (int b = 0; b < WN; ++b)
#pragma unroll
    for (int e = 0; e < 4; ++e) psum[b][e] = 0.f;
#pragma unroll
  for (int b = 0; b < WN; ++b) {
    const int c = cb + 16 * b;
    const f32x4_q bi = op.bias ? *(const f32x4_q*)(op.bias + c) : f32x4_q{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < WM; ++a) {
      const int m = mb + 16 * a;
      if (m >= M) continue;
      f32x4_q v = acc[a][b] + bi;
      if (op.img_bias) {
        const int im = m / HW;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += op.img_bias[im * op.N + c + e];
      }
      if (res1) v += rv[a][b];
      if (op.relu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (res2) v += res1 ? *(const f32x4_q*)(res2 + (size_t)m * op.res2_cs + c) : rv[a][b];
      *(f32x4_q*)(out + (size_t)m * op.out_cs + op.out_coff + c) = v;
      if (op.pool) {
#pragma unroll
        for (int e = 0; e < 4; ++e) psum[b][e] += v[e];
      }
    }
  }
  if (op.pool) {
    // wave partials -> LDS [16 fr][WAVES_M][BN], then one thread per channel
    // adds them in a fixed order and issues one fixed-point atomic
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is done with the stages
    float* Ps = (float*)smem;
#pragma unroll
    for (int b = 0; b < WN; ++b)
#pragma unroll
      for (int e = 0; e < 4; ++e) Ps[(fr * C::WAVES_M + wm) * BN + (cb - n0) + 16 * b + e] = psum[b][e];
    __syncthreads();
    if (tid < BN) {
      float t = 0.f;
      for (int g = 0; g < 16 * C::WAVES_M; ++g) t += Ps[g * BN + tid];
      pool_add(op.pool, (size_t)img0 * op.N + n0 + tid, t);
    }
  }
}

// OCC = co-resident blocks per CU the register budget must allow (1: 256
// VGPRs; 2: 128 VGPRs, one block's prologue / epilogue overlaps the other's MFMAs)
template <int BM, int BN, bool PIPE, int OCC, bool DS = false>
__global__ __launch_bounds__(512, 2 * OCC) void conv_wide32_kernel(ConvOp op) {
  using C = Q32Cfg<BM, BN>;
  constexpr int WM = C::WM;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % C::WAVES_M;
  const int wn = wave / C::WAVES_M;

  const int M = op.B * op.Ho * op.Wo;
  const int HW = op.Ho * op.Wo;
  const int mtiles = (M + BM - 1) / BM;
  const int ntiles = op.N / BN;
  const int L = q_xcd_remap(blockIdx.x, mtiles * ntiles);
  const int ntile = L % ntiles;  // the n-tiles of one pixel tile run back to back (A reuse in L2)
  const int mtile = L / ntiles;
  const int m0 = mtile * BM;
  const int n0 = ntile * BN;

  // this lane's A rows (output pixels) for the DMA: row wave*(BM/8) + i*8 + lane/8
  const int q8 = lane >> 3;
  const int qc = lane & 7;
  int rb[C::AI], ry[C::AI], rx[C::AI];
#pragma unroll
  for (int i = 0; i < C::AI; ++i) {
    const int m = m0 + wave * (BM / 8) + i * 8 + q8;
    if (m < M) {
      const int b = m / HW, r = m - b * HW;
      rb[i] = b;
      ry[i] = r / op.Wo;
      rx[i] = r - ry[i] * op.Wo;
    } else {
      rb[i] = -1; ry[i] = 0; rx[i] = 0;
    }
  }
  // chunk stored at LDS chunk qc of row R is qc ^ ((R >> 1) & 7); A rows
  // R = (multiple of 16) + 8i + q8 -> (4i + lane >> 4) & 7
  const int sw_lane = lane >> 4;

  int total_steps = 0;
  for (int s = 0; s < op.nseg; ++s) total_steps += op.seg[s].kh * op.seg[s].kw * (op.seg[s].C / Q_BK);

  const float* Wt = (const float*)op.W;
  const float* zero = (const float*)g_w32_zero;
  Q32Cursor<C::AI> cur(op, rb, ry, rx);

  auto issue = [&](int stage) {
    unsigned char* As = smem + stage * C::STAGE;
    unsigned char* Bs = As + C::A_BYTES;
#pragma unroll
    for (int i = 0; i < C::AI; ++i) {
      const int ch = qc ^ ((4 * i + sw_lane) & 7);
      q_glds16(cur.a_src(i, zero) + ch * 4, As + (wave * (BM / 8) + i * 8) * 128);
    }
    const int kb = cur.kb();
#pragma unroll
    for (int j = 0; j < C::BJ; ++j) {
      const int t = wave + 8 * j;  // 8-row group of B rows
      if (BN / 8 >= 8 * (j + 1) || t < BN / 8) {
        const int n = t * 8 + q8;
        const int ch = qc ^ ((n >> 1) & 7);
        q_glds16(Wt + (size_t)(n0 + n) * op.Kpad + kb + ch * 4, Bs + t * 8 * 128);
      }
    }
    cur.advance();
  };

  constexpr int WN = C::WN;
  f32x4_q acc[WM][WN];
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = f32x4_q{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15;
  const int fg = lane >> 4;
  const int rsw = (fr >> 1) & 7;

  // fragments of one half step (chunk kk*4 + fg of each row)
  auto rd = [&](int buf, int kk, f32x4_q (&af)[WM], f32x4_q (&bf)[WN]) {
    const float* As = (const float*)(smem + buf * C::STAGE);
    const float* Bs = As + C::A_BYTES / 4;
    const int pc = ((kk * 4 + fg) ^ rsw) * 4;
#pragma unroll
    for (int b = 0; b < WN; ++b) bf[b] = *(const f32x4_q*)(Bs + (wn * WN * 16 + b * 16 + fr) * 32 + pc);
#pragma unroll
    for (int a = 0; a < WM; ++a) af[a] = *(const f32x4_q*)(As + (wm * WM * 16 + a * 16 + fr) * 32 + pc);
  };
  auto mm = [&](const f32x4_q (&af)[WM], const f32x4_q (&bf)[WN]) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WN; ++b) {
          if constexpr (DS)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(bf[b][e], af[a][e], acc[a][b], 0, 0, 0);
          else
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a][e], bf[b][e], acc[a][b], 0, 0, 0);
        }
  };
  // one fragment read of the next half beside each group of MFMAs of this one
  auto interleave = [&]() {
    constexpr int NR = WM + WN;
    constexpr int NM = 4 * WM * WN;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, NM / NR, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };

  f32x4_q a0[WM], b0[WN], a1[WM], b1[WN];
  if constexpr (!PIPE) {
    if (total_steps > 0) issue(0);
    for (int step = 0; step < total_steps; ++step) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (step + 1 < total_steps) issue((step + 1) & 1);
      rd(step & 1, 0, a0, b0);
      rd(step & 1, 1, a1, b1);
      mm(a0, b0);
      mm(a1, b1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    // (the host routes total_steps < 2 to the plain loop)
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(1);
    rd(0, 0, a0, b0);
    for (int step = 0; step < total_steps - 1; ++step) {
      rd(step & 1, 1, a1, b1);
      mm(a0, b0);
      interleave();
      // RAW: own DMA of step+1 retired; WAR: own reads of buffer step&1 retired
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (step + 2 < total_steps) issue(step & 1);
      rd((step + 1) & 1, 0, a0, b0);
      mm(a1, b1);
      interleave();
    }
    rd((total_steps - 1) & 1, 1, a1, b1);
    mm(a0, b0);
    mm(a1, b1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if constexpr (DS)
    q32_direct_epilogue<BM, BN>(op, acc, smem, m0, n0, M, HW);
  else
    q32_epilogue<BM, BN>(op, acc, smem, m0, n0, M, HW);
}

template <int BM, int BN, int OCC, bool DS>
static int launch_w32_k(const ConvOp& op, int steps, hipStream_t st) {
  using C = Q32Cfg<BM, BN>;
  static_assert(C::LDS * OCC <= 160 * 1024, "LDS for OCC blocks per CU");
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_wide32_kernel<BM, BN, true, OCC, DS>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)conv_wide32_kernel<BM, BN, false, OCC, DS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  const int M = op.B * op.Ho * op.Wo;
  const int grid = ((M + BM - 1) / BM) * (op.N / BN);
  if (steps >= 2)
    hipLaunchKernelGGL((conv_wide32_kernel<BM, BN, true, OCC, DS>), dim3(grid), dim3(512), C::LDS, st, op);
  else
    hipLaunchKernelGGL((conv_wide32_kernel<BM, BN, false, OCC, DS>), dim3(grid), dim3(512), C::LDS, st, op);
  return (int)hipGetLastError();
}

// direct-store epilogue: NHWC outputs (the ConvTranspose pixel shuffle keeps
// the LDS epilogue), pools only when no tile straddles two images, tiles >= 128
// channels wide.  Same-box A/B (profiles/r3_w32_ds_ab.txt): neutral on the fp32
// step (the fp32 MFMAs hide the epilogue: 27.65 -> 27.63 ms), bneck / fuse /
// enc3 s2 -1%, the 64-wide dec2 tile +1.3% (kept on the LDS epilogue).
template <int BM, int BN, int OCC>
static int launch_w32(const ConvOp& op, int steps, hipStream_t st) {
  const bool ds = BN >= 128 && op.store == kStoreNHWC && (!op.pool || (op.Ho * op.Wo) % BM == 0);
  return ds ? launch_w32_k<BM, BN, OCC, true>(op, steps, st) : launch_w32_k<BM, BN, OCC, false>(op, steps, st);
}

// fp32 only; kErrUnsupported for shapes this kernel does not take (N % 64:
// the row ring / halo kernels).
int launch_conv_wide32(const ConvOp& op, hipStream_t st) {
  if (op.store == kStoreHeadIllu || op.N % 64) return kErrUnsupported;
  if (op.store == kStoreConvT2x2 && (op.N / 4) % 8) return kErrUnsupported;
  if (op.Kpad % 4 || ((uintptr_t)op.W % 16) || op.scale) return kErrUnsupported;
  if (op.out_cs % 4 || op.out_coff % 4 || ((uintptr_t)op.out % 16)) return kErrUnsupported;
  if ((op.res1 && (op.res1_cs % 4 || (uintptr_t)op.res1 % 16)) || (op.res2 && (op.res2_cs % 4 || (uintptr_t)op.res2 % 16)))
    return kErrUnsupported;
  if (op.bias && (uintptr_t)op.bias % 16) return kErrUnsupported;
  int steps = 0;
  for (int s = 0; s < op.nseg; ++s) {
    const ConvSeg& sg = op.seg[s];
    if (sg.pre != kPreNone || sg.C % Q_BK || sg.cs % 4 || sg.coff % 4 || sg.kbase % 4) return kErrUnsupported;
    if ((uintptr_t)sg.src % 16) return kErrUnsupported;
    steps += sg.kh * sg.kw * (sg.C / Q_BK);
  }
  const bool n128 = op.N % 128 == 0;
  // Tile per width, from per-shape sweeps on MI355X (tools/r2_w32sweep.sh, bs
  // 32, fp32): 128 x 128 at two blocks per CU beats 256 x 128 at one on every
  // 128/256/512-wide GEMM of the graph (enc3 s2 121.7 -> 128.3 TF/s, ASPP d18
  // 125.8 -> 130.8, dec3 117.7 -> 127.6, ConvT dec3.up 98.8 -> 111.3); the
  // 64-wide convs run best as 256 x 64 (dec2 / enc1.conv2 117 TF/s, 512 x 64
  // 99.6, 128 x 64 115.7).
  if (n128) return launch_w32<128, 128, 2>(op, steps, st);
  return launch_w32<256, 64, 1>(op, steps, st);
}

}  // namespace upr
