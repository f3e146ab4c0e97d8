// Wide-tile implicit-GEMM convolution, fp16 operands / fp32 accumulate, for the
// MFMA-bound layers of the UP-Retinex graph (>= 64 input channels, >= 128
// output channels: encoder blocks 2-3, bottleneck ResBlocks, ASPP branches and
// fusion, decoder 3 and the ConvTranspose GEMMs; models/model.py:100-274).
//
// Why a second GEMM kernel: the 128x128 register-staged tiles of conv.hip and
// the 128-pixel halo tiles of conv_halo.hip move ~64 B/clk/CU of operands at
// full MFMA rate, which the L2 cannot feed.  Here:
//
// * Tile 256 pixels x BN (256 or 128) channels, 8 waves (512 threads); each wave
//   owns a 128x64 (BN 256) or 64x64 (BN 128) accumulator block of
//   v_mfma_f32_16x16x32_f16 tiles -> half the operand bytes per flop.
// * K step = 64 channels of one tap of one segment.  Both operands go global ->
//   LDS by LDS-DMA (global_load_lds_dwordx4): no staging registers, no
//   ds_write pass.  A is a per-lane gather (each lane's source is its output
//   pixel shifted by the tap; out-of-image taps and rows past M read a
//   128-byte zero line), B rows are the packed [N][Kpad] weights.
// * Two LDS stages, one barrier per K step: the DMA of step s+1 is issued right
//   after the barrier and flies while the MFMAs of step s run.  The fragments
//   of the second 32-deep half of step s are read before the barrier and its
//   MFMAs run after it (half-step software pipeline), so the MFMA pipe stays
//   busy across the barrier and the next step's first fragment reads; the
//   fragment reads of one half are interleaved with the MFMAs of the other
//   (sched_group_barrier), which also keeps the wave at 254 VGPRs, no spills.
// * The (segment, tap, channel) cursor keeps the current segment's geometry in
//   registers (no kernarg loads in the K loop).
// * Measured on bneck (bs 32, 64x64x256 -> 256, 3x3): 0.189 ms = 820 TF/s; with
//   both DMAs removed (timing ablation) 0.119 ms = 1300 TF/s, i.e. ~1/3 of the
//   time is operand traffic; a 4-stage 32-deep ring (three steps of DMA in
//   flight across each barrier) measured 3-8% SLOWER (twice the per-step
//   overhead for no latency it could still hide).
// * LDS image: 128-byte rows (64 fp16), lane-linear as LDS-DMA requires; the
//   16-byte chunk index is XOR-swizzled by (row >> 1) & 7 on the SOURCE
//   address, and the fragment reads apply the same XOR -> the ds_read_b128
//   lane groups hit 16 distinct bank slots (conflict free).
//
// Segments must be plain (no pre-activation / max-pool prologue: those need
// register staging and stay on conv.hip / conv_halo.hip), C % 64 == 0.
#include <cstdlib>
#include <cstring>
#include <utility>

#include "upr_common.h"
#include "wide_common.h"

namespace upr {


// 128 zero bytes: the source of every padded / out-of-range A chunk
__device__ __attribute__((aligned(128))) uint4 g_wide_zero[8];


template <int BN>
struct WideCfg {
  static constexpr int WAVES_M = BN == 256 ? 2 : 4;
  static constexpr int WAVES_N = 8 / WAVES_M;
  static constexpr int WM = WBM / WAVES_M / 16;  // 16x16 tiles per wave along M
  static constexpr int WN = BN / WAVES_N / 16;   // along N
  static constexpr int A_BYTES = WBM * WBK * 2;
  static constexpr int B_BYTES = BN * WBK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int LDS = 2 * STAGE;
  static constexpr int BJ = BN / 64;  // B DMA instructions per wave per step (8 rows each)
};

// (segment, tap, channel) cursor of the K loop with the current segment's
// geometry held in registers: the per-step DMA issue needs no kernarg loads
// (a dynamically indexed op.seg[] read is a scalar load + lgkmcnt wait in
// every step), only a reload when the cursor crosses into the next segment.
template <int NR, int BK>
struct SegCursor {
  const ConvOp& op;
  const int (&rb)[NR];  // per lane row: image (-1 = past M), output row, output column
  const int (&ry)[NR];
  const int (&rx)[NR];
  const int chunk;
  int seg, ty, tx, c0;
  const half_t* src;
  int Hin, Win, cs, stride, kh, kw, dil, pad, C, kbase;

  __device__ SegCursor(const ConvOp& o, const int (&b)[NR], const int (&y)[NR], const int (&x)[NR], int ch)
      : op(o), rb(b), ry(y), rx(x), chunk(ch), seg(0), ty(0), tx(0), c0(0) {
    load();
  }
  __device__ __forceinline__ void load() {
    const ConvSeg& sg = op.seg[seg];
    src = (const half_t*)sg.src + sg.coff + chunk * 8;
    Hin = sg.Hin; Win = sg.Win; cs = sg.cs; stride = sg.stride; kh = sg.kh; kw = sg.kw;
    dil = sg.dil; pad = sg.pad; C = sg.C; kbase = sg.kbase;
  }
  // source of row i at the current (tap, c0); `zero` when padded / past M
  __device__ __forceinline__ const half_t* a_src(int i, const half_t* zero) const {
    const int iy = ry[i] * stride + ty * dil - pad;
    const int ix = rx[i] * stride + tx * dil - pad;
    if (rb[i] >= 0 && (unsigned)iy < (unsigned)Hin && (unsigned)ix < (unsigned)Win)
      return src + c0 + (size_t)((rb[i] * Hin + iy) * Win + ix) * cs;
    return zero;
  }
  __device__ __forceinline__ int kb() const { return kbase + (ty * kw + tx) * C + c0; }
  __device__ __forceinline__ void advance() {
    c0 += BK;
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

// Epilogue shared by the wide kernels: 256 x BN accumulator tile -> LDS ->
// scale / bias / per-image bias / residuals / ReLU -> 16-byte fp16 stores.
// RPF: the tile's residual rows (res1, else res2) are loaded into registers
// before the accumulators are parked -- one batch of independent loads
// instead of one exposed HBM round trip per 16-byte store (a residual cost
// the bottleneck / dec3 convs 10-25% of their time)
template <int BN, int WM, int WN, int WAVES_M, int BM = WBM, bool RPF = false, int QW = 0>
__device__ __forceinline__ void wide_epilogue(const ConvOp& op, f32x4_w (&acc)[WM][WN], unsigned char* smem, int m0,
                                              int n0, int M, int HW) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WAVES_M;
  const int wn = wave / WAVES_M;
  const int fr = lane & 15;
  const int fg = lane >> 4;
  // ---- epilogue through LDS ---------------------------------------------------
  // BM / 64 passes of 64 tile rows: the waves owning those rows park their raw
  // fp32 accumulators in LDS ([64][BN + 4] floats: conflict-free 4-byte
  // writes), then every thread finishes 8 consecutive channels of one pixel
  // per iteration (scale / bias / per-image bias / residuals / ReLU, 16-byte
  // loads and stores).  With 512 threads and BN/8 chunks per row, a thread's
  // channel chunk is the same in every iteration, so the per-image pooled sums
  // (ASPP global branch) stay in registers until the end.
  constexpr int EST = BN + 4;
  constexpr int CPR = BN / 8;             // 8-channel chunks per row
  constexpr int RPI = 512 / CPR;          // rows per iteration
  constexpr int APP = 4;                  // 16-row accumulator tiles per pass
  constexpr int PPW = WM / APP;        // passes per wave-row group
  float* Es = (float*)smem;
  const int col8 = tid % CPR;
  const int nch = n0 + col8 * 8;
  // scale / bias are re-read per row (L1 hits) rather than held: with the
  // accumulators of the later passes still live, 16 more registers spill
  float psum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) psum[e] = 0.f;
  const bool one_image = (m0 / HW) == (min(m0 + BM, M) - 1) / HW;
  const bool convt = op.store == kStoreConvT2x2;
  // the row a thread finishes advances by exactly RPI per iteration (passes of
  // 64 rows, 64 / RPI iterations each): (image, y, x) of that row are carried
  // along instead of divided out per row (three integer divisions per
  // 16-byte store made the K = 64 ConvTranspose GEMM VALU-bound)
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
  constexpr int NQ = RPF ? BM / RPI : 1;  // rows this thread finishes (q = p * 64 / RPI + it)
  const half_t* rpf = (const half_t*)(op.res1 ? op.res1 : op.res2);
  const int rpf_cs = op.res1 ? op.res1_cs : op.res2_cs;
  f16x8_w rv[NQ];
  if (RPF && rpf) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int m = m0 + tid / CPR + q * RPI;
      rv[q] = m < M ? *(const f16x8_w*)(rpf + (size_t)m * rpf_cs + nch) : f16x8_w{};
    }
  }
  __syncthreads();  // every wave is done with the last stage
#pragma unroll
  for (int p = 0; p < BM / 64; ++p) {
    if constexpr (QW == 0) {
      if (wm == p / PPW) {
#pragma unroll
        for (int a = 0; a < APP; ++a)
#pragma unroll
          for (int b = 0; b < WN; ++b)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              Es[(a * 16 + fg * 4 + i) * EST + wn * WN * 16 + b * 16 + fr] = acc[(p % PPW) * APP + a][b][i];
      }
    } else {
      // column-block wave mapping (conv_hwide4_kernel): wave wm owns columns
      // [CW*wm, CW*wm + CW) of every image row of the tile, fragment a = image
      // row a / FPR, columns CW*wm + (a % FPR)*16 ..; pass p = tile pixels
      // [64p, 64p + 64) = image row 64p / QW, columns from (64p) % QW
      constexpr int CW = QW / WAVES_M;
      constexpr int FPR = CW / 16;
      const int rr = (p * 64) / QW, cb = (p * 64) % QW;
#pragma unroll
      for (int a = 0; a < WM; ++a) {
        if (a / FPR != rr) continue;
        const int col = CW * wm + (a % FPR) * 16 - cb;
        if (col >= 0 && col < 64) {
#pragma unroll
          for (int b = 0; b < WN; ++b)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              Es[(col + fg * 4 + i) * EST + wn * WN * 16 + b * 16 + fr] = acc[a][b][i];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 64 / RPI; ++it) {
      const int row = tid / CPR + it * RPI;
      const int m = m0 + p * 64 + row;
      if (p + it > 0) {
        px += RPI;
        while (px >= op.Wo) {
          px -= op.Wo;
          if (++py >= op.Ho) { py = 0; ++img; }
        }
      }
      if (m < M) {
        const f32x4_w lo = *(const f32x4_w*)(Es + row * EST + col8 * 8);
        const f32x4_w hi = *(const f32x4_w*)(Es + row * EST + col8 * 8 + 4);
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        if (op.scale) {
          const f32x4_w s0 = *(const f32x4_w*)(op.scale + nch), s1 = *(const f32x4_w*)(op.scale + nch + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) { v[e] *= s0[e]; v[e + 4] *= s1[e]; }
        }
        if (op.bias) {
          const f32x4_w b0 = *(const f32x4_w*)(op.bias + nch), b1 = *(const f32x4_w*)(op.bias + nch + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) { v[e] += b0[e]; v[e + 4] += b1[e]; }
        }
        if (op.img_bias) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += op.img_bias[img * op.N + nch + e];
        }
        const int q = RPF ? p * (64 / RPI) + it : 0;
        if (op.res1) {
          const f16x8_w r = RPF ? rv[q] : *(const f16x8_w*)((const half_t*)op.res1 + (size_t)m * op.res1_cs + nch);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)r[e];
        }
        if (op.relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (op.res2) {
          const f16x8_w r = RPF && !op.res1 ? rv[q] : *(const f16x8_w*)((const half_t*)op.res2 + (size_t)m * op.res2_cs + nch);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)r[e];
        }
        f16x8_w o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (half_t)v[e];
        // output pixel and its channel offset
        size_t pix;
        int ch;
        if (convt) {
          pix = ((size_t)img * 2 * op.Ho + 2 * py + (cq >> 1)) * (2 * op.Wo) + 2 * px + (cq & 1);
          ch = cco;
        } else {
          pix = (size_t)m;
          ch = nch;
        }
        if (op.out32) {
          float* d32 = op.out32 + pix * op.out32_cs + op.out32_coff + ch;
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {  // one 16-byte half at a time (register pressure of the 128-VGPR variant)
            f32x4_w t;
#pragma unroll
            for (int e = 0; e < 4; ++e) t[e] = (float)o[hh * 4 + e];
            if (op.res32) t += *(const f32x4_w*)(op.res32 + pix * op.res32_cs + ch + hh * 4);
            if (op.mask16) {
              typedef _Float16 h4m __attribute__((ext_vector_type(4)));
              const h4m mk = *(const h4m*)((const half_t*)op.mask16 + pix * op.mask16_cs + ch + hh * 4);
#pragma unroll
              for (int e = 0; e < 4; ++e) t[e] = (float)mk[e] > 0.f ? t[e] : 0.f;
            }
            if (!op.skip32) *(f32x4_w*)(d32 + hh * 4) = t;
            if (op.out32_h16) {
              typedef _Float16 h4w __attribute__((ext_vector_type(4)));
              *(h4w*)((half_t*)op.out32_h16 + pix * op.out32_h16_cs + ch + hh * 4) =
                  h4w{(half_t)t[0], (half_t)t[1], (half_t)t[2], (half_t)t[3]};
            }
          }
        } else {
          *(f16x8_w*)((half_t*)op.out + pix * op.out_cs + op.out_coff + ch) = o;
        }
        if (op.out2) {
          const f32x4_w s0 = *(const f32x4_w*)(op.pre2_scale + nch), s1 = *(const f32x4_w*)(op.pre2_scale + nch + 4);
          const f32x4_w h0 = *(const f32x4_w*)(op.pre2_shift + nch), h1 = *(const f32x4_w*)(op.pre2_shift + nch + 4);
          f16x8_w q;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            q[e] = (half_t)fmaxf(__builtin_fmaf((float)o[e], s0[e], h0[e]), 0.f);
            q[e + 4] = (half_t)fmaxf(__builtin_fmaf((float)o[e + 4], s1[e], h1[e]), 0.f);
          }
          *(f16x8_w*)((half_t*)op.out2 + (size_t)m * op.out2_cs + nch) = q;
        }
        if (op.pool) {
          if (one_image) {
#pragma unroll
            for (int e = 0; e < 8; ++e) psum[e] += (float)o[e];
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) pool_add(op.pool, (size_t)img * op.N + nch + e, (float)o[e]);
          }
        }
      }
    }
    __syncthreads();
  }
  if (op.pool && one_image && !convt) {
    // block-level reduction of the RPI partial sums per channel through LDS
    // (the last pass ended with a barrier), then ONE atomic per channel: the
    // pooled vector of an image is hit by HW/256 tiles, not by 16x that many
    // per-wave atomics (contended same-address atomics serialise)
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

// MINW: minimum waves per SIMD (HIP's second launch-bounds argument); 4 = two
// 512-thread blocks per CU
// (MINW 4 also selects ONE LDS stage: load -> compute per step, the other
// block on the CU overlapping)
// DS: operand-swapped MFMAs, B rows DMA'd in hw4_perm32 order and the
// direct-store epilogue (wide_ds_ok decides per op)
template <int BN, bool PIPE, int MINW = 2, int SCHED = 0, bool DS = false>
__global__ __launch_bounds__(512, MINW) void conv_wide_kernel(ConvOp op) {
  constexpr bool ONE = MINW >= 4;
  using C = WideCfg<BN>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % C::WAVES_M;
  const int wn = wave / C::WAVES_M;

  const int M = op.B * op.Ho * op.Wo;
  const int HW = op.Ho * op.Wo;
  const int mtiles = (M + WBM - 1) / WBM;
  const int ntiles = op.N / BN;
  const int L = wide_xcd_remap(blockIdx.x, mtiles * ntiles);
  const int ntile = L % ntiles;  // the n-tiles of one pixel tile run back to back (A reuse in L2)
  const int mtile = L / ntiles;
  const int m0 = mtile * WBM;
  const int n0 = ntile * BN;

  // ---- this lane's 4 A rows (output pixels) and DMA chunk swizzles ---------
  const int q8 = lane >> 3;       // row within an 8-row DMA group
  const int qc = lane & 7;        // LDS chunk this lane fills
  int rb[4], ry[4], rx[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wave * 32 + i * 8 + q8;
    if (m < M) {
      const int b = m / HW, r = m - b * HW;
      rb[i] = b;
      ry[i] = r / op.Wo;
      rx[i] = r - ry[i] * op.Wo;
    } else {
      rb[i] = -1; ry[i] = 0; rx[i] = 0;
    }
  }
  // logical chunk stored at LDS chunk qc of row R is qc ^ ((R >> 1) & 7); for
  // R = wave*32 + i*8 + q8 (A) or wave*BN/8 + j*8 + q8 (B) that is (4i + lane>>4) & 7
  const int sw_lane = lane >> 4;

  int total_steps = 0;
  for (int s = 0; s < op.nseg; ++s) total_steps += op.seg[s].kh * op.seg[s].kw * (op.seg[s].C / WBK);

  const half_t* Wt = (const half_t*)op.W;
  const half_t* zero = (const half_t*)g_wide_zero;
  // the 4 rows share the chunk swizzle pattern per i: chunk = qc ^ ((4i + lane>>4) & 7)
  SegCursor<4, WBK> cur(op, rb, ry, rx, 0);

  auto issue = [&](int stage) {
    unsigned char* As = smem + stage * C::STAGE;
    unsigned char* Bs = As + C::A_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = qc ^ ((4 * i + sw_lane) & 7);
      glds16(cur.a_src(i, zero) + ch * 8, As + (wave * 32 + i * 8) * 128);
    }
    const int kb = cur.kb();
#pragma unroll
    for (int j = 0; j < C::BJ; ++j) {
      const int n = wave * (BN / 8) + j * 8 + q8;
      const int ch = qc ^ ((4 * j + sw_lane) & 7);
      glds16(Wt + (size_t)(n0 + (DS ? hw4_perm32(n) : n)) * op.Kpad + kb + ch * 8, Bs + (wave * (BN / 8) + j * 8) * 128);
    }
    cur.advance();
  };

  f32x4_w acc[C::WM][C::WN];
#pragma unroll
  for (int a = 0; a < C::WM; ++a)
#pragma unroll
    for (int b = 0; b < C::WN; ++b) acc[a][b] = f32x4_w{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15;
  const int fg = lane >> 4;
  const int rsw = (fr >> 1) & 7;  // swizzle of every fragment row this lane reads

  if constexpr (!PIPE) {
    if (total_steps > 0) issue(0);
    for (int step = 0; step < total_steps; ++step) {
      // stage step&1 has landed (own DMA retired, then everyone's via the
      // barrier) and every wave is done reading the other stage (step-1)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (!ONE && step + 1 < total_steps) issue((step + 1) & 1);
      const half_t* As = (const half_t*)(smem + (ONE ? 0 : (step & 1)) * C::STAGE);
      const half_t* Bs = As + C::A_BYTES / 2;
  #pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int pc = ((kk * 4 + fg) ^ rsw) * 8;
        f16x8_w bf[C::WN];
  #pragma unroll
        for (int b = 0; b < C::WN; ++b) bf[b] = *(const f16x8_w*)(Bs + (wn * C::WN * 16 + b * 16 + fr) * 64 + pc);
  #pragma unroll
        for (int a = 0; a < C::WM; ++a) {
          const f16x8_w af = *(const f16x8_w*)(As + (wm * C::WM * 16 + a * 16 + fr) * 64 + pc);
  #pragma unroll
          for (int b = 0; b < C::WN; ++b) {
            if constexpr (DS)
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[b], af, acc[a][b], 0, 0, 0);
            else
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[b], acc[a][b], 0, 0, 0);
          }
        }
      }
      if (ONE && step + 1 < total_steps) {
        __syncthreads();  // every wave is done reading the single stage
        issue(0);
      }
    }
  } else {
    // Half-step software pipeline: the fragments of the second 32-deep half
    // of step s are read BEFORE the barrier that releases step s+1, and the
    // MFMAs of that half run AFTER it, so the MFMA pipe stays busy across the
    // barrier, the DMA issue and the first fragment reads of step s+1.
    // WAR: each wave retires its reads of buffer s&1 (lgkmcnt(0)) before the
    // barrier after which buffer s&1 is refilled.  RAW: own DMA of step s+1
    // retired (vmcnt(0)) before that same barrier.
    f16x8_w a0[C::WM], b0[C::WN], a1[C::WM], b1[C::WN];
    auto rd = [&](int buf, int kk, f16x8_w (&af)[C::WM], f16x8_w (&bf)[C::WN]) {
      const half_t* As = (const half_t*)(smem + buf * C::STAGE);
      const half_t* Bs = As + C::A_BYTES / 2;
      const int pc = ((kk * 4 + fg) ^ rsw) * 8;
#pragma unroll
      for (int b = 0; b < C::WN; ++b) bf[b] = *(const f16x8_w*)(Bs + (wn * C::WN * 16 + b * 16 + fr) * 64 + pc);
#pragma unroll
      for (int a = 0; a < C::WM; ++a) af[a] = *(const f16x8_w*)(As + (wm * C::WM * 16 + a * 16 + fr) * 64 + pc);
    };
    auto mm = [&](const f16x8_w (&af)[C::WM], const f16x8_w (&bf)[C::WN]) {
#pragma unroll
      for (int a = 0; a < C::WM; ++a)
#pragma unroll
        for (int b = 0; b < C::WN; ++b) {
          if constexpr (DS)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[b], af[a], acc[a][b], 0, 0, 0);
          else
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
    };
    // (the host routes total_steps < 2 to the plain loop)
    // ds_read / MFMA interleave of one half-step: one A fragment (and, for the
    // first four, one B fragment) of the next half between each group of WN
    // MFMAs, so the fragments of the half being consumed free registers as the
    // next half's arrive
    auto interleave = [&]() {
      if constexpr (SCHED == 2) {
        // one fragment read after every two MFMAs, VALU between (measured on the halo-wide kernel)
#pragma unroll
        for (int a = 0; a < (C::WM * C::WN) / 2; ++a) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
      } else {
#pragma unroll
        for (int a = 0; a < C::WN; ++a) {
          __builtin_amdgcn_sched_group_barrier(0x008, C::WN, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
#pragma unroll
        for (int a = C::WN; a < C::WM; ++a) {
          __builtin_amdgcn_sched_group_barrier(0x008, C::WN, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
    };
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(1);
    rd(0, 0, a0, b0);
    for (int step = 0; step < total_steps - 1; ++step) {
      rd(step & 1, 1, a1, b1);
      mm(a0, b0);
      interleave();
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      issue(step & 1);  // step + 2 (past the end: a harmless re-read into a buffer nobody reads again)
      rd((step + 1) & 1, 0, a0, b0);
      mm(a1, b1);
      interleave();
    }
    rd((total_steps - 1) & 1, 1, a1, b1);
    mm(a0, b0);
    mm(a1, b1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (!DS) __syncthreads();  // every wave is done with both stages before the epilogue reuses LDS
  }

  if constexpr (DS) {
    // (no pool in this form: the LDS is not reused, no barrier)
    f16x8_w rv0[C::WM];
    const int mb = m0 + wm * C::WM * 16 + (lane & 15);
    direct_epilogue<BN, C::WM, C::WN, C::WAVES_M, false>(
        op, acc, n0, wm, wn, lane, rv0, smem, [&](int a) { return mb + a * 16; }, M, HW, -1);
  } else {
    wide_epilogue<BN, C::WM, C::WN, C::WAVES_M, WBM, !ONE>(op, acc, smem, m0, n0, M, HW);
  }
}

// ---------------------------------------------------------------------------
// Halo-tiled A operand: stride-1 3x3 (dilation 1) single-segment convs whose
// 256-pixel tile is whole image rows (W = 64: 4 rows, W = 128: 2 rows) --
// the bottleneck ResBlock convs (64^2 x 256) and the dec3 UpBlock convs
// (128^2 x 128), models/model.py:100-178, :261-269.
//
// The gathered-A kernel above DMAs every input pixel 9 times (once per tap)
// from L2; with both operands at 32 KB per K step the L2 -> LDS gather (~70
// GB/s per CU) and the MFMAs run at about the same rate and serialise.  Here
// the K loop is chunk-major, tap-minor: the tile's input REGION (its TR
// output rows plus the two halo rows, W pixels wide) of one 64-channel chunk
// is DMA'd once, and the 9 taps read their A fragments from it at a per-tap
// pixel offset.  A traffic per chunk: 48 KB (W 64) / 64 KB (W 128) instead of
// 9 x 32 KB.
// * LDS: two region buffers (chunk parity) + two B stages = 160 KiB for
//   (BN 256, W 64) and (BN 128, W 128).  The next chunk's region is DMA'd one
//   1-KiB piece per wave per step during the first RI taps of the current
//   chunk; B is double-buffered per step as in the gathered kernel, and the
//   same half-step software pipeline runs across the one barrier per step.
// * A region pixel is a 128-byte LDS row; its logical 16-byte chunk q sits at
//   q ^ T[p & 15].  The tap shift starts a fragment's 16 pixels at p = 16k +
//   tx (tx in {-1, 0, 1}); T (exhaustive search over the ds_read_b128 lane
//   groups {0-3,12-15,20-27}, ...) keeps every shift conflict-free, where
//   the aligned-row swizzle (p >> 1) & 7 would be 2-way at tx = +-1.  The
//   first table (0,0,1,2,2,0,4,4,5,5,6,2,2,6,6,7) covered shifts -1 / 0 / +1
//   only; the dilated hwide4 reads at +-6 / 12 / 18 conflicted (PMC
//   SQ_LDS_BANK_CONFLICT 5.5-6.3M cycles per ASPP launch).  T[p] = 2((p >> 1) & 3)
//   is conflict-free at all 16 start offsets (tools/halo_swz_search.py).
// * No padding columns: the one lane of an edge fragment whose tap leaves
//   the image row is zeroed after the read (top / bottom halo rows outside
//   the image are DMA'd from the zero line).
// ---------------------------------------------------------------------------
constexpr unsigned long long kHaloSwz = 0x6644220066442200ull;  // T[p] = 0,0,2,2,4,4,6,6,0,0,2,2,4,4,6,6
__device__ __forceinline__ int halo_swz(int p) { return (int)(kHaloSwz >> ((p & 15) * 4)) & 7; }

template <int BN, int W>
struct HaloCfg {
  using C = WideCfg<BN>;
  static constexpr int TR = WBM / W;        // output rows per tile
  static constexpr int RPX = (TR + 2) * W;  // region pixels
  static constexpr int R_BYTES = RPX * 128;
  static constexpr int RI = RPX / 64;       // region DMA pieces per wave per chunk
  static constexpr int LDS = 2 * R_BYTES + 2 * C::B_BYTES;
  // wave row offsets (wm * WM * 16) are multiples of GW modulo W: fragment a
  // can start a row (left edge) only if a * 16 % GW == 0
  static constexpr int GW = (C::WM * 16) % W == 0 ? W : (C::WM * 16) % W;
  static_assert(LDS <= 163840, "LDS");
  static_assert(RI <= 8, "a chunk's region pieces go out during taps 0..RI-1 of the previous chunk");
  static_assert(W % 16 == 0 && WBM % W == 0, "tiles of whole rows");
};

template <int BN, int W>
__global__ __launch_bounds__(512, 2) void conv_hwide_kernel(ConvOp op) {
  using C = WideCfg<BN>;
  using HC = HaloCfg<BN, W>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % C::WAVES_M;
  const int wn = wave / C::WAVES_M;

  const int HW = op.Ho * W;
  const int M = op.B * HW;
  const int mtiles = M / WBM;
  const int ntiles = op.N / BN;
  const int L = wide_xcd_remap(blockIdx.x, mtiles * ntiles);
  const int ntile = L % ntiles;
  const int mtile = L / ntiles;
  const int m0 = mtile * WBM;
  const int n0 = ntile * BN;
  const int img = m0 / HW;
  const int oy0 = (m0 - img * HW) / W;
  const ConvSeg& sg = op.seg[0];
  const int cs = sg.cs, Cin = sg.C, H = op.Ho;
  const int nchunks = Cin / WBK;
  const int total = nchunks * 9;
  const half_t* zero = (const half_t*)g_wide_zero;

  // region DMA: piece i of wave w covers region pixels (8i + w) * 8 .. +7; lane
  // -> pixel w * 8 + lane / 8 of the 64-pixel slab, logical chunk (lane & 7) ^ T[p]
  const int rpx = wave * 8 + (lane >> 3);
  const half_t* rsrc =
      (const half_t*)sg.src + sg.coff + ((size_t)img * HW + rpx) * cs + (((lane & 7) ^ halo_swz(rpx)) * 8);
  auto region_piece = [&](int c, int i) {
    const int r = i * 64 / W, col = i * 64 % W;
    const int iy = oy0 - 1 + r;
    const half_t* g = (unsigned)iy < (unsigned)H ? rsrc + ((size_t)iy * W + col) * cs + c * WBK : zero;
    glds16(g, smem + (c & 1) * HC::R_BYTES + (i * 8 + wave) * 1024);
  };

  const int q8 = lane >> 3;
  const int qc = lane & 7;
  const int sw_lane = lane >> 4;
  const half_t* Wt = (const half_t*)op.W;
  auto issue_b = [&](int buf, int c, int t) {
    unsigned char* Bs = smem + 2 * HC::R_BYTES + buf * C::B_BYTES;
    const int kb = sg.kbase + t * Cin + c * WBK;
#pragma unroll
    for (int j = 0; j < C::BJ; ++j) {
      const int n = wave * (BN / 8) + j * 8 + q8;
      const int ch = qc ^ ((4 * j + sw_lane) & 7);
      glds16(Wt + (size_t)(n0 + n) * op.Kpad + kb + ch * 8, Bs + (wave * (BN / 8) + j * 8) * 128);
    }
  };

  f32x4_w acc[C::WM][C::WN];
#pragma unroll
  for (int a = 0; a < C::WM; ++a)
#pragma unroll
    for (int b = 0; b < C::WN; ++b) acc[a][b] = f32x4_w{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15;
  const int fg = lane >> 4;
  const int rsw = (fr >> 1) & 7;
  const bool lane_l = fr == 0, lane_r = fr == 15;
  // fragments of read step (c, t): B from stage bbuf, A from region c & 1 at tap (t / 3, t % 3)
  auto rd = [&](int bbuf, int c, int ty, int tx, int kk, f16x8_w (&af)[C::WM], f16x8_w (&bf)[C::WN]) {
    const half_t* Bs = (const half_t*)(smem + 2 * HC::R_BYTES + bbuf * C::B_BYTES);
    const int pc = ((kk * 4 + fg) ^ rsw) * 8;
#pragma unroll
    for (int b = 0; b < C::WN; ++b) bf[b] = *(const f16x8_w*)(Bs + (wn * C::WN * 16 + b * 16 + fr) * 64 + pc);
    const int p = fr + tx - 1;  // lane pixel relative to the fragment's first output pixel
    const unsigned char* Rs = smem + (c & 1) * HC::R_BYTES + p * 128 + (((kk * 4 + fg) ^ halo_swz(p)) * 16);
    const bool zl = tx == 0 && lane_l, zr = tx == 2 && lane_r;
#pragma unroll
    for (int a = 0; a < C::WM; ++a) {
      const int m = wm * C::WM * 16 + a * 16;
      const int oy = m / W, ox = m % W;
      f16x8_w v = *(const f16x8_w*)(Rs + ((oy + ty) * W + ox) * 128);
      if ((a * 16) % HC::GW == 0) {
        if (zl && ox == 0) v = f16x8_w{};
      }
      if ((a * 16 + 16) % HC::GW == 0) {
        if (zr && ox == W - 16) v = f16x8_w{};
      }
      af[a] = v;
    }
  };
  auto mm = [&](const f16x8_w (&af)[C::WM], const f16x8_w (&bf)[C::WN]) {
#pragma unroll
    for (int a = 0; a < C::WM; ++a)
#pragma unroll
      for (int b = 0; b < C::WN; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a], bf[b], acc[a][b], 0, 0, 0);
  };
  auto interleave = [&]() {
#pragma unroll
    for (int a = 0; a < C::WN; ++a) {
      __builtin_amdgcn_sched_group_barrier(0x008, C::WN, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
#pragma unroll
    for (int a = C::WN; a < C::WM; ++a) {
      __builtin_amdgcn_sched_group_barrier(0x008, C::WN, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };

  // step cursors: (chunk, tap row, tap column) of the read step and of the B DMA
  int rc = 0, ry = 0, rx = 0;
  int bc = 0, by = 0, bx = 1;
  auto adv = [](int& c, int& y, int& x) {
    if (++x == 3) {
      x = 0;
      if (++y == 3) { y = 0; ++c; }
    }
  };
  f16x8_w a0[C::WM], b0[C::WN], a1[C::WM], b1[C::WN];
#pragma unroll
  for (int i = 0; i < HC::RI; ++i) region_piece(0, i);
  issue_b(0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  issue_b(1, bc, by * 3 + bx);
  adv(bc, by, bx);
  if (nchunks > 1) region_piece(1, 0);
  rd(0, rc, ry, rx, 0, a0, b0);
  for (int step = 0; step < total - 1; ++step) {
    rd(step & 1, rc, ry, rx, 1, a1, b1);
    mm(a0, b0);
    interleave();
    // RAW: own DMA (B of step + 1, region pieces) retired before the barrier;
    // WAR: own reads of B stage step & 1 (and of region (c - 1) & 1) retired
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    adv(rc, ry, rx);  // read cursor -> step + 1
    if (step + 2 < total) {
      issue_b(step & 1, bc, by * 3 + bx);
      adv(bc, by, bx);
    }
    const int t = ry * 3 + rx;
    if (t < HC::RI && rc + 1 < nchunks) region_piece(rc + 1, t);
    rd((step + 1) & 1, rc, ry, rx, 0, a0, b0);
    mm(a1, b1);
    interleave();
  }
  rd((total - 1) & 1, rc, ry, rx, 1, a1, b1);
  mm(a0, b0);
  mm(a1, b1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave is done with the regions and stages before the epilogue reuses LDS

  wide_epilogue<BN, C::WM, C::WN, C::WAVES_M>(op, acc, smem, m0, n0, M, HW);
}

template <int BN, int W>
static int launch_hwide(const ConvOp& op, hipStream_t st) {
  using HC = HaloCfg<BN, W>;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute((const void*)conv_hwide_kernel<BN, W>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, HC::LDS);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  const int grid = (op.B * op.Ho * W / WBM) * (op.N / BN);
  hipLaunchKernelGGL((conv_hwide_kernel<BN, W>), dim3(grid), dim3(512), HC::LDS, st, op);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Halo A with a region ROW RING and three B stages (BN 256, W 64: the 64^2 x
// 256-channel bottleneck convs).  The two-stage form above waits for each
// step's B DMA within one step (vmcnt(0) before every barrier); measured on
// bneck, its B DMA alone costs 10% (no-B-DMA ablation 0.170 -> 0.153 ms) and
// all DMA 27% (-> 0.124).  Here:
// * Region rows live in an 8-row ring (64 KB) instead of two 6-row buffers
//   (96 KB): chunk c's region row r is ring row (6c + r) & 7, so the next
//   chunk's rows 0-3 reuse the two spare rows and chunk c's rows 0 / 1 once
//   taps 0-2 / 3-5 are done, and its rows 4 / 5 overwrite chunk c's rows 2 /
//   3 at the start of the next chunk (needed from taps 3 / 6 on).
// * The freed 32 KB hold a third B stage: B(s + 3) goes out after barrier s,
//   and the wait before barrier s leaves the previous iteration's DMAs in
//   flight (counted vmcnt, never 0 in the loop): two steps of lookahead for
//   every operand.
// * Edge masks (tap column outside the image row) are applied to the A
//   fragments right before their MFMAs, not at the read (a select on freshly
//   read registers stalls the wave on the LDS read).
// ---------------------------------------------------------------------------
// TR_ = output rows per tile: 4 (the 8-row ring over several chunks), or 2
// for one 64-channel chunk at W 256 (hwide4 only: its 4 region rows are the
// whole "ring", DMA'd in the prologue)
// RR_: ring rows when not the default (the pointwise form: 12 = three chunks' 4 rows)
template <int BN, int W, int TR_ = 4, int RR_ = 0>
struct Halo3Cfg {
  static constexpr int TR = TR_;             // output rows per tile
  static constexpr int BM = TR * W;          // 256 (W 64) / 512 (W 128, W 256 x 2 rows) pixels
  static constexpr int WAVES_N = BN / 64;    // each wave: BM / WAVES_M pixels x 64 channels
  static constexpr int WAVES_M = 8 / WAVES_N;
  static constexpr int WM = BM / WAVES_M / 16, WN = BN / WAVES_N / 16;
  static constexpr int ROW = W * 128;        // one region row of one 64-channel chunk
  static constexpr int RP = W / 64;          // DMA pieces per wave per region row
  static constexpr int RR = RR_ ? RR_ : TR == 4 ? 8 : TR + 2;  // ring rows
  static constexpr int RING = RR * ROW;
  static constexpr int B_BYTES = BN * WBK * 2;
  static constexpr int BJ = BN / 64;         // B DMA instructions per wave per step
  static constexpr int NBS = RING + 3 * B_BYTES <= 163840 ? 3 : 2;  // B stages
  static constexpr int LDS = RING + NBS * B_BYTES;
  static_assert(WN == 4 && WAVES_M * WAVES_N == 8, "wave tile (BM / WAVES_M) x 64");
  static_assert(LDS <= 163840, "LDS");
};

template <int BN, int W, int SCHED>
__global__ __launch_bounds__(512, 2) void conv_hwide3_kernel(ConvOp op) {
  using HC = Halo3Cfg<BN, W>;
  constexpr int WM = HC::WM, WN = HC::WN, BM = HC::BM;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % HC::WAVES_M;
  const int wn = wave / HC::WAVES_M;

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
  const int cs = sg.cs, Cin = sg.C, H = op.Ho;
  const int nchunks = Cin / WBK;
  const int total = nchunks * 9;
  const half_t* zero = (const half_t*)g_wide_zero;

  // region row r of chunk cc: RP 1-KiB pieces per wave (pixels (wave + 8k) * 8 .. +7)
  const int rpx = wave * 8 + (lane >> 3);
  const half_t* rsrc =
      (const half_t*)sg.src + sg.coff + ((size_t)img * HW + rpx) * cs + (((lane & 7) ^ halo_swz(rpx)) * 8);
  auto region_row = [&](int cc, int r) {
    const int iy = oy0 - 1 + r;
    const bool in = (unsigned)iy < (unsigned)H;
    unsigned char* dst = smem + ((6 * cc + r) & 7) * HC::ROW + wave * 1024;
#pragma unroll
    for (int k = 0; k < HC::RP; ++k)
      glds16(in ? rsrc + ((size_t)iy * W + 64 * k) * cs + cc * WBK : zero, dst + k * 8192);
  };
  // rows issued before the reads of step (c, t): this chunk's rows 4 / 5 at
  // t 0 / 1, the next chunk's rows 0, 2, 1, 3 at t 2, 3, 4, 6
  auto rows_at = [&](int c, int t) -> int {
    if (t < 2) return 1;
    return (t <= 4 || t == 6) && c + 1 < nchunks ? 1 : 0;
  };
  auto issue_rows = [&](int c, int t) {
    if (t < 2) region_row(c, 4 + t);
    else if (c + 1 < nchunks) {
      if (t == 2) region_row(c + 1, 0);
      else if (t == 3) region_row(c + 1, 2);
      else if (t == 4) region_row(c + 1, 1);
      else if (t == 6) region_row(c + 1, 3);
    }
  };

  const int q8 = lane >> 3;
  const int qc = lane & 7;
  const int sw_lane = lane >> 4;
  const half_t* Wt = (const half_t*)op.W;
  // B of step (c, t) into stage stg; steps past the end re-read the last
  // step's rows into a stage nobody reads again (keeps the DMA count uniform)
  auto issue_b = [&](int stg, int c, int t) {
    unsigned char* Bs = smem + HC::RING + stg * HC::B_BYTES;
    const int kb = sg.kbase + t * Cin + c * WBK;
#pragma unroll
    for (int j = 0; j < HC::BJ; ++j) {
      const int n = wave * (BN / 8) + j * 8 + q8;
      const int ch = qc ^ ((4 * j + sw_lane) & 7);
      glds16(Wt + (size_t)(n0 + n) * op.Kpad + kb + ch * 8, Bs + (wave * (BN / 8) + j * 8) * 128);
    }
  };

  f32x4_w acc[WM][WN];
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = f32x4_w{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15;
  const int fg = lane >> 4;
  const int rsw = (fr >> 1) & 7;
  const bool lane_l = fr == 0, lane_r = fr == 15;
  const int wrow = wm * 128 / W;  // the wave's first output row in the tile
  // fragments of step (c, ty, tx), half kk; B from stage stg
  auto rd = [&](int stg, int c, int ty, int tx, int kk, f16x8_w (&af)[WM], f16x8_w (&bf)[WN]) {
    const half_t* Bs = (const half_t*)(smem + HC::RING + stg * HC::B_BYTES);
    const int pc = ((kk * 4 + fg) ^ rsw) * 8;
#pragma unroll
    for (int b = 0; b < WN; ++b) bf[b] = *(const f16x8_w*)(Bs + (wn * WN * 16 + b * 16 + fr) * 64 + pc);
    const int p = fr + tx - 1;
    const int lofs = p * 128 + (((kk * 4 + fg) ^ halo_swz(p)) * 16);
    const int rbase = 6 * c + ty + wrow;  // ring row of the wave's first output row, before & 7
#pragma unroll
    for (int a = 0; a < WM; ++a) {
      const int rr = (rbase + a * 16 / W) & 7;
      af[a] = *(const f16x8_w*)(smem + rr * HC::ROW + (a * 16 % W) * 128 + lofs);
    }
  };
  // MFMAs of one half; the edge lane of a row's first / last 16-pixel group
  // is zeroed when the tap column leaves the image
  auto mm = [&](f16x8_w (&af)[WM], const f16x8_w (&bf)[WN], int tx) {
    const bool zl = tx == 0 && lane_l, zr = tx == 2 && lane_r;
#pragma unroll
    for (int a = 0; a < WM; ++a) {
      if ((a * 16) % W == 0 && zl) af[a] = f16x8_w{};
      if ((a * 16 + 16) % W == 0 && zr) af[a] = f16x8_w{};
#pragma unroll
      for (int b = 0; b < WN; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
  };
  auto interleave = [&]() {
    if constexpr (SCHED == 0) {
#pragma unroll
      for (int a = 0; a < WN; ++a) {
        __builtin_amdgcn_sched_group_barrier(0x008, WN, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
#pragma unroll
      for (int a = WN; a < WM; ++a) {
        __builtin_amdgcn_sched_group_barrier(0x008, WN, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    } else if constexpr (SCHED == 2) {
      // one fragment read after every two MFMAs, VALU between
#pragma unroll
      for (int a = 0; a < (WM * WN) / 2; ++a) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      }
    }
  };
  auto adv = [](int& c, int& y, int& x) {
    if (++x == 3) {
      x = 0;
      if (++y == 3) { y = 0; ++c; }
    }
  };
  constexpr int NBS = HC::NBS;
  // cursors: read step (rc, ry, rx) in B stage rs; B DMA step (bc, by, bx) into stage bs
  int rc = 0, ry = 0, rx = 0, rs = 0;
  int bc = 0, by = 0, bx = NBS - 1, bs = NBS - 1;
  const int lc = nchunks - 1;  // clamp for B past the end
  f16x8_w a0[WM], b0[WN], a1[WM], b1[WN];
  region_row(0, 0);
  region_row(0, 1);
  region_row(0, 2);
  region_row(0, 3);
  issue_b(0, 0, 0);
  if constexpr (NBS == 3) {
    issue_b(1, 0, 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(HC::BJ) : "memory");  // rows 0-3 and B(0) landed
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  issue_b(bs, 0, NBS - 1);  // B(NBS - 1)
  adv(bc, by, bx);          // -> step NBS
  bs = 0;
  issue_rows(0, 0);
  rd(0, 0, 0, 0, 0, a0, b0);
  int tx0 = 0;
  for (int step = 0; step < total - 1; ++step) {
    rd(rs, rc, ry, rx, 1, a1, b1);
    const int tx1 = rx;
    mm(a0, b0, tx0);
    interleave();
    // RAW: B(step + 1) and the region rows step + 1 reads have landed: the
    // only DMAs allowed in flight are the previous iteration's region rows
    // (issued two steps ahead of their first reader) and, with three stages,
    // its B(step + 2).  WAR: own fragment reads of step retired.
    constexpr int VB = NBS == 3 ? HC::BJ : 0;
    if (rows_at(rc, ry * 3 + rx)) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(VB + HC::RP) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(VB) : "memory");
    __builtin_amdgcn_s_barrier();
    adv(rc, ry, rx);  // -> step + 1
    rs = rs == NBS - 1 ? 0 : rs + 1;
    issue_b(bs, bc > lc ? lc : bc, bc > lc ? 8 : by * 3 + bx);  // B(step + NBS) into the stage step read
    adv(bc, by, bx);
    bs = bs == NBS - 1 ? 0 : bs + 1;
    issue_rows(rc, ry * 3 + rx);
    rd(rs, rc, ry, rx, 0, a0, b0);
    tx0 = rx;
    mm(a1, b1, tx1);
    interleave();
  }
  rd(rs, rc, ry, rx, 1, a1, b1);
  mm(a0, b0, tx0);
  mm(a1, b1, rx);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave is done with the ring and stages before the epilogue reuses LDS

  wide_epilogue<BN, WM, WN, HC::WAVES_M, BM, true>(op, acc, smem, m0, n0, M, HW);
}

template <int BN, int W, int SCHED>
static int launch_hwide3_s(const ConvOp& op, hipStream_t st) {
  using HC = Halo3Cfg<BN, W>;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute((const void*)conv_hwide3_kernel<BN, W, SCHED>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, HC::LDS);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  const int grid = (op.B * op.Ho * W / HC::BM) * (op.N / BN);
  hipLaunchKernelGGL((conv_hwide3_kernel<BN, W, SCHED>), dim3(grid), dim3(512), HC::LDS, st, op);
  return (int)hipGetLastError();
}
// schedule 2: one fragment read per two MFMAs, VALU between (measured bneck
// 0.177 -> 0.172 ms, dec3 0.219 -> 0.214 against the grouped interleave and
// hipcc's own schedule)
template <int BN, int W>
static int launch_hwide3(const ConvOp& op, hipStream_t st) {
  return launch_hwide3_s<BN, W, 2>(op, st);
}

// ---------------------------------------------------------------------------
// conv_hwide4_kernel: conv_hwide3's ring / three-B-stage algorithm with every
// step's control decided at COMPILE time.  hwide3 walks (chunk, tap) with
// runtime cursors, so its main loop carried ~170 SALU + ~88 VALU per 64 MFMAs
// (branches on the tap for the region-row DMA and the counted waits, ring-row
// arithmetic, the halo swizzle looked up from a 64-bit table per read, edge
// masks selected on runtime taps).  Here:
// * the Cin / 64 chunks x 9 taps are a template-unrolled sequence: ring rows,
//   B stages, DMA schedule and vmcnt counts are constants, every LDS fragment
//   read is a per-lane base register + an immediate offset;
// * waves own COLUMN blocks (32 columns of all 4 tile rows) instead of row
//   pairs, so a fragment's ring row depends on (chunk, tap, fragment) only --
//   not on the wave -- and stays static (the epilogue parks accumulators with
//   the matching mapping, wide_epilogue QW);
// * the A / B fragment lane offsets (swizzle included) for the 3 tap columns x
//   2 half-steps are computed once per block.
// Same arithmetic as hwide3: identical operands, MFMA order and epilogue.
// ---------------------------------------------------------------------------
// zero source of the out-of-image halo rows: a lane reads at its lane offset
// (< 8 pixels x 1024 channels x 2 B), so a 16 KiB zero block
__device__ __attribute__((aligned(256))) uint4 g_halo_zero[1024];

// ABL (timing ablations only, compiled on request -- the dispatcher instantiates
// ABL = 0; results are garbage; profiles/r3_hwide4_bneck_ablations*): bit 0 drops
// the main loop's DMA (region rows + B stages), bit 1 its LDS fragment reads,
// bit 2 the epilogue, bit 3 the MFMAs.  DS: operand-swapped MFMAs + the
// direct-store epilogue above (hw4_ds_ok decides per op).
// DL: dilated 3x3 (the ASPP branches, dilation = padding = d, any d < W): the
// three tap rows of a chunk read three disjoint 4-row bands, so the K loop is
// (tap row, chunk, tap column) and each (tap row, chunk) REGION of 4 rows is
// DMA'd once into one half of the 8-row ring (region k -> half k & 1, issued
// after the barrier that ends region k - 1's reads, three steps ahead of its
// first reader) and read by its 3 taps at per-lane column offsets +-d (lanes
// whose column falls outside the image row read through the void LDS base)
// NSC = 1: a second K segment after the 3x3 chunks, the projecting shortcut
// of ResBlock / PreActResBlock (1x1 stride 2 over 64 channels of a 2H x 2W
// source, kbase 9 * Cin: models/model.py:119-122, 159-162): one more K step
// whose 4 region rows are the source rows 2(oy0 + r), every other pixel,
// DMA'd into the ring slots the last chunk frees (the schedule of a next
// chunk's rows 0-3) and read without a tap shift
// PW: pointwise (1x1 stride 1) over NCH chunks, one K step per chunk (the
// ASPP fusion, K 1024, and conv1x1, K 256: models/model.py:231-251).  A
// chunk's region is its 4 tile rows (no halo), read by one step only, so the
// ring holds three chunks (12 rows, 96 KB) and two B stages fill the rest:
// chunk S + 3's rows go out after barrier S into the rows chunk S freed (two
// steps of lookahead for the HBM stream), B(S + 2) into B(S)'s stage (one
// step for the L2-resident filter)
// S2: 3x3 stride 2 pad 1 over a 2H x 2W source (enc2.conv1 / enc3.conv1,
// models/model.py:100-178) in the dilated form's region order (tap row,
// chunk, tap column): region k = (tap row ty, chunk c) is the TR source rows
// 2 (oy0 + r) + ty - 1, each DMA'd de-interleaved into an even-column and an
// odd-column plane of W pixels (a per-lane 2-pixel source stride), so the
// three taps read unit-stride fragments: tx 1 the even plane at column j, tx 0
// / 2 the odd plane at j - 1 / j (j - 1 < 0 through the void base).  Region k
// fills ring half k & 1 (2 x TR x ROW: 64 KB at W 64 x 4 rows, W 128 x 2
// rows); BN 128 leaves two 16 KB B stages.  Region k + 2 is issued after
// region k's last tap (three steps of lookahead), B(S + 2) after barrier S.
// NR: the op has no residual (res1 = res2 = null): no residual prefetch
// registers (rv0) -- 32 VGPRs the bottleneck conv1 / ASPP programs spilled for
template <int BN, int W, int NCH, int ABL = 0, bool DS = false, bool DL = false, int TR = 4, int NSC = 0,
          bool PW = false, bool S2 = false, bool NR = false>
__global__ __launch_bounds__(512, 2) void conv_hwide4_kernel(ConvOp op) {
  using HC = Halo3Cfg<BN, W, TR, PW ? 12 : S2 ? 4 * TR : 0>;
  static_assert(TR == 4 || (NCH == 1 && !DL && DS), "2-row tiles: one chunk, direct store");
  static_assert(NSC == 0 || (NSC <= 2 && !DL && TR == 4 && DS), "shortcut segment: 4-row tiles, direct store");
  static_assert(!PW || (!DL && NSC == 0 && TR == 4 && DS && HC::NBS == 2 && NCH >= 3), "pointwise form");
  static_assert(!S2 || (!DL && !PW && NSC == 0 && DS && HC::NBS == 2), "stride-2 form");
  constexpr int WM = HC::WM, WN = HC::WN, BM = HC::BM, NBS = HC::NBS;
  constexpr int KT = PW ? 1 : 9;  // K steps (taps) per chunk
  constexpr int TOTAL = NCH * KT + NSC;
  // (chunk, tap) of K step S; the shortcut step is chunk NCH with the centre column (tap 1: row 0, column 1);
  // a pointwise step reads its chunk's rows 0-3 at the centre column (tap 4 with the ring rows below)
  constexpr auto step_c = [](int S) -> int { return S < NCH * KT ? S / KT : NCH + (S - NCH * KT); };
  constexpr auto step_t = [](int S) -> int { return PW ? 4 : S < NCH * 9 ? S % 9 : 1; };
  constexpr int CW = W / HC::WAVES_M;  // columns per wave
  constexpr int FPR = CW / 16;         // fragments per tile row per wave
  static_assert(CW % 16 == 0 && WM == HC::TR * FPR, "column blocks of whole 16-pixel fragments");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  // wave-uniform values live in SGPRs: every DMA address below is a uniform
  // 64-bit base (scalar arithmetic per step) + a per-lane 32-bit offset fixed
  // for the block, so the unrolled steps keep no per-step address registers
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % HC::WAVES_M;
  const int wn = wave / HC::WAVES_M;

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
  constexpr int Cin = NCH * WBK;

  // region row r of chunk cc: RP 1-KiB pieces per wave, wave w's piece k =
  // pixels (w + 8k) * 8 .. +7 of the row; lane = (pixel, 16-byte chunk)
  const int rpx = wave * 8 + (lane >> 3);
  const unsigned voff_a = (unsigned)(((lane >> 3) * cs + (((lane & 7) ^ halo_swz(rpx)) * 8)) * 2);
  const unsigned char* abase =
      (const unsigned char*)((const half_t*)sg.src + sg.coff + ((size_t)img * HW + (size_t)wave * 8) * cs);
  const size_t row_bytes = (size_t)W * cs * 2;
  // shortcut region row r: source row 2 (oy0 + r), source pixels 2p
  const ConvSeg& sc = op.seg[NSC ? 1 : 0];
  const unsigned voff_sc = (unsigned)(((lane >> 3) * 2 * sc.cs + (((lane & 7) ^ halo_swz(rpx)) * 8)) * 2);
  const unsigned char* scbase =
      (const unsigned char*)((const half_t*)sc.src + sc.coff +
                             ((size_t)img * sc.Hin * sc.Win + (size_t)wave * 8 * 2) * sc.cs);
  // PW: the K chunk of step cc is (cc + rot) % NCH (op.krot): tiles in flight
  // together start at different chunks, so their row DMAs (a pixel's 2 KB of
  // 1024 channels read 128 B per step) do not all land on the same HBM
  // channels at once
  const int rot = PW && op.krot ? __builtin_amdgcn_readfirstlane(mtile % NCH) : 0;
  auto kchunk = [&](int cc) { const int k = cc + rot; return k >= NCH ? k - NCH : k; };
  // ring row of region row r of chunk cc: (6 cc + r) & 7; with two shortcut
  // chunks the second takes the last 3x3 chunk's rows 2-5 (free once its
  // last tap is read; the first shortcut chunk holds the two spare rows and
  // that chunk's rows 0 / 1)
  constexpr auto ring_slot = [](int cc, int r) -> int {
    return NSC == 2 && cc == NCH + 1 ? (6 * (NCH - 1) + 2 + r) & 7 : (6 * cc + r) & 7;
  };
  auto region_row = [&](int cc, int r) {  // cc, r compile-time at every call site
    if constexpr (PW) {  // tile row r of chunk cc -> ring row (4 cc + r) % 12 (always inside the image)
      unsigned char* dst = smem + ((4 * cc + r) % HC::RR) * HC::ROW + wave * 1024;
#pragma unroll
      for (int k = 0; k < HC::RP; ++k)
        glds16_s(abase + (size_t)(oy0 + r) * row_bytes + (size_t)k * 64 * cs * 2 + kchunk(cc) * WBK * 2, voff_a,
                 dst + k * 8192);
      return;
    }
    if (NSC && cc >= NCH) {
      unsigned char* dst = smem + ring_slot(cc, r) * HC::ROW + wave * 1024;
      const size_t srow = (size_t)2 * (oy0 + r) * sc.Win * sc.cs * 2 + (size_t)(cc - NCH) * WBK * 2;
#pragma unroll
      for (int k = 0; k < HC::RP; ++k)
        glds16_s(scbase + srow + (size_t)k * 128 * sc.cs * 2, voff_sc, dst + k * 8192);
      return;
    }
    const int iy = oy0 - 1 + r;
    const bool in = (unsigned)iy < (unsigned)H;
    unsigned char* dst = smem + ((6 * cc + r) & 7) * HC::ROW + wave * 1024;
#pragma unroll
    for (int k = 0; k < HC::RP; ++k) {
      const unsigned char* ub = in ? abase + (size_t)iy * row_bytes + (size_t)k * 64 * cs * 2 + cc * WBK * 2
                                   : (const unsigned char*)g_halo_zero;
      glds16_s(ub, voff_a, dst + k * 8192);
    }
  };
  // region rows issued right before the reads of step (c, t): this chunk's
  // rows 4 / 5 at t 0 / 1, the next chunk's rows 0, 2, 1, 3 at t 2, 3, 4, 6
  constexpr auto rows_at = [](int c, int t) -> int {
    if (TR != 4) return 0;  // 2-row tiles: all 4 region rows in the prologue
    if (t < 2) return c < NCH ? 1 : 0;  // (the shortcut region has no rows 4 / 5)
    return (t <= 4 || t == 6) && c + 1 < NCH + NSC ? 1 : 0;
  };
  auto issue_rows = [&](int c, int t) {
    if (TR != 4) return;
    if (t < 2) {
      if (c < NCH) region_row(c, 4 + t);
      // second shortcut chunk: all 4 rows right before the first shortcut step
      // reads (one step of lookahead; the wait of that step drains them)
      if (NSC == 2 && c == NCH) {
#pragma unroll
        for (int r = 0; r < 4; ++r) region_row(NCH + 1, r);
      }
    } else if (c + 1 < NCH + NSC) {
      if (t == 2) region_row(c + 1, 0);
      else if (t == 3) region_row(c + 1, 2);
      else if (t == 4) region_row(c + 1, 1);
      else if (t == 6) region_row(c + 1, 3);
    }
  };
  // DL: region k = (tap row k / NCH, chunk k % NCH), 4 rows into ring half k & 1;
  // regions past the last re-read the last one into the free half (uniform DMA count)
  constexpr int NREG = 3 * NCH;
  const int dil = sg.dil;
  auto region_dl = [&](int k) {  // k compile-time at every call site
    const int kk = k < NREG ? k : NREG - 1;
    const int ty = kk / NCH, cc = kk % NCH;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int iy = oy0 + (ty - 1) * dil + r;
      const bool in = (unsigned)iy < (unsigned)H;
      unsigned char* dst = smem + ((k & 1) * 4 + r) * HC::ROW + wave * 1024;
#pragma unroll
      for (int pc = 0; pc < HC::RP; ++pc) {
        const unsigned char* ub = in ? abase + (size_t)iy * row_bytes + (size_t)pc * 64 * cs * 2 + cc * WBK * 2
                                     : (const unsigned char*)g_halo_zero;
        glds16_s(ub, voff_a, dst + pc * 8192);
      }
    }
  };

  // S2 region k (regions past the last are not issued; the waits count them)
  const unsigned char* s2base =
      (const unsigned char*)((const half_t*)sg.src + sg.coff + ((size_t)img * sg.Hin * sg.Win + (size_t)wave * 16) * cs);
  const size_t s2row_bytes = (size_t)sg.Win * cs * 2;
  const unsigned voff_s2 = (unsigned)(((lane >> 3) * 2 * cs + (((lane & 7) ^ halo_swz(rpx)) * 8)) * 2);
  auto region_s2 = [&](int k) {  // k compile-time at every call site
    const int ty = k / NCH, cc = k % NCH;
#pragma unroll
    for (int r = 0; r < TR; ++r) {
      const int iy = 2 * (oy0 + r) + ty - 1;
      const bool in = (unsigned)iy < (unsigned)sg.Hin;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        unsigned char* dst = smem + ((k & 1) * 2 * TR + q * TR + r) * HC::ROW + wave * 1024;
#pragma unroll
        for (int pc = 0; pc < HC::RP; ++pc) {
          const unsigned char* ub = in ? s2base + (size_t)iy * s2row_bytes + (size_t)pc * 128 * cs * 2 + cc * WBK * 2 +
                                             q * cs * 2
                                       : (const unsigned char*)g_halo_zero;
          glds16_s(ub, voff_s2, dst + pc * 8192);
        }
      }
    }
  };
  constexpr int S2DMA = 2 * TR * HC::RP;  // DMAs per wave per S2 region

  const int q8 = lane >> 3;
  const int qc = lane & 7;
  const int sw_lane = lane >> 4;
  // B row n0 + wave*BN/8 + j*8 + q8, chunk qc ^ ((4j + sw_lane) & 7): the lane
  // offset depends on j's parity only
  const unsigned voff_b[2] = {(unsigned)((q8 * op.Kpad + ((qc ^ (sw_lane & 7)) * 8)) * 2),
                              (unsigned)((q8 * op.Kpad + ((qc ^ ((4 + sw_lane) & 7)) * 8)) * 2)};
  const unsigned char* bbase =
      (const unsigned char*)((const half_t*)op.W + (size_t)(n0 + wave * (BN / 8)) * op.Kpad + sg.kbase);
  // DS: LDS row R of the B tile is filled from weight row hw4_perm32(R); the
  // lane offsets are taken from the row's 32-row group base (unsigned)
  const int g32 = (wave * (BN / 8)) & ~31;
  const unsigned char* bbase_ds =
      (const unsigned char*)((const half_t*)op.W + (size_t)(n0 + g32) * op.Kpad + sg.kbase);
  unsigned voff_ds[HC::BJ];
#pragma unroll
  for (int j = 0; j < HC::BJ; ++j) {
    // LDS row R's chunk swizzle (R >> 1) & 7 (for BN 64 it depends on the wave's parity)
    const int R = wave * (BN / 8) + j * 8 + q8;
    voff_ds[j] = (unsigned)(((hw4_perm32(R) - g32) * op.Kpad + ((qc ^ ((R >> 1) & 7)) * 8)) * 2);
  }
  // B of step (c, t) into stage stg; steps past the end re-read the last
  // step's rows into a stage nobody reads again (uniform DMA count)
  auto issue_b = [&](int stg, int c, int t) {  // DL: c = region, t = tap column
    unsigned char* Bs = smem + HC::RING + stg * HC::B_BYTES;
    const int kb = PW   ? kchunk(c) * WBK
                   : (DL || S2) ? ((c / NCH) * 3 + t) * Cin + (c % NCH) * WBK
                   : c < NCH ? t * Cin + c * WBK : 9 * Cin + (c - NCH) * WBK;
#pragma unroll
    for (int j = 0; j < HC::BJ; ++j) {
      if constexpr (DS)
        glds16_s(bbase_ds + (size_t)kb * 2, voff_ds[j], Bs + (wave * (BN / 8) + j * 8) * 128);
      else
        glds16_s(bbase + ((size_t)j * 8 * op.Kpad + kb) * 2, voff_b[j & 1], Bs + (wave * (BN / 8) + j * 8) * 128);
    }
  };

  f32x4_w acc[WM][WN];
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = f32x4_w{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15;
  const int fg = lane >> 4;
  const int rsw = (fr >> 1) & 7;
  // per-lane fragment offsets of half 0: A for tap column tx, B; half 1 is the
  // same with chunk bit 2 flipped (XOR 64: the swizzles act on the chunk index).
  // Edge lanes (a tap column outside the image row; ring rows have no padding
  // columns) of a row's first / last fragment read through a base far beyond
  // the block's LDS allocation: out-of-range LDS reads return zero, so no
  // per-fragment select is needed (aofs_e[0] for tx 0, aofs_e[1] for tx 2).
  constexpr int kLdsVoid = 1 << 30;
  int aofs[3], aofs_e[2], bofs;
#pragma unroll
  for (int tx = 0; tx < 3; ++tx) {
    const int p = CW * wm + fr + tx - 1;
    aofs[tx] = p * 128 + ((fg ^ halo_swz(p)) * 16);
  }
  aofs_e[0] = (wm == 0 && fr == 0) ? kLdsVoid : aofs[0];
  aofs_e[1] = (wm == HC::WAVES_M - 1 && fr == 15) ? kLdsVoid : aofs[2];
  // DL: per (tap column, fragment of the row) lane offsets, void outside the row
  int aofs_d[DL ? 3 : 1][DL ? FPR : 1];
  if constexpr (DL) {
#pragma unroll
    for (int tx = 0; tx < 3; ++tx)
#pragma unroll
      for (int f = 0; f < FPR; ++f) {
        // a void lane keeps the bank bits of an in-row pixel of the same
        // parity and residue: void lanes on one bank serialised the edge
        // fragments' reads (SQ_LDS_BANK_CONFLICT 5.5M cycles per launch at d 6-18)
        const int p = CW * wm + f * 16 + fr + (tx - 1) * dil;
        aofs_d[tx][f] = (unsigned)p < (unsigned)W ? p * 128 + ((fg ^ halo_swz(p)) * 16)
                                                  : kLdsVoid + (p & 15) * 128 + ((fg ^ halo_swz(p & 15)) * 16);
      }
  }
  // S2: per (tap column, fragment) lane offsets into the region's planes
  int aofs_s[S2 ? 3 : 1][S2 ? FPR : 1];
  if constexpr (S2) {
#pragma unroll
    for (int tx = 0; tx < 3; ++tx)
#pragma unroll
      for (int f = 0; f < FPR; ++f) {
        const int j = CW * wm + f * 16 + fr;
        const int p = tx == 0 ? j - 1 : j;
        const int plane = tx == 1 ? 0 : 1;
        aofs_s[tx][f] = p >= 0 ? plane * TR * HC::ROW + p * 128 + ((fg ^ halo_swz(p)) * 16)
                               : kLdsVoid + (p & 15) * 128 + ((fg ^ halo_swz(p & 15)) * 16);
      }
  }
  bofs = HC::RING + (wn * WN * 16 + fr) * 128 + ((fg ^ rsw) * 16);

  // fragments of step S, half KK: B (all WN) and A row fragment a
  auto rd_b = [&](auto S_, auto KK_, f16x8_w (&bf)[WN]) {
    constexpr int S = decltype(S_)::value, KK = decltype(KK_)::value;
    constexpr int stg = S % NBS;
    const int bo = KK ? (bofs ^ 64) : bofs;
#pragma unroll
    for (int b = 0; b < WN; ++b) bf[b] = *(const f16x8_w*)(smem + bo + stg * HC::B_BYTES + b * 16 * 128);
  };
  auto rd_a = [&](auto S_, auto KK_, auto A_) -> f16x8_w {
    constexpr int S = decltype(S_)::value, KK = decltype(KK_)::value, a = decltype(A_)::value;
    constexpr int c = step_c(S), t = step_t(S), ty = t / 3, tx = t % 3;
    if constexpr (DL) {
      constexpr int h = (S / 3) & 1, dtx = S % 3;
      const int ao = KK ? (aofs_d[dtx][a % FPR] ^ 64) : aofs_d[dtx][a % FPR];
      return *(const f16x8_w*)(smem + ao + (h * 4 + a / FPR) * HC::ROW);
    } else if constexpr (S2) {
      constexpr int h = (S / 3) & 1, dtx = S % 3;
      constexpr int off = (h * 2 * TR + a / FPR) * HC::ROW;
      int ao = KK ? (aofs_s[dtx][a % FPR] ^ 64) : aofs_s[dtx][a % FPR];
      if constexpr (off >= 65536) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(ao) : "n"(off & ~0xffff));
      return *(const f16x8_w*)(smem + ao + (off & 0xffff));
    } else {
      constexpr bool edge = (tx == 0 && a % FPR == 0) || (tx == 2 && a % FPR == FPR - 1);
      constexpr int rr = PW ? (4 * c + a / FPR) % HC::RR : ring_slot(c, ty + a / FPR);
      constexpr int off = rr * HC::ROW + (a % FPR) * 16 * 128;
      int ao;
      if constexpr (edge && tx == 0) ao = KK ? (aofs_e[0] ^ 64) : aofs_e[0];
      else if constexpr (edge) ao = KK ? (aofs_e[1] ^ 64) : aofs_e[1];
      else ao = KK ? (aofs[tx] ^ 64) : aofs[tx];
      // ds_read's immediate offset is 16 bits: a ring row at >= 64 KiB (W 128)
      // needs a base of its own.  Formed here, per step, by an add the
      // compiler may not hoist -- hoisted, one base per (row, tap column,
      // half) stayed live across the unrolled loop and spilled.
      if constexpr (off >= 65536) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(ao) : "n"(off & ~0xffff));
      return *(const f16x8_w*)(smem + ao + (off & 0xffff));
    }
  };
  // one A row fragment against all WN B fragments
  auto mm_row = [&](int a, const f16x8_w& af, const f16x8_w (&bf)[WN]) {
    if constexpr ((ABL & 8) != 0) return;
#pragma unroll
    for (int b = 0; b < WN; ++b) {
      if constexpr (DS)
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[b], af, acc[a][b], 0, 0, 0);
      else
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[b], acc[a][b], 0, 0, 0);
    }
  };
  // A fragments roll: each row fragment is replaced by the next half's as
  // soon as its MFMAs are issued, so one A set (WM) and two B sets (2 WN) are
  // live instead of two of each -- 32 VGPRs less, the difference between
  // spilling (each reload drained the DMA queue with a vmcnt(0)) and not
  f16x8_w af[WM], b0[WN], b1[WN];
  f16x8_w rv0[WM];  // DS: pair-0 residual rows (hw4_res_load)
  // half KK of step S (af, bf) issued; af rolls to (S2, KK2)
  auto mm_roll = [&](auto S2_, auto KK2_, const f16x8_w (&bf)[WN], bool roll) {
    static_for<WM>([&](auto A_) {
      constexpr int a = decltype(A_)::value;
      mm_row(a, af[a], bf);
      if (roll) af[a] = rd_a(S2_, KK2_, A_);
    });
  };
  static_assert(!DL || (DS && NBS == 3), "dilated form: direct-store epilogue, three B stages");
  if constexpr (S2) {
    region_s2(0);
    issue_b(0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue_b(1, 0, 1);
    if constexpr (3 * NCH > 1) region_s2(1);
  } else if constexpr (PW) {
    // chunk 0 + B(0) landed, chunk 1 may fly; then B(1) and chunk 2
#pragma unroll
    for (int r = 0; r < 4; ++r) region_row(0, r);
    issue_b(0, 0, 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) region_row(1, r);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * HC::RP) : "memory");
    __builtin_amdgcn_s_barrier();
    issue_b(1, 1, 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) region_row(2, r);
  } else if constexpr (DL) {
    region_dl(0);
  } else if constexpr (!S2) {
    region_row(0, 0);
    region_row(0, 1);
    region_row(0, 2);
    region_row(0, 3);
  }
  if constexpr (!PW && !S2) {
    issue_b(0, 0, 0);
    if constexpr (NBS == 3) {
      issue_b(1, 0, 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(HC::BJ) : "memory");  // rows 0-3 and B(0) landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if constexpr (DL) {
      issue_b(2, 0, 2);  // B(2)
      region_dl(1);
    } else {
      issue_b(NBS - 1, (NBS - 1) / 9, (NBS - 1) % 9);  // B(NBS - 1)
      issue_rows(0, 0);
    }
  }
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  rd_b(I0{}, I0{}, b0);
  static_for<WM>([&](auto A_) { af[decltype(A_)::value] = rd_a(I0{}, I0{}, A_); });
  static_steps(
      [&](auto S_) {
        constexpr int S = decltype(S_)::value;
        rd_b(S_, I1{}, b1);
        if constexpr (S + 1 < TOTAL) {
          constexpr int c = step_c(S), t = step_t(S);
          constexpr int n = S + 1, nc = step_c(n), nt = step_t(n);
          // B DMA of step S + NBS (clamped past the end) into the stage step S read
          constexpr int bstep = S + NBS < TOTAL ? S + NBS : TOTAL - 1;
          constexpr int bc = (DL || S2) ? (S + NBS < TOTAL ? bstep / 3 : NREG - 1) : step_c(bstep);
          constexpr int bt = (DL || S2) ? (S + NBS < TOTAL ? bstep % 3 : 2) : step_t(bstep);
          mm_roll(S_, I1{}, b0, true);
          // RAW: B(S + 1) and the region rows step S + 1 reads have landed: in
          // flight may stay the previous iteration's region rows (issued two
          // steps ahead of their first reader) and, with three stages, its
          // B(S + 2).  WAR: own fragment reads of step S retired.
          constexpr int VB = NBS == 3 ? HC::BJ : 0;
          // DL: at S = 3k + 2 region k + 1 (issued after B(S + 1) at S - 3) and
          // B(S + 1) must have landed; B(S + 2) may fly.  Otherwise B(S + 1)
          // must have landed; B(S + 2) and the region issued at 3k - 1 may fly.
          // PW: B(S + 1) (issued at barrier S - 1, before chunk S + 2) and chunk S +
          // 1 (barrier S - 2) must have landed; chunk S + 2 may fly when it exists
          if constexpr (PW) {
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(S + 2 < NCH ? 4 * HC::RP : 0) : "memory");
          } else if constexpr (S2) {
            // B(S + 1) (issued at barrier S - 1) must have landed, and so must the
            // region step S + 1 reads (issued 3+ steps earlier); in flight may stay
            // region S / 3 + 1 when it was issued after B(S + 1) (S % 3 == 0)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(S % 3 == 0 && S / 3 + 1 < NREG ? S2DMA : 0)
                         : "memory");
          } else if constexpr (DL) {
            if constexpr (S % 3 == 2)
              asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(HC::BJ) : "memory");
            else
              asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(HC::BJ + 4 * HC::RP) : "memory");
          } else if constexpr (NSC == 2 && S == NCH * 9) {
            // the second shortcut chunk's rows (issued last, at barrier S - 1) are read next
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          } else if constexpr (rows_at(c, t))
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(VB + HC::RP) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(VB) : "memory");
          __builtin_amdgcn_s_barrier();
          if constexpr (!(ABL & 1)) {
            issue_b(S % NBS, bc, bt);
            if constexpr (S2) {
              if constexpr (S % 3 == 2 && S / 3 + 2 < NREG) region_s2(S / 3 + 2);
            } else if constexpr (PW) {
              if constexpr (S + 3 < NCH) {
#pragma unroll
                for (int r = 0; r < 4; ++r) region_row(S + 3, r);
              }
            } else if constexpr (DL) {
              if constexpr (S % 3 == 2) region_dl(S / 3 + 2);
            } else {
              issue_rows(nc, nt);
            }
          }
          if constexpr (DS && !NR && S == TOTAL - 2)
            hw4_res_load<WM, WN, HC::WAVES_M, W>(op, rv0, m0, n0, wm, wn, lane);
          rd_b(std::integral_constant<int, n>{}, I0{}, b0);
          mm_roll(std::integral_constant<int, n>{}, I0{}, b1, true);
        } else {
          mm_roll(S_, I1{}, b0, true);
          mm_roll(S_, I1{}, b1, false);
        }
      },
      std::make_integer_sequence<int, TOTAL>{});
  if constexpr (DS) {
    // the last steps' (unread) DMAs land before the block ends; with a
    // residual, the compiler's own wait for the residual loads (issued after
    // them, in order) already covers them
    if (!op.res1 && !op.res2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (op.pool) {
      // the pool partials reuse LDS: every wave's DMAs landed, every wave's reads done
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if constexpr ((ABL & 4) != 0) {
      if (acc[0][0][0] == 12345.f)
        hw4_direct_epilogue<BN, WM, WN, HC::WAVES_M, W, !NR>(op, acc, m0, n0, wm, wn, lane, rv0, smem);
    } else {
      hw4_direct_epilogue<BN, WM, WN, HC::WAVES_M, W, !NR>(op, acc, m0, n0, wm, wn, lane, rv0, smem);
    }
    if constexpr ((ABL & 4) != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  // the last steps' (unread) DMAs land before the epilogue reuses LDS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave is done with the ring and stages before the epilogue reuses LDS

  if constexpr ((ABL & 4) != 0) {
    if (acc[0][0][0] == 12345.f) wide_epilogue<BN, WM, WN, HC::WAVES_M, BM, true, W>(op, acc, smem, m0, n0, M, HW);
  } else {
    wide_epilogue<BN, WM, WN, HC::WAVES_M, BM, true, W>(op, acc, smem, m0, n0, M, HW);
  }
}

template <int BN, int W, int NCH, int ABL = 0, bool DS = false, bool DL = false, int TR = 4, int NSC = 0,
          bool PW = false, bool S2 = false, bool NR = false>
static int launch_hwide4_k(const ConvOp& op, hipStream_t st) {
  using HC = Halo3Cfg<BN, W, TR, PW ? 12 : S2 ? 4 * TR : 0>;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e =
        hipFuncSetAttribute((const void*)conv_hwide4_kernel<BN, W, NCH, ABL, DS, DL, TR, NSC, PW, S2, NR>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, HC::LDS);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  const int grid = (op.B * op.Ho * W / HC::BM) * (op.N / BN);
  hipLaunchKernelGGL((conv_hwide4_kernel<BN, W, NCH, ABL, DS, DL, TR, NSC, PW, S2, NR>), dim3(grid), dim3(512),
                     HC::LDS, st, op);
  return (int)hipGetLastError();
}

template <int BN, int W, int NCH>
static int launch_hwide4(const ConvOp& op, hipStream_t st) {
  if (hw4_ds_ok(op)) {
    if constexpr (BN == 256 && W == 64 && NCH == 4) {
      // UPR_HW4_ABL: timing ablations of the bottleneck form (garbage results; profiles/r6_hw4_abl*)
      static const int abl = [] { const char* e = getenv("UPR_HW4_ABL"); return e ? atoi(e) : 0; }();
      if (!op.res1 && !op.res2 && abl == 1) return launch_hwide4_k<BN, W, NCH, 1, true, false, 4, 0, false, false, true>(op, st);
      if (!op.res1 && !op.res2 && abl == 4) return launch_hwide4_k<BN, W, NCH, 4, true, false, 4, 0, false, false, true>(op, st);
      if (!op.res1 && !op.res2 && abl == 5) return launch_hwide4_k<BN, W, NCH, 5, true, false, 4, 0, false, false, true>(op, st);
      if (!op.res1 && !op.res2 && abl == 7) return launch_hwide4_k<BN, W, NCH, 7, true, false, 4, 0, false, false, true>(op, st);
    }
    if (!op.res1 && !op.res2) return launch_hwide4_k<BN, W, NCH, 0, true, false, 4, 0, false, false, true>(op, st);
    return launch_hwide4_k<BN, W, NCH, 0, true>(op, st);
  }
  return launch_hwide4_k<BN, W, NCH, 0, false>(op, st);
}

// the compile-time-schedule hwide4 for the graph's shapes (bottleneck: W 64,
// Cin 256; dec3: W 128, Cin 128), the runtime-cursor hwide3 otherwise
template <int BN, int W>
static int launch_hwide34(const ConvOp& op, hipStream_t st) {
  const int nch = op.seg[0].C / WBK;
  if (op.seg[0].kbase == 0) {
    if constexpr (W == 64) {
      if (nch == 4) return launch_hwide4<BN, W, 4>(op, st);
    } else {
      // dec3 (W 128, 2 chunks) on the direct-store form only (its LDS-epilogue
      // straight line spilled 40 VGPRs): dec3.conv.0 shape 0.196 -> 0.153 ms,
      // conv.3 (+ residual) 0.223 -> 0.186 (same-box A/B, profiles/r3_hw4_ds_ab.txt)
      if (nch == 2 && hw4_ds_ok(op)) return launch_hwide4_k<BN, W, 2, 0, true>(op, st);
      // 256-channel inputs at W 128 (the training step's VGG-19 conv3_x and
      // their input gradients, losses/loss.py:198-211)
      if (nch == 4 && hw4_ds_ok(op)) return launch_hwide4_k<BN, W, 4, 0, true>(op, st);
    }
  }
  return launch_hwide3<BN, W>(op, st);
}

// halo-tiled convs: the ring / three-stage form (hwide4 / hwide3) for W 64 x
// N 256 and W 128 x N 128, the two-stage halo kernel for W 64 x N 128
// (measured against the gathered-A kernel: profiles/r2_halo*, r3_hw4_*)
// the 3x3 segment + projecting-shortcut programs hwide4 takes: enc2.conv2 (128
// -> 128 at W 128, shortcut over the block's 64-channel input: NSC 1) and
// enc3.conv2 (256 -> 256 at W 64, shortcut over 128 channels: NSC 2).
// Returns the shortcut chunk count, 0 when neither fits
static int hw4_sc_ok(const ConvOp& op) {
  if (op.nseg != 2 || op.store != kStoreNHWC) return 0;
  const ConvSeg& s = op.seg[0];
  const ConvSeg& q = op.seg[1];
  if (s.kh != 3 || s.kw != 3 || s.stride != 1 || s.pad != 1 || s.dil != 1 || s.pre != kPreNone || s.kbase != 0)
    return 0;
  if (q.kh != 1 || q.kw != 1 || q.stride != 2 || q.pad != 0 || q.pre != kPreNone || q.kbase != 9 * s.C) return 0;
  if (s.Hin != op.Ho || s.Win != op.Wo || q.Hin != 2 * op.Ho || q.Win != 2 * op.Wo) return 0;
  if (q.cs % 8 || q.coff % 8 || (uintptr_t)q.src % 16 || s.cs % 8 || s.coff % 8 || (uintptr_t)s.src % 16) return 0;
  if (op.Kpad != 9 * s.C + q.C || !hw4_ds_ok(op)) return 0;
  if (s.C == 128 && op.Wo == 128 && op.N == 128 && (op.Ho * op.Wo) % 512 == 0 && q.C == 64) return 1;
  if (s.C == 256 && op.Wo == 64 && op.N == 256 && op.Ho % 4 == 0 && q.C == 128) return 2;
  return 0;
}

// 1x1 stride-1 GEMMs over whole 64-pixel rows, K 256 / 1024 / 1280 -> N 256k (the ASPP
// conv1x1 and fusion, models/model.py:231-251): the pointwise hwide4 form
static int hw4_pw_route(const ConvOp& op, hipStream_t st) {
  const ConvSeg& s = op.seg[0];
  if (s.kh != 1 || s.kw != 1 || s.stride != 1 || s.pad != 0 || s.dil != 1 || s.pre != kPreNone || s.kbase != 0)
    return kErrUnsupported;
  if (s.Hin != op.Ho || s.Win != op.Wo || op.Wo != 64 || op.N % 256 || (op.Ho * op.Wo) % 256 || op.Kpad != s.C)
    return kErrUnsupported;
  if (s.cs % 8 || s.coff % 8 || (uintptr_t)s.src % 16 || !hw4_ds_ok(op)) return kErrUnsupported;
  // UPR_HW4_PW: 0 = the gathered kernel instead, 2 = no chunk rotation (A/B, tools/convbench.py)
  static const int mode = [] { const char* e = getenv("UPR_HW4_PW"); return e ? atoi(e) : 1; }();
  if (mode == 0) return kErrUnsupported;
  ConvOp o = op;
  o.krot = mode != 2;
  if (s.C == 256) return launch_hwide4_k<256, 64, 4, 0, true, false, 4, 0, true>(o, st);
  if (s.C == 1024) return launch_hwide4_k<256, 64, 16, 0, true, false, 4, 0, true>(o, st);
  if (s.C == 1280) return launch_hwide4_k<256, 64, 20, 0, true, false, 4, 0, true>(o, st);  // (+ global branch)
  return kErrUnsupported;
}

// 3x3 stride-2 convs over 64-channel chunks, N 128k: W 64 x 4-row tiles
// (enc3.conv1: 128 -> 256 at 128^2 -> 64^2) and W 128 x 2-row tiles (enc2.conv1:
// 64 -> 128 at 256^2 -> 128^2) on the stride-2 hwide4 form
static int hw4_s2_route(const ConvOp& op, hipStream_t st) {
  const ConvSeg& s = op.seg[0];
  if (s.kh != 3 || s.kw != 3 || s.stride != 2 || s.pad != 1 || s.dil != 1 || s.pre != kPreNone || s.kbase != 0)
    return kErrUnsupported;
  if (s.Hin != 2 * op.Ho || s.Win != 2 * op.Wo || op.N % 128 || op.Kpad != 9 * s.C || !hw4_ds_ok(op))
    return kErrUnsupported;
  static const bool off = [] { const char* e = getenv("UPR_HW4_S2"); return e && atoi(e) == 0; }();
  if (off) return kErrUnsupported;  // A/B against the gathered kernel (tools/convbench.py)
  if (op.Wo == 64 && op.Ho % 4 == 0) {
    if (s.C == 64) return launch_hwide4_k<128, 64, 1, 0, true, false, 4, 0, false, true>(op, st);
    if (s.C == 128) return launch_hwide4_k<128, 64, 2, 0, true, false, 4, 0, false, true>(op, st);
    if (s.C == 256) return launch_hwide4_k<128, 64, 4, 0, true, false, 4, 0, false, true>(op, st);
  }
  if (op.Wo == 128 && op.Ho % 2 == 0 && s.C == 64)
    return launch_hwide4_k<128, 128, 1, 0, true, false, 2, 0, false, true>(op, st);
  return kErrUnsupported;
}

static int halo_route(const ConvOp& op, hipStream_t st) {
  if (const int nsc = hw4_sc_ok(op)) {
    if (nsc == 1) return launch_hwide4_k<128, 128, 2, 0, true, false, 4, 1>(op, st);
    static const bool off = [] { const char* e = getenv("UPR_HW4_SC2"); return e && atoi(e) == 0; }();
    if (!off) return launch_hwide4_k<256, 64, 4, 0, true, false, 4, 2>(op, st);  // (UPR_HW4_SC2=0: A/B)
  }
  if (op.nseg != 1 || op.store != kStoreNHWC) return kErrUnsupported;
  const ConvSeg& s = op.seg[0];
  if (s.kh == 1 && s.kw == 1) return hw4_pw_route(op, st);
  if (s.stride == 2) return hw4_s2_route(op, st);
  // dilated 3x3 over 256 channels at W 64 (the ASPP branches, d = 6 / 12 / 18):
  // the region form of hwide4 (gathered kernel: 0.168 / 0.153 / 0.143 ms vs
  // 0.158 / 0.145 / 0.136, profiles/r3_hw4_dil_ab.txt)
  if (s.kh == 3 && s.kw == 3 && s.stride == 1 && s.dil > 1 && s.pad == s.dil && s.dil < 64 && s.pre == kPreNone &&
      s.kbase == 0 && s.C == 256 && s.Hin == op.Ho && s.Win == op.Wo && op.Wo == 64 && op.N % 256 == 0 &&
      (op.Ho * op.Wo) % WBM == 0 && hw4_ds_ok(op)) {
    if (!op.res1 && !op.res2) return launch_hwide4_k<256, 64, 4, 0, true, true, 4, 0, false, false, true>(op, st);
    return launch_hwide4_k<256, 64, 4, 0, true, true>(op, st);
  }
  if (s.kh != 3 || s.kw != 3 || s.stride != 1 || s.pad != 1 || s.dil != 1 || s.pre != kPreNone) return kErrUnsupported;
  if (s.Hin != op.Ho || s.Win != op.Wo || s.C % WBK || (op.Ho * op.Wo) % WBM) return kErrUnsupported;
  // (64 -> 64 at W 256, the dec2 UpBlock convs, as hwide4 2-row tiles measured
  // 9% slower than the row ring: dec2p 0.234 -> 0.255 ms, profiles/r3_hw4_64_ab.txt)
  if (op.N % 128) return kErrUnsupported;
  if (op.Wo == 64 && op.N % 256 == 0) return launch_hwide34<256, 64>(op, st);
  if (op.Wo == 64) return launch_hwide<128, 64>(op, st);
  if (op.Wo == 128 && (op.Ho * op.Wo) % 512 == 0) return launch_hwide34<128, 128>(op, st);
  return kErrUnsupported;
}


// the gathered kernel's direct-store form takes what hwide4's does minus the
// per-image pool (its tiles may straddle images)
static bool wide_ds_ok(const ConvOp& op) { return !op.pool && hw4_ds_ok(op); }

template <int BN, bool PIPE, int SCHED, bool DS>
static int launch_wide_bn_k(const ConvOp& op, hipStream_t st) {
  using C = WideCfg<BN>;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute((const void*)conv_wide_kernel<BN, PIPE, 2, SCHED, DS>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  const int M = op.B * op.Ho * op.Wo;
  const int grid = ((M + WBM - 1) / WBM) * (op.N / BN);
  hipLaunchKernelGGL((conv_wide_kernel<BN, PIPE, 2, SCHED, DS>), dim3(grid), dim3(512), C::LDS, st, op);
  return (int)hipGetLastError();
}
template <int BN, bool PIPE, int SCHED>
static int launch_wide_bn_s(const ConvOp& op, hipStream_t st) {
  return wide_ds_ok(op) ? launch_wide_bn_k<BN, PIPE, SCHED, true>(op, st) : launch_wide_bn_k<BN, PIPE, SCHED, false>(op, st);
}

// schedule 2: one fragment read per two MFMAs (beat the grouped interleave)
template <int BN, bool PIPE>
static int launch_wide_bn(const ConvOp& op, hipStream_t st) {
  return launch_wide_bn_s<BN, PIPE, 2>(op, st);
}

static int launch_wide_onestep128(const ConvOp& op, hipStream_t st);

// Routing of the 128-wide single-stage two-blocks-per-CU variant (measured,
// fp16 preact+ASPP bs 32: it beats the one-block double-buffered kernel on
// every 128-wide GEMM of the graph -- enc2.conv1 0.184 -> 0.160 ms, enc2.conv2
// 0.255 -> 0.204, dec1.up 0.369 -> 0.258 -- and, as 128-wide halves, on the
// 2-step 256-wide dec2.up 0.178 -> 0.157; the 4-step 256-wide ASPP conv1x1
// 0.070 -> 0.053 ms; the 16-step ASPP fusion breaks even, so it stays whole).
// 128-wide GEMMs always take it; 256-wide ones of <= kSplit256 K steps (and
// stride-2 ones) run as two 128-wide halves on it.
constexpr int kSplit256 = 4;

template <int BN>
static int launch_wide_any(const ConvOp& op, hipStream_t st) {
  int steps = 0;
  for (int s = 0; s < op.nseg; ++s) steps += op.seg[s].kh * op.seg[s].kw * (op.seg[s].C / WBK);
  // stride-2 256-wide convs (enc3.conv1, 18 steps) also gain as halves: 0.125 -> 0.108 ms,
  // where the 16-step 1x1 ASPP fusion loses (0.127 -> 0.156)
  bool s2 = false;
  for (int s = 0; s < op.nseg; ++s) s2 = s2 || op.seg[s].stride == 2;
  if (BN == 128 || steps <= kSplit256 || s2) return launch_wide_onestep128(op, st);
  if (steps < 2) return launch_wide_bn<BN, false>(op, st);
  return launch_wide_bn<BN, true>(op, st);
}

// One-step GEMMs (K = 64: the dec1 ConvTranspose) are latency-bound at one
// block per CU (load -> MFMA -> epilogue, nothing to overlap): with one LDS
// stage and <= 128 VGPRs two blocks share a CU and one's epilogue hides the
// other's operand fetch (dec1.up 0.369 -> 0.258 ms).  128-wide tiles only (a
// 256-wide tile needs 128 accumulator registers per lane on its own).
static int launch_wide_onestep128(const ConvOp& op, hipStream_t st) {
  using C = WideCfg<128>;
  constexpr int EPI = 64 * (128 + 4) * 4;
  constexpr int LDS1 = C::STAGE > EPI ? C::STAGE : EPI;
  const int M = op.B * op.Ho * op.Wo;
  const int grid = ((M + WBM - 1) / WBM) * (op.N / 128);
  if (wide_ds_ok(op))
    hipLaunchKernelGGL((conv_wide_kernel<128, false, 4, 0, true>), dim3(grid), dim3(512), LDS1, st, op);
  else
    hipLaunchKernelGGL((conv_wide_kernel<128, false, 4>), dim3(grid), dim3(512), LDS1, st, op);
  return (int)hipGetLastError();
}

// fp16 only; returns kErrUnsupported for shapes this kernel does not take
int launch_conv_wide(const ConvOp& op, hipStream_t st) {
  if (op.out2 && ((uintptr_t)op.out2 % 16 || op.store != kStoreNHWC)) return kErrUnsupported;
  if (op.out32 && ((uintptr_t)op.out32 % 16 || op.out32_cs % 4 || op.out32_coff % 4)) return kErrUnsupported;
  if (op.res32 && ((uintptr_t)op.res32 % 16 || op.res32_cs % 4)) return kErrUnsupported;
  if (op.store == kStoreHeadIllu || op.N % 64) return kErrUnsupported;
  if (op.Kpad % 8 || ((uintptr_t)op.W % 16)) return kErrUnsupported;
  for (int s = 0; s < op.nseg; ++s) {
    const ConvSeg& sg = op.seg[s];
    if (sg.pre != kPreNone || sg.C % WBK || sg.cs % 8 || sg.coff % 8 || sg.kbase % 8) return kErrUnsupported;
    if ((uintptr_t)sg.src % 16) return kErrUnsupported;
  }
  // UPR_HALO=0: skip the halo-tiled forms (A/B against the gathered kernel, tools/convbench.py)
  static const bool halo_off = [] { const char* e = getenv("UPR_HALO"); return e && atoi(e) == 0; }();
  if (!halo_off) {
    const int rc = halo_route(op, st);
    if (rc != kErrUnsupported) return rc;
  }
  if (op.N % 128) return kErrUnsupported;  // (64-wide: only the halo route above)
  if (op.N % 256 == 0) return launch_wide_any<256>(op, st);
  // (128-channel stride-1 3x3 convs: faster here than on the old halo kernel,
  // dec3.conv.0 0.264 -> 0.191 ms, conv.3 0.276 -> 0.217)
  return launch_wide_any<128>(op, st);
}

}  // namespace upr
