// Implicit-GEMM convolution for gfx950 (CDNA4), NHWC activations.
//
// One kernel covers every conv of the UP-Retinex graph that has >= 32 input
// channels (models/model.py: ResBlock/PreActResBlock convs :106-118/:149-162,
// ASPP :196-229, UpBlock :261-269, residual head :324-328, EnhancedFAM
// :29-44) plus ConvTranspose2d(k2,s2) as a pixel-shuffled GEMM.
//
//   M = B*Ho*Wo pixels (rows), N = output channels (cols), K = virtual concat of
//   up to 4 segments, each a kh x kw window over C channels of an NHWC source.
//
// Tile: 256 threads = 4 waves of 64.  BM x BN output tile, BK = 32 channels per
// K step.  A (pixels x channels) and B (weights, [N][K]) are staged through LDS
// with a register prefetch of the next K step (issue-early / write-late).
//
// MFMA: each lane's fragment is 8 k of one row: fp16 [8g, 8g+8) as 1 x
// v_mfma_f32_16x16x32_f16 (fp32 accumulate), fp32 [4g, 4g+4) u [16+4g, 16+4g+4)
// as 8 x v_mfma_f32_16x16x4_f32 (exact fp32), g = lane>>4.  The permutation of k
// across MFMA k-slots is the same for A and B, so the sum is unchanged.
#include <cstdlib>
#include <cstring>
#include <cstdio>

#include "upr_common.h"

namespace upr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <typename T> struct Frag;
template <> struct Frag<float> {
  static constexpr int EPC = 4;  // elements per 16-byte chunk
};
template <> struct Frag<half_t> {
  static constexpr int EPC = 8;
};

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(half_t v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ half_t from_f<half_t>(float v) { return (half_t)v; }

// XCD-aware bijective remap: consecutive logical tiles land on one XCD (blocks
// b and b+8 share an XCD under round-robin dispatch; speed only).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  int q = nwg >> 3, r = nwg & 7;
  int xcd = bid & 7, idx = bid >> 3;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

template <typename T, int WAVES_M, int WAVES_N, int WM, int WN, int BK>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvOp op) {
  static_assert(BK == 32 || (BK == 64 && sizeof(T) == 2), "BK 64 is the fp16 variant");
  constexpr int EPC = Frag<T>::EPC;
  constexpr int CH = BK / EPC;              // 16-byte chunks per row of a K step
  constexpr int ROWS_PASS = 256 / CH;
  constexpr int BM = WAVES_M * WM * 16;
  constexpr int BN = WAVES_N * WN * 16;
  constexpr int A_IT = BM / ROWS_PASS;
  constexpr int B_IT = (BN * CH + 255) / 256;
  // LDS row stride: fp32 10 x 16 B with the k-permutation {g, g+4} below, fp16
  // 6 x 16 B (BK 32) / 9 x 16 B (BK 64): the fragment reads (16 rows x 4
  // chunks per ds_read_b128) are then bank-conflict free (row r starts at bank
  // 36r mod 64 for the 144-byte rows: 16 distinct multiples of 4)
  constexpr int LDS_ROW = sizeof(T) == 4 ? 40 : (BK == 64 ? 72 : 48);
  static_assert(A_IT >= 1, "tile too small");

  __shared__ __attribute__((aligned(16))) T As[BM * LDS_ROW];
  __shared__ __attribute__((aligned(16))) T Bs[BN * LDS_ROW];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WAVES_M;
  const int wn = wave / WAVES_M;

  const int M = op.B * op.Ho * op.Wo;
  const int HW = op.Ho * op.Wo;
  const int mtiles = (M + BM - 1) / BM;
  const int ntiles = op.N / BN;
  const int L = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int ntile = L % ntiles;
  const int mtile = L / ntiles;
  const int m0 = mtile * BM;
  const int n0 = ntile * BN;

  // ---- per-thread A-load rows ------------------------------------------
  const int a_chunk = tid % CH;
  const int a_row0 = tid / CH;
  int pb[A_IT], py[A_IT], px[A_IT];
#pragma unroll
  for (int i = 0; i < A_IT; ++i) {
    int m = m0 + a_row0 + i * ROWS_PASS;
    if (m < M) {
      int b = m / HW, r = m - b * HW;
      pb[i] = b;
      py[i] = r / op.Wo;
      px[i] = r - py[i] * op.Wo;
    } else {
      pb[i] = -1; py[i] = 0; px[i] = 0;
    }
  }

  // ---- K-step cursor ------------------------------------------------------
  int total_steps = 0;
  for (int s = 0; s < op.nseg; ++s) total_steps += op.seg[s].kh * op.seg[s].kw * (op.seg[s].C / BK);

  uint4 ra[A_IT];
  uint4 rb[B_IT];

  int cur_seg = 0, cur_tap = 0, cur_c0 = 0;

  auto load_step = [&](int seg_i, int tap, int c0) {
    const ConvSeg& sg = op.seg[seg_i];
    const int r = tap / sg.kw, s = tap - r * sg.kw;
    const int cbase = c0 + a_chunk * EPC;
    const T* src = (const T*)sg.src;
    float psc[EPC], psh[EPC];
    if (sg.pre == kPreAffineRelu) {
#pragma unroll
      for (int e = 0; e < EPC; ++e) { psc[e] = sg.pre_scale[cbase + e]; psh[e] = sg.pre_shift[cbase + e]; }
    }
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (pb[i] >= 0) {
        const int iy = py[i] * sg.stride - sg.pad + r * sg.dil;
        const int ix = px[i] * sg.stride - sg.pad + s * sg.dil;
        if (iy >= 0 && iy < sg.Hin && ix >= 0 && ix < sg.Win) {
          const size_t pix = ((size_t)pb[i] * sg.Hin + iy) * sg.Win + ix;
          if (sg.pre == kPreMaxPool3) {
            float mx[EPC];
#pragma unroll
            for (int e = 0; e < EPC; ++e) mx[e] = -INFINITY;
            for (int dy = -1; dy <= 1; ++dy) {
              const int yy = iy + dy;
              if (yy < 0 || yy >= sg.Hin) continue;
              for (int dx = -1; dx <= 1; ++dx) {
                const int xx = ix + dx;
                if (xx < 0 || xx >= sg.Win) continue;
                const size_t p2 = ((size_t)pb[i] * sg.Hin + yy) * sg.Win + xx;
                uint4 w = *(const uint4*)(src + p2 * sg.cs + sg.coff + cbase);
                const T* wv = (const T*)&w;
#pragma unroll
                for (int e = 0; e < EPC; ++e) mx[e] = fmaxf(mx[e], to_f(wv[e]));
              }
            }
            T* vv = (T*)&v;
#pragma unroll
            for (int e = 0; e < EPC; ++e) vv[e] = from_f<T>(mx[e]);
          } else {
            v = *(const uint4*)(src + pix * sg.cs + sg.coff + cbase);
            if (sg.pre == kPreAffineRelu) {
              T* vv = (T*)&v;
#pragma unroll
              for (int e = 0; e < EPC; ++e) vv[e] = from_f<T>(fmaxf(to_f(vv[e]) * psc[e] + psh[e], 0.f));
            }
          }
        }
      }
      ra[i] = v;
    }
    const int kb = sg.kbase + tap * sg.C + c0;
    const T* W = (const T*)op.W;
#pragma unroll
    for (int j = 0; j < B_IT; ++j) {
      const int idx = tid + j * 256;
      if (idx < BN * CH) {
        const int nrow = idx / CH, ch = idx % CH;
        rb[j] = *(const uint4*)(W + (size_t)(n0 + nrow) * op.Kpad + kb + ch * EPC);
      }
    }
  };
  auto advance = [&]() {
    const ConvSeg& sg = op.seg[cur_seg];
    cur_c0 += BK;
    if (cur_c0 >= sg.C) {
      cur_c0 = 0;
      if (++cur_tap >= sg.kh * sg.kw) { cur_tap = 0; ++cur_seg; }
    }
  };

  f32x4 acc[WM][WN];
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (total_steps > 0) { load_step(cur_seg, cur_tap, cur_c0); advance(); }

  const int fr = lane & 15;
  const int fg = lane >> 4;
  // fp16: lane reads k [8g, 8g+8); fp32: k [4g, 4g+4) u [16+4g, 16+4g+4)
  const int fk = sizeof(T) == 4 ? fg * 4 : fg * 8;

  for (int step = 0; step < total_steps; ++step) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < A_IT; ++i)
      *(uint4*)(As + (a_row0 + i * ROWS_PASS) * LDS_ROW + a_chunk * EPC) = ra[i];
#pragma unroll
    for (int j = 0; j < B_IT; ++j) {
      const int idx = tid + j * 256;
      if (idx < BN * CH) *(uint4*)(Bs + (idx / CH) * LDS_ROW + (idx % CH) * EPC) = rb[j];
    }
    __syncthreads();
    if (step + 1 < total_steps) { load_step(cur_seg, cur_tap, cur_c0); advance(); }

    if constexpr (sizeof(T) == 4) {
      f32x4 af[WM][2], bf[WN][2];
#pragma unroll
      for (int a = 0; a < WM; ++a) {
        const float* p = (const float*)As + (wm * WM * 16 + a * 16 + fr) * LDS_ROW + fk;
        af[a][0] = *(const f32x4*)p;
        af[a][1] = *(const f32x4*)(p + 16);
      }
#pragma unroll
      for (int b = 0; b < WN; ++b) {
        const float* p = (const float*)Bs + (wn * WN * 16 + b * 16 + fr) * LDS_ROW + fk;
        bf[b][0] = *(const f32x4*)p;
        bf[b][1] = *(const f32x4*)(p + 16);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int a = 0; a < WM; ++a)
#pragma unroll
          for (int b = 0; b < WN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a][j >> 2][j & 3], bf[b][j >> 2][j & 3],
                                                            acc[a][b], 0, 0, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        f16x8 af[WM], bf[WN];
#pragma unroll
        for (int a = 0; a < WM; ++a)
          af[a] = *(const f16x8*)((const half_t*)As + (wm * WM * 16 + a * 16 + fr) * LDS_ROW + kk * 32 + fk);
#pragma unroll
        for (int b = 0; b < WN; ++b)
          bf[b] = *(const f16x8*)((const half_t*)Bs + (wn * WN * 16 + b * 16 + fr) * LDS_ROW + kk * 32 + fk);
#pragma unroll
        for (int a = 0; a < WM; ++a)
#pragma unroll
          for (int b = 0; b < WN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a], bf[b], acc[a][b], 0, 0, 0);
      }
    }
  }

  // ---- epilogue -------------------------------------------------------------
  const int rq = (lane >> 4) * 4;  // first of this lane's 4 accumulator rows
  if (op.store == kStoreHeadIllu) {
    // residual head (models/model.py:324-328, :351-358): per pixel
    // r = sum_c relu(conv3x3(d1)+b)_c * w2_c + b2 ; illu = sigmoid(mean_c(x) + r)
#pragma unroll
    for (int a = 0; a < WM; ++a) {
      float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int b = 0; b < WN; ++b) {
        const int n = n0 + wn * WN * 16 + b * 16 + fr;
        const float sc = op.scale ? op.scale[n] : 1.f;
        const float bi = op.bias ? op.bias[n] : 0.f;
        const float w2 = op.head_w[n];
#pragma unroll
        for (int i = 0; i < 4; ++i) part[i] += fmaxf(acc[a][b][i] * sc + bi, 0.f) * w2;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = part[i];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        part[i] = v;
      }
      if (fr == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wm * WM * 16 + a * 16 + rq + i;
          if (m >= M) continue;
          const int b = m / HW, p = m - b * HW;
          float x0, x1, x2;
          if (op.x_f16) {
            const half_t* x = (const half_t*)op.x_nchw + (size_t)b * 3 * HW + p;
            x0 = (float)x[0]; x1 = (float)x[HW]; x2 = (float)x[2 * HW];
          } else {
            const float* x = op.x_nchw + (size_t)b * 3 * HW + p;
            x0 = x[0]; x1 = x[HW]; x2 = x[2 * HW];
          }
          const float z = (x0 + x1 + x2) / 3.f + (part[i] + op.head_b);
          const float il = 1.f / (1.f + expf(-z));
          if (op.illu_f16) ((half_t*)op.illu)[m] = (half_t)il;
          else op.illu[m] = il;
        }
      }
    }
    return;
  }

  const bool one_image = (m0 / HW) == (min(m0 + BM, M) - 1) / HW;
  T* out = (T*)op.out;
  const T* res1 = (const T*)op.res1;
  const T* res2 = (const T*)op.res2;
#pragma unroll
  for (int b = 0; b < WN; ++b) {
    const int n = n0 + wn * WN * 16 + b * 16 + fr;
    const float sc = op.scale ? op.scale[n] : 1.f;
    const float bi = op.bias ? op.bias[n] : 0.f;
    float psum = 0.f;
#pragma unroll
    for (int a = 0; a < WM; ++a) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * WM * 16 + a * 16 + rq + i;
        if (m >= M) continue;
        float v = acc[a][b][i] * sc + bi;
        const int img = m / HW;
        if (op.img_bias) v += op.img_bias[img * op.N + n];
        if (res1) v += to_f(res1[(size_t)m * op.res1_cs + n]);
        if (op.relu) v = fmaxf(v, 0.f);
        if (res2) v += to_f(res2[(size_t)m * op.res2_cs + n]);
        if (op.store == kStoreConvT2x2) {
          const int cout = op.N >> 2;
          const int q = n / cout, co = n - q * cout;
          const int p = m - img * HW;
          const int oy = p / op.Wo, ox = p - oy * op.Wo;
          const int Y = 2 * oy + (q >> 1), X = 2 * ox + (q & 1);
          const size_t opix = ((size_t)img * 2 * op.Ho + Y) * (2 * op.Wo) + X;
          out[opix * op.out_cs + op.out_coff + co] = from_f<T>(v);
        } else {
          const T tv = from_f<T>(v);
          out[(size_t)m * op.out_cs + op.out_coff + n] = tv;
          if (op.pool) {
            if (one_image) psum += to_f(tv);
            else pool_add(op.pool, (size_t)img * op.N + n, to_f(tv));
          }
        }
      }
    }
    if (op.pool && one_image) {
      psum += __shfl_xor(psum, 16);
      psum += __shfl_xor(psum, 32);
      if (lane < 16) pool_add(op.pool, (size_t)(m0 / HW) * op.N + n, psum);
    }
  }
}

template <typename T, int WAVES_M, int WAVES_N, int WM, int WN, int BK = 32>
static int launch_cfg(const ConvOp& op, hipStream_t stream) {
  constexpr int BM = WAVES_M * WM * 16;
  constexpr int BN = WAVES_N * WN * 16;
  const int M = op.B * op.Ho * op.Wo;
  if (op.N % BN) return kErrShape;
  const int grid = ((M + BM - 1) / BM) * (op.N / BN);
  hipLaunchKernelGGL((conv_igemm_kernel<T, WAVES_M, WAVES_N, WM, WN, BK>), dim3(grid), dim3(256), 0, stream, op);
  return (int)hipGetLastError();
}

// fp16 with every segment a multiple of 64 channels: 64-deep K steps (half the
// barriers and LDS round trips per MFMA)
static bool k64_ok(const ConvOp& op) {
  for (int s = 0; s < op.nseg; ++s)
    if (op.seg[s].C % 64) return false;
  return true;
}

template <typename T>
static int launch_t(const ConvOp& op, hipStream_t stream) {
  if (op.store == kStoreHeadIllu) {
    if (op.N != 32) return kErrShape;
    return launch_cfg<T, 4, 1, 4, 2>(op, stream);
  }
  if constexpr (sizeof(T) == 2) {
    if (k64_ok(op)) {
      if (op.N % 128 == 0 && op.N >= 256) return launch_cfg<T, 2, 2, 4, 4, 64>(op, stream);
      if (op.N % 64 == 0) return launch_cfg<T, 2, 2, 4, 2, 64>(op, stream);
      if (op.N % 32 == 0) return launch_cfg<T, 4, 1, 4, 2, 64>(op, stream);
    }
  }
  if (op.N % 128 == 0 && op.N >= 256) return launch_cfg<T, 2, 2, 4, 4>(op, stream);
  if (op.N % 64 == 0) return launch_cfg<T, 2, 2, 4, 2>(op, stream);
  if (op.N % 32 == 0) return launch_cfg<T, 4, 1, 4, 2>(op, stream);
  return kErrShape;
}

int launch_conv_halo(const ConvOp& op, int dtype, hipStream_t st);
int launch_conv_wide(const ConvOp& op, hipStream_t st);
int launch_conv_ring(const ConvOp& op, hipStream_t st);
int launch_conv_ring32(const ConvOp& op, hipStream_t st);
int launch_conv_wide32(const ConvOp& op, hipStream_t st);
int launch_conv_t2(const ConvOp& op, int dtype, hipStream_t st);

int launch_preact_f16(const void* x, const float* sc, const float* sh, void* o, size_t npix, int C, hipStream_t st);

// UPR_TRACE_ROUTE=1: one stderr line per fp16 conv call naming the kernel family
// it fell to and its shape (tools: which training convs still take a fallback)
static void trace_route(const char* fam, const ConvOp& op) {
  static const bool on = [] { const char* e = getenv("UPR_TRACE_ROUTE"); return e && atoi(e) != 0; }();
  if (!on) return;
  const ConvSeg& s = op.seg[0];
  fprintf(stderr, "upr_route %s nseg %d B %d Cin %d Hin %d Win %d -> N %d Ho %d Wo %d k %dx%d s %d p %d d %d pre %d "
                  "out32 %d res %d relu %d\n", fam, op.nseg, op.B, s.C, s.Hin, s.Win, op.N, op.Ho, op.Wo, s.kh, s.kw,
          s.stride, s.pad, s.dil, s.pre, op.out32 != nullptr, op.res1 != nullptr || op.res2 != nullptr, op.relu);
}

int launch_conv_out32(const ConvOp& op, hipStream_t stream) {
  if (!op.out32 || op.out || op.out2 || op.pool || op.store == kStoreHeadIllu) return kErrArg;
  if (op.nseg < 1 || op.nseg > 4 || op.B <= 0 || op.Ho <= 0 || op.Wo <= 0) return kErrArg;
  // narrow 1x1 GEMMs stream (conv_pw.hip); the stride-2 scatter form exists only there
  int rc = launch_conv_pw(op, stream);
  if (rc != kErrUnsupported || op.out_s2) return trace_route("pw", op), rc;
  rc = launch_conv_wide(op, stream);
  if (rc != kErrUnsupported) return trace_route("wide", op), rc;
  rc = launch_conv_ring(op, stream);
  if (rc != kErrUnsupported) return trace_route("ring", op), rc;
  trace_route("halo", op);
  return launch_conv_halo(op, kF16, stream);
}

int launch_conv(const ConvOp& op, int dtype, hipStream_t stream) {
  if (op.nseg < 1 || op.nseg > 4 || op.B <= 0 || op.Ho <= 0 || op.Wo <= 0) return kErrArg;
  if (op.out32 || op.out_s2) return kErrArg;  // launch_conv_out32
  if (op.out2) {
    // fused second output: only the wide-tile and row-ring epilogues write it;
    // any other kernel runs the plain op and the PreAct pass separately
    if (dtype != kF16 || op.store != kStoreNHWC || op.out_coff || op.out_cs != op.N || op.out2_cs != op.N ||
        !op.pre2_scale || !op.pre2_shift)
      return kErrArg;
    int rc = launch_conv_wide(op, stream);
    if (rc != kErrUnsupported) return rc;
    rc = launch_conv_ring(op, stream);
    if (rc != kErrUnsupported) return rc;
    ConvOp c = op;
    c.out2 = nullptr;
    rc = launch_conv(c, dtype, stream);
    if (rc != kOk) return rc;
    return launch_preact_f16(op.out, op.pre2_scale, op.pre2_shift, op.out2, (size_t)op.B * op.Ho * op.Wo, op.N, stream);
  }
  for (int s = 0; s < op.nseg; ++s)
    if (op.seg[s].C % 32 || op.seg[s].src == nullptr) return kErrShape;
  {
    if (dtype == kF16) {
      int rc = launch_conv_t2(op, dtype, stream);
      if (rc != kErrUnsupported) return trace_route("t2", op), rc;
      rc = launch_conv_wide(op, stream);
      if (rc != kErrUnsupported) return trace_route("wide", op), rc;
      rc = launch_conv_ring(op, stream);
      if (rc != kErrUnsupported) return trace_route("ring", op), rc;
    } else {
      // 32 -> 64 3x3 without a residual (EnhancedFAM branch34_conv1): the fp32
      // ring with its filter in registers first (measured 2.80 -> 2.53 ms at
      // 512^2 bs 32 against the wide32 tile)
      const bool ring_first = op.nseg == 1 && op.seg[0].C == 32 && op.N == 64 && !op.res1 && !op.res2;
      int rc = ring_first ? launch_conv_ring32(op, stream) : launch_conv_t2(op, dtype, stream);
      if (rc != kErrUnsupported) return rc;
      rc = launch_conv_wide32(op, stream);
      if (rc != kErrUnsupported) return rc;
      rc = launch_conv_ring32(op, stream);
      if (rc != kErrUnsupported) return rc;
    }
    const int rc = launch_conv_halo(op, dtype, stream);
    if (rc != kErrUnsupported) return trace_route("halo", op), rc;
  }
  trace_route("igemm", op);
  return dtype == kF16 ? launch_t<half_t>(op, stream) : launch_t<float>(op, stream);
}

}  // namespace upr
