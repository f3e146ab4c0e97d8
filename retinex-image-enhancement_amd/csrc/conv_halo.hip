// Halo-tiled direct convolution for gfx950 (stride-1 3x3 / 1x1 segments).
//
// The generic implicit-GEMM kernel (conv.hip) re-reads the A operand once per
// filter tap.  Here a block owns a TH x 32 output-pixel tile of one image and
// stages, per K step (= one segment x 32-channel chunk), the input REGION the
// tile needs (tile + (k-1)*dil halo) into LDS once; every tap then reads its A
// fragments from LDS at shifted offsets.  The step's weights for all taps sit
// next to it (staged once per block when the whole K is one step).
//
// * Blocks loop over tiles (persistent grid).  With PREF the region of the NEXT
//   step (possibly of the next tile) is loaded into registers while the
//   current step's MFMAs run; the prologue (pre-activation BN+ReLU) is applied
//   when the registers are written to LDS; a 1x1 max-pool segment is pooled
//   synchronously (EnhancedFAM branch2 only).
// * Region geometry is a compile-time function of the step kind (1x1, 3x3 d1,
//   3x3 d2), so every index division is by a constant.
// * LDS pixel / weight-row strides are chosen so the 16-byte fragment reads of
//   the MFMA operands are bank-conflict free (fp32: 10 chunks per row with the
//   k-permutation {g, g+4}; fp16: 6 chunks per row) — brute-forced against
//   the ds_read_b128 lane groups of MI355X_MICROARCH.md §LDS.
// * Epilogue goes through LDS: residual chunks are all requested before the
//   first is used, and every global store is a full 16-byte chunk of
//   consecutive channels (NHWC rows are contiguous).
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
constexpr int HALO_MAXEXT = 4;  // 3x3 with dilation <= 2

template <typename T, int NB, int TH>
struct HaloCfg {
  static constexpr int EPC = 16 / sizeof(T);   // elements per 16-byte chunk
  static constexpr int CCH = 32 / EPC;         // chunks per 32-channel slice
  static constexpr int PSTR = sizeof(T) == 4 ? 40 : 48;  // row stride (elements): 10 / 6 chunks
  static constexpr int HALO_ELEMS = (TH + HALO_MAXEXT) * (HALO_TW + HALO_MAXEXT) * PSTR;
  static constexpr int CSTR = NB + 4;          // fp32 epilogue staging stride
  static constexpr int EPI_BYTES = TH * HALO_TW * CSTR * 4;
  static constexpr int REGION_BYTES =
      HALO_ELEMS * (int)sizeof(T) > EPI_BYTES ? HALO_ELEMS * (int)sizeof(T) : EPI_BYTES;
  static constexpr int B_ELEMS = 9 * NB * PSTR;
  static constexpr int BYTES = REGION_BYTES + B_ELEMS * (int)sizeof(T);
  static constexpr int PF = ((TH + HALO_MAXEXT) * (HALO_TW + HALO_MAXEXT) * CCH + 255) / 256;
  static constexpr int CHN = NB / EPC;         // epilogue chunks per pixel
  static constexpr int PPP = 256 / CHN;        // epilogue pixels per pass
  static constexpr int PASSES = TH * HALO_TW / PPP;
};

// step kind: 0 = 1x1, 1 = 3x3 dil 1, 2 = 3x3 dil 2  ->  EXT = 0, 2, 4
__device__ __forceinline__ int step_kind(const ConvSeg& s) { return s.kh == 1 ? 0 : (s.dil == 1 ? 1 : 2); }

template <typename T, int NB, int TH, int EXT>
__device__ __forceinline__ void halo_load(uint4* pf, const ConvSeg& sg, int b, int oy0,
                                          int ox0, int c0, int tid) {
  using C = HaloCfg<T, NB, TH>;
  constexpr int HW = HALO_TW + EXT, HH = TH + EXT, NCH = HH * HW * C::CCH;
  constexpr int PAD = EXT / 2;
  const T* base = (const T*)sg.src + (size_t)b * sg.Hin * sg.Win * sg.cs + sg.coff + c0;
  // Every step kind writes EVERY pf[] entry at a constant index: when the kinds
  // write different subsets, the compiler merges their stores through a phi'd
  // address and demotes pf[] to scratch (each prefetch then waits on vmcnt(0)).
#pragma unroll
  for (int j = 0; j < C::PF; ++j) {
    const int q = tid + j * 256;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (j * 256 < NCH) {
      const int px = q / C::CCH, ch = q % C::CCH;
      const int hy = px / HW, hx = px % HW;
      const int iy = oy0 - PAD + hy, ix = ox0 - PAD + hx;
      const bool ok = q < NCH && iy >= 0 && iy < sg.Hin && ix >= 0 && ix < sg.Win;
      if (ok) v = *(const uint4*)(base + ((size_t)iy * sg.Win + ix) * sg.cs + ch * C::EPC);
    }
    pf[j] = v;
  }
}

template <typename T, int NB, int TH, int EXT>
__device__ __forceinline__ void halo_store(const uint4* pf, const ConvSeg& sg, int oy0,
                                           int ox0, int c0, int tid, T* halo) {
  using C = HaloCfg<T, NB, TH>;
  constexpr int HW = HALO_TW + EXT, HH = TH + EXT, NCH = HH * HW * C::CCH;
  constexpr int PAD = EXT / 2;
  const bool aff = sg.pre == kPreAffineRelu;
#pragma unroll
  for (int j = 0; j < C::PF; ++j) {
    const int q = tid + j * 256;
    if (j * 256 < NCH && q < NCH) {
      const int px = q / C::CCH, ch = q % C::CCH;
      uint4 v = pf[j];
      if (aff) {
        const int hy = px / HW, hx = px % HW;
        const int iy = oy0 - PAD + hy, ix = ox0 - PAD + hx;
        if (iy >= 0 && iy < sg.Hin && ix >= 0 && ix < sg.Win) {  // zero padding stays zero
          const int cb = c0 + ch * C::EPC;
          T* vv = (T*)&v;
#pragma unroll
          for (int e = 0; e < C::EPC; ++e)
            vv[e] = hfrom_f<T>(fmaxf(hto_f(vv[e]) * sg.pre_scale[cb + e] + sg.pre_shift[cb + e], 0.f));
        }
      }
      *(uint4*)(halo + px * C::PSTR + ch * C::EPC) = v;
    }
  }
}

// 3x3/s1/p1 max-pool of the source for a 1x1 segment (EnhancedFAM branch2, model.py:32,69)
template <typename T, int NB, int TH>
__device__ void halo_pool(const ConvSeg& sg, int b, int oy0, int ox0, int c0, int tid, T* halo) {
  using C = HaloCfg<T, NB, TH>;
  const T* src = (const T*)sg.src;
  for (int q = tid; q < TH * HALO_TW * C::CCH; q += 256) {
    const int px = q / C::CCH, ch = q % C::CCH;
    const int iy = oy0 + px / HALO_TW, ix = ox0 + px % HALO_TW;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (iy < sg.Hin && ix < sg.Win) {
      float mx[C::EPC];
#pragma unroll
      for (int e = 0; e < C::EPC; ++e) mx[e] = -INFINITY;
      for (int dy = -1; dy <= 1; ++dy) {
        const int yy = iy + dy;
        if (yy < 0 || yy >= sg.Hin) continue;
        for (int dx = -1; dx <= 1; ++dx) {
          const int xx = ix + dx;
          if (xx < 0 || xx >= sg.Win) continue;
          const uint4 w4 =
              *(const uint4*)(src + (((size_t)b * sg.Hin + yy) * sg.Win + xx) * sg.cs + sg.coff + c0 + ch * C::EPC);
          const T* wv = (const T*)&w4;
#pragma unroll
          for (int e = 0; e < C::EPC; ++e) mx[e] = fmaxf(mx[e], hto_f(wv[e]));
        }
      }
      T* vv = (T*)&v;
#pragma unroll
      for (int e = 0; e < C::EPC; ++e) vv[e] = hfrom_f<T>(mx[e]);
    }
    *(uint4*)(halo + px * C::PSTR + ch * C::EPC) = v;
  }
}

// all taps of one step
template <typename T, int NB, int TH, int K, int D>
__device__ __forceinline__ void halo_taps(f32x4_h (&acc)[TH / 2][NB / 16], const T* halo, const T* Bs, int wave,
                                          int fr, int fg) {
  using C = HaloCfg<T, NB, TH>;
  constexpr int PSTR = C::PSTR;
  constexpr int RPW = TH / 4;
  constexpr int MT = 2 * RPW;
  constexpr int NT = NB / 16;
  constexpr int HW = HALO_TW + (K - 1) * D;
  constexpr int NTAP = K * K;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int tap = 0; tap < NTAP; ++tap) {
      const int r = tap / K, c = tap % K;
      f16x8_h bf[NT], af[MT];
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[j] = *(const f16x8_h*)(Bs + (tap * NB + j * 16 + fr) * PSTR + fg * 8);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int py = wave * RPW + (i >> 1) + r * D, pxx = (i & 1) * 16 + fr + c * D;
        af[i] = *(const f16x8_h*)(halo + (py * HW + pxx) * PSTR + fg * 8);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int tap = 0; tap < NTAP; ++tap) {
      const int r = tap / K, c = tap % K;
      f32x4_h bf[NT][2], af[MT][2];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const float* p = (const float*)Bs + (tap * NB + j * 16 + fr) * PSTR + fg * 4;
        bf[j][0] = *(const f32x4_h*)p;
        bf[j][1] = *(const f32x4_h*)(p + 16);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int py = wave * RPW + (i >> 1) + r * D, pxx = (i & 1) * 16 + fr + c * D;
        const float* p = (const float*)halo + (py * HW + pxx) * PSTR + fg * 4;
        af[i][0] = *(const f32x4_h*)p;
        af[i][1] = *(const f32x4_h*)(p + 16);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][e >> 2][e & 3], bf[j][e >> 2][e & 3], acc[i][j],
                                                            0, 0, 0);
    }
  }
}

// The next step's region (possibly of the next tile) is loaded into registers
// during the current step's MFMAs.  OCC = waves per SIMD the register
// allocation must allow (= co-resident 256-thread blocks per CU): above 1 the
// compiler stops hoisting every tap's fragment reads and a second block's
// MFMAs overlap this block's staging / epilogue.  KM = bitmask of the step
// kinds the op contains (1: 1x1, 2: 3x3 d1, 4: 3x3 d2); a single-kind op gets
// a kernel with only that kind's region / tap code (fewer live registers).
template <typename T, int NB, int TH, int OCC, int KM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void conv_halo_kernel(
    ConvOp op, int tiles_x, int tiles_y, int ntiles, int region_bytes) {
  constexpr bool PREF = true;
  using C = HaloCfg<T, NB, TH>;
  constexpr int EPC = C::EPC, CCH = C::CCH, PSTR = C::PSTR;
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
  const T* W = (const T*)op.W;
  // at most one residual per op (launch_conv_halo checks): added before (res1) or after (res2) the ReLU
  const T* resp = (const T*)(op.res1 ? op.res1 : op.res2);
  const int res_cs = op.res1 ? op.res1_cs : op.res2_cs;
  const bool res_pre = op.res1 != nullptr;

  int nsteps = 0;
  for (int s = 0; s < op.nseg; ++s) nsteps += op.seg[s].C / 32;
  const bool b_keep = nsteps == 1 && nblk_n == 1;  // weights identical for every tile of the block

  auto tile_coords = [&](int tile, int& b, int& oy0, int& ox0, int& n0) {
    int t = tile;
    const int nb = t % nblk_n; t /= nblk_n;
    const int tx = t % tiles_x; t /= tiles_x;
    const int ty = t % tiles_y; t /= tiles_y;
    b = t; oy0 = ty * TH; ox0 = tx * TW; n0 = nb * NB;
  };
  auto step_seg = [&](int step, int& si, int& c0) {
    si = 0;
    int s = step;
    while (s >= op.seg[si].C / 32) { s -= op.seg[si].C / 32; ++si; }
    c0 = s * 32;
  };
  auto kind_of = [&](const ConvSeg& sg) -> int {
    if constexpr (KM == 1) return 0;
    if constexpr (KM == 2) return 1;
    if constexpr (KM == 4) return 2;
    return step_kind(sg);
  };
  uint4 pf[C::PF];
  auto load = [&](int step, int tile) {
    int b, oy0, ox0, n0, si, c0;
    tile_coords(tile, b, oy0, ox0, n0);
    step_seg(step, si, c0);
    const ConvSeg& sg = op.seg[si];
    const int kind = kind_of(sg);
    if ((KM & 1) && kind == 0) {
      if (sg.pre != kPreMaxPool3) halo_load<T, NB, TH, 0>(pf, sg, b, oy0, ox0, c0, tid);
    } else if ((KM & 2) && kind == 1) {
      halo_load<T, NB, TH, 2>(pf, sg, b, oy0, ox0, c0, tid);
    } else if (KM & 4) {
      halo_load<T, NB, TH, 4>(pf, sg, b, oy0, ox0, c0, tid);
    }
  };
  auto stage_b = [&](const ConvSeg& sg, int c0, int n0) {
    const int nbq = sg.kh * sg.kw * NB * CCH;
    for (int q = tid; q < nbq; q += 256) {
      const int row = q / CCH, ch = q % CCH;  // row = tap*NB + n
      const int tap = row / NB, n = row % NB;
      *(uint4*)(Bs + row * PSTR + ch * EPC) =
          *(const uint4*)(W + (size_t)(n0 + n) * op.Kpad + sg.kbase + tap * sg.C + c0 + ch * EPC);
    }
  };

  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  if (b_keep) {
    int b, oy0, ox0, n0, si, c0;
    tile_coords(tile, b, oy0, ox0, n0);
    step_seg(0, si, c0);
    stage_b(op.seg[si], c0, n0);
  }
  if constexpr (PREF) load(0, tile);

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
    uint4 rr[PASSES];
    for (int step = 0; step < nsteps; ++step) {
      int si, c0;
      step_seg(step, si, c0);
      const ConvSeg& sg = op.seg[si];
      const int kind = kind_of(sg);
      if constexpr (!PREF) load(step, tile);
      __syncthreads();  // LDS free (previous step's MFMAs / previous tile's epilogue)
      if ((KM & 1) && kind == 0) {
        if (sg.pre == kPreMaxPool3)
          halo_pool<T, NB, TH>(sg, b, oy0, ox0, c0, tid, halo);
        else
          halo_store<T, NB, TH, 0>(pf, sg, oy0, ox0, c0, tid, halo);
      } else if ((KM & 2) && kind == 1) {
        halo_store<T, NB, TH, 2>(pf, sg, oy0, ox0, c0, tid, halo);
      } else if (KM & 4) {
        halo_store<T, NB, TH, 4>(pf, sg, oy0, ox0, c0, tid, halo);
      }
      if (!b_keep) stage_b(sg, c0, n0);
      __syncthreads();
      if constexpr (PREF) {
        const int nstep = step + 1 < nsteps ? step + 1 : 0;
        const int ntile = step + 1 < nsteps ? tile : tile + gridDim.x;
        if (ntile < ntiles) load(nstep, ntile);
      }
      if (step == nsteps - 1 && resp) {
        // residual chunks of this tile, requested before the last step's MFMAs
#pragma unroll
        for (int ps = 0; ps < PASSES; ++ps) {
          const int p = tid / CHN + ps * PPP;
          const int oy = oy0 + p / TW, ox = ox0 + p % TW;
          const size_t m = ((size_t)b * op.Ho + oy) * op.Wo + ox;
          rr[ps] = (oy < op.Ho && ox < op.Wo) ? *(const uint4*)(resp + m * res_cs + n0 + nb0) : make_uint4(0, 0, 0, 0);
        }
      }
      if ((KM & 1) && kind == 0)
        halo_taps<T, NB, TH, 1, 1>(acc, halo, Bs, wave, fr, fg);
      else if ((KM & 2) && kind == 1)
        halo_taps<T, NB, TH, 3, 1>(acc, halo, Bs, wave, fr, fg);
      else if (KM & 4)
        halo_taps<T, NB, TH, 3, 2>(acc, halo, Bs, wave, fr, fg);
    }

    // ---- epilogue ------------------------------------------------------------
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
    T* out = (T*)op.out;
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const int p = tid / CHN + ps * PPP;
      const int oy = oy0 + p / TW, ox = ox0 + p % TW;
      const bool valid = oy < op.Ho && ox < op.Wo;
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
        for (int e = 0; e < EPC; ++e) part += fmaxf(v[e], 0.f) * op.head_w[nb0 + e];
#pragma unroll
        for (int s = 1; s < CHN; s <<= 1) part += __shfl_xor(part, s);
        if (ch == 0 && valid) {
          float x0, x1, x2;
          const size_t pp = (size_t)oy * op.Wo + ox;
          if (op.x_f16) {
            const half_t* x = (const half_t*)op.x_nchw + (size_t)b * 3 * HWo + pp;
            x0 = (float)x[0]; x1 = (float)x[HWo]; x2 = (float)x[2 * HWo];
          } else {
            const float* x = op.x_nchw + (size_t)b * 3 * HWo + pp;
            x0 = x[0]; x1 = x[HWo]; x2 = x[2 * HWo];
          }
          const float z = (x0 + x1 + x2) / 3.f + (part + op.head_b);
          op.illu[m] = 1.f / (1.f + expf(-z));
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
      *(uint4*)(out + m * op.out_cs + op.out_coff + n0 + nb0) = o;
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
        atomicAdd(op.pool + b * op.N + n0 + tid, s);
      }
    }
  }
}

template <typename T, int NB, int TH, int OCC, int KM>
static int launch_halo_cfg(const ConvOp& op, hipStream_t st) {
  const int tiles_x = cdiv(op.Wo, HALO_TW), tiles_y = cdiv(op.Ho, TH);
  const int ntiles = op.B * tiles_x * tiles_y * (op.N / NB);
  using C = HaloCfg<T, NB, TH>;
  // LDS: region for the largest halo extent / tap count among this op's segments
  int ext = 0, taps = 1;
  for (int s = 0; s < op.nseg; ++s) {
    const int e = (op.seg[s].kh - 1) * op.seg[s].dil;
    ext = e > ext ? e : ext;
    taps = op.seg[s].kh * op.seg[s].kw > taps ? op.seg[s].kh * op.seg[s].kw : taps;
  }
  const int halo_bytes = (TH + ext) * (HALO_TW + ext) * C::PSTR * (int)sizeof(T);
  const int region = (int)align_up((size_t)(halo_bytes > C::EPI_BYTES ? halo_bytes : C::EPI_BYTES), 16);
  const int lds = region + taps * NB * C::PSTR * (int)sizeof(T);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)conv_halo_kernel<T, NB, TH, OCC, KM>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  // Persistent grid = blocks that are actually co-resident (registers AND LDS);
  // an oversized grid leaves a second, partial wave of blocks (tail).  Speed only.
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)conv_halo_kernel<T, NB, TH, OCC, KM>, 256,
                                                   lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const int lds_cap = (160 * 1024) / lds;
  if (per_cu > lds_cap) per_cu = lds_cap < 1 ? 1 : lds_cap;
  int grid = 256 * per_cu;
  if (grid > ntiles) grid = ntiles;
  hipLaunchKernelGGL((conv_halo_kernel<T, NB, TH, OCC, KM>), dim3(grid), dim3(256), lds, st, op, tiles_x, tiles_y,
                     ntiles, region);
  return (int)hipGetLastError();
}

template <typename T, int NB, int KM>
static int launch_halo_th(const ConvOp& op, int th, int occ, hipStream_t st) {
  if constexpr (KM == 2) {  // single-kind ops: registers leave room for 2-3 blocks per CU
    if (th == 4) {
      if (occ >= 3) return launch_halo_cfg<T, NB, 4, 3, KM>(op, st);
      return occ == 2 ? launch_halo_cfg<T, NB, 4, 2, KM>(op, st) : launch_halo_cfg<T, NB, 4, 1, KM>(op, st);
    }
    return occ >= 2 ? launch_halo_cfg<T, NB, 8, 2, KM>(op, st) : launch_halo_cfg<T, NB, 8, 1, KM>(op, st);
  }
  return th == 4 ? launch_halo_cfg<T, NB, 4, 1, KM>(op, st) : launch_halo_cfg<T, NB, 8, 1, KM>(op, st);
}

template <typename T, int NB>
static int launch_halo_km(const ConvOp& op, int km, int th, int occ, hipStream_t st) {
  if (km == 2) return launch_halo_th<T, NB, 2>(op, th, occ, st);
  return launch_halo_th<T, NB, 7>(op, th, occ, st);
}

// Tile rows / occupancy per layer class; UPR_HALO="<th>,<occ>" overrides (experiments).
// Measured on MI355X (tools/halo_sweep.sh, UP-Retinex layer shapes, bs 32):
// single-kind 3x3 ops run 2 blocks per CU — fp16 with 8-row tiles, fp32 with
// 4-row tiles (8-row fp32 tiles need > 256 registers); mixed-kind ops (the
// FAM fusion GEMM, dilated convs) 8-row tiles, 1 block per CU.
static void halo_choice(int dtype, int N, int km, int& th, int& occ) {
  (void)N;
  if (km == 2) {
    th = dtype == kF16 ? 8 : 4;
    occ = 2;
  } else {
    th = 8;
    occ = 1;
  }
  const char* e = getenv("UPR_HALO");
  if (e) {
    int a = 0, b = 0;
    if (sscanf(e, "%d,%d", &a, &b) == 2 && (a == 4 || a == 8) && b >= 1 && b <= 3) { th = a; occ = b; }
  }
}

// Returns kErrUnsupported when the op is not a halo-kernel shape (caller falls back).
int launch_conv_halo(const ConvOp& op, int dtype, hipStream_t st) {
  if (op.store == kStoreConvT2x2) return kErrUnsupported;
  if (op.Wo < 24 || op.Ho < 8) return kErrUnsupported;
  for (int s = 0; s < op.nseg; ++s) {
    const ConvSeg& g = op.seg[s];
    if (g.stride != 1 || g.kh != g.kw) return kErrUnsupported;
    if (g.kh == 3) {
      if (g.dil < 1 || g.dil > HALO_MAXEXT / 2 || g.pad != g.dil) return kErrUnsupported;
    } else if (g.kh == 1) {
      if (g.pad != 0) return kErrUnsupported;
      if (g.pre == kPreMaxPool3 && g.dil != 1) return kErrUnsupported;
    } else {
      return kErrUnsupported;
    }
    if (g.Hin != op.Ho || g.Win != op.Wo) return kErrUnsupported;
  }
  const int elt = dtype == kF16 ? 2 : 4;
  if (op.out && ((op.out_cs * elt) % 16 || (op.out_coff * elt) % 16)) return kErrUnsupported;
  if (op.res1 && (op.res1_cs * elt) % 16) return kErrUnsupported;
  if (op.res2 && (op.res2_cs * elt) % 16) return kErrUnsupported;
  if (op.res1 && op.res2) return kErrUnsupported;
  if (op.store == kStoreHeadIllu && op.N != 32) return kErrUnsupported;
  if (op.bias && ((uintptr_t)op.bias % 16)) return kErrUnsupported;
  if (op.scale) return kErrUnsupported;  // the graph folds every scale into the weights
  int km = 0;
  for (int s = 0; s < op.nseg; ++s) km |= 1 << (op.seg[s].kh == 1 ? 0 : (op.seg[s].dil == 1 ? 1 : 2));
  int th, occ;
  halo_choice(dtype, op.N, km, th, occ);
  if (dtype == kF16) {
    if (op.N == 32) return launch_halo_km<half_t, 32>(op, km, th, occ, st);
    if (op.N % 64 == 0) return launch_halo_km<half_t, 64>(op, km, th, occ, st);
  } else {
    if (op.N % 32 == 0) return launch_halo_km<float, 32>(op, km, th, occ, st);
  }
  return kErrUnsupported;
}

}  // namespace upr
