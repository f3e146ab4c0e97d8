// Halo-tiled direct convolution for gfx950 (stride-1 3x3 / 1x1 segments).
//
// The generic implicit-GEMM kernel (conv.hip) re-reads the A operand once per
// filter tap.  Here a block owns an 8 x 32 output-pixel tile of one image and
// stages, per (segment, 32-channel chunk), the input REGION the tile needs
// (tile + (k-1)*dil halo) into LDS once; all taps then read their A fragments
// from LDS at shifted offsets.  The chunk's weights for every tap are staged
// next to it.  Blocks loop over tiles (persistent grid).
//
// Epilogue goes through LDS so every global store / residual load is a full
// 16-byte chunk of consecutive channels (NHWC rows are contiguous).
//
// MFMA fragment convention as in conv.hip: lane (r = lane&15, g = lane>>4)
// owns 8 consecutive channels [8g, 8g+8) of pixel / weight row r.
#include "upr_common.h"

namespace upr {

typedef float f32x4_h __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8_h __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float hto_f(float v) { return v; }
__device__ __forceinline__ float hto_f(half_t v) { return (float)v; }
template <typename T> __device__ __forceinline__ T hfrom_f(float v);
template <> __device__ __forceinline__ float hfrom_f<float>(float v) { return v; }
template <> __device__ __forceinline__ half_t hfrom_f<half_t>(float v) { return (half_t)v; }

template <typename T> struct HaloCfg {
  static constexpr int EPC = 16 / sizeof(T);   // elements per 16-byte chunk
  static constexpr int CCH = 32 / EPC;         // chunks per 32-channel slice
  static constexpr int PSTR = 32 + EPC;        // LDS pixel stride (elements), odd # of 16B chunks
};

constexpr int HALO_TW = 32;
constexpr int HALO_MAXPAD = 2;  // 3x3 with dilation <= 2

template <typename T, int NB, int TH>
struct HaloLds {
  static constexpr int PSTR = HaloCfg<T>::PSTR;
  static constexpr int HH = TH + 2 * HALO_MAXPAD;
  static constexpr int HW = HALO_TW + 2 * HALO_MAXPAD;
  static constexpr int HALO_ELEMS = HH * HW * PSTR;
  static constexpr int B_ELEMS = 9 * NB * PSTR;
  static constexpr int CSTR = NB + 4;  // fp32 epilogue staging stride
  static constexpr int MAIN_BYTES = (HALO_ELEMS + B_ELEMS) * (int)sizeof(T);
  static constexpr int EPI_BYTES = TH * HALO_TW * CSTR * 4;
  static constexpr int BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
};

template <typename T, int NB, int TH>
__global__ __launch_bounds__(256) void conv_halo_kernel(ConvOp op, int tiles_x, int tiles_y, int ntiles) {
  constexpr int EPC = HaloCfg<T>::EPC;
  constexpr int CCH = HaloCfg<T>::CCH;
  constexpr int PSTR = HaloCfg<T>::PSTR;
  constexpr int TW = HALO_TW;
  constexpr int RPW = TH / 4;           // tile rows per wave
  constexpr int MT = 2 * RPW;           // 16-pixel M tiles per wave
  constexpr int NT = NB / 16;           // 16-channel N tiles
  using LDS = HaloLds<T, NB, TH>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS::BYTES];
  T* halo = (T*)smem;
  T* Bs = halo + LDS::HALO_ELEMS;
  float* Cs = (float*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int nblk_n = op.N / NB;
  const int HWo = op.Ho * op.Wo;

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int t = tile;
    const int nb = t % nblk_n; t /= nblk_n;
    const int tx = t % tiles_x; t /= tiles_x;
    const int ty = t % tiles_y; t /= tiles_y;
    const int b = t;
    const int oy0 = ty * TH, ox0 = tx * TW, n0 = nb * NB;

    f32x4_h acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_h{0.f, 0.f, 0.f, 0.f};

    for (int si = 0; si < op.nseg; ++si) {
      const ConvSeg& sg = op.seg[si];
      const int k = sg.kh;                  // 1 or 3 (square)
      const int d = sg.dil;
      const int ext = (k - 1) * d;          // halo extent
      const int hh = TH + ext, hw = TW + ext;
      const int ntap = k * k;
      const T* src = (const T*)sg.src;
      for (int c0 = 0; c0 < sg.C; c0 += 32) {
        __syncthreads();  // previous chunk's compute / previous tile's epilogue done
        // ---- stage the input region (zero padded) ----
        const int nch = hh * hw * CCH;
        for (int q = tid; q < nch; q += 256) {
          const int px = q / CCH, ch = q - px * CCH;
          const int hy = px / hw, hx = px - hy * hw;
          const int iy = oy0 - sg.pad + hy, ix = ox0 - sg.pad + hx;
          const int cb = c0 + ch * EPC;
          uint4 v = make_uint4(0, 0, 0, 0);
          if (iy >= 0 && iy < sg.Hin && ix >= 0 && ix < sg.Win) {
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
                  const uint4 w = *(const uint4*)(src + (((size_t)b * sg.Hin + yy) * sg.Win + xx) * sg.cs +
                                                  sg.coff + cb);
                  const T* wv = (const T*)&w;
#pragma unroll
                  for (int e = 0; e < EPC; ++e) mx[e] = fmaxf(mx[e], hto_f(wv[e]));
                }
              }
              T* vv = (T*)&v;
#pragma unroll
              for (int e = 0; e < EPC; ++e) vv[e] = hfrom_f<T>(mx[e]);
            } else {
              v = *(const uint4*)(src + (((size_t)b * sg.Hin + iy) * sg.Win + ix) * sg.cs + sg.coff + cb);
              if (sg.pre == kPreAffineRelu) {
                T* vv = (T*)&v;
#pragma unroll
                for (int e = 0; e < EPC; ++e)
                  vv[e] = hfrom_f<T>(fmaxf(hto_f(vv[e]) * sg.pre_scale[cb + e] + sg.pre_shift[cb + e], 0.f));
              }
            }
          }
          *(uint4*)(halo + (hy * hw + hx) * PSTR + ch * EPC) = v;
        }
        // ---- stage the weights of every tap for this chunk ----
        const T* W = (const T*)op.W;
        const int nbq = ntap * NB * CCH;
        for (int q = tid; q < nbq; q += 256) {
          const int row = q / CCH, ch = q - row * CCH;  // row = tap*NB + n
          const int tap = row / NB, n = row - tap * NB;
          *(uint4*)(Bs + row * PSTR + ch * EPC) =
              *(const uint4*)(W + (size_t)(n0 + n) * op.Kpad + sg.kbase + tap * sg.C + c0 + ch * EPC);
        }
        __syncthreads();
        // ---- taps ----
        for (int tap = 0; tap < ntap; ++tap) {
          const int r = tap / k, c = tap - r * k;
          const int oy = r * d, ox = c * d;
          if constexpr (sizeof(T) == 2) {
            f16x8_h bf[NT];
#pragma unroll
            for (int j = 0; j < NT; ++j)
              bf[j] = *(const f16x8_h*)(Bs + ((tap * NB) + j * 16 + fr) * PSTR + fg * 8);
#pragma unroll
            for (int i = 0; i < MT; ++i) {
              const int py = wave * RPW + (i >> 1), pxx = (i & 1) * 16 + fr;
              const f16x8_h af = *(const f16x8_h*)(halo + ((py + oy) * hw + pxx + ox) * PSTR + fg * 8);
#pragma unroll
              for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], acc[i][j], 0, 0, 0);
            }
          } else {
            f32x4_h bf[NT][2];
#pragma unroll
            for (int j = 0; j < NT; ++j) {
              const float* p = (const float*)Bs + ((tap * NB) + j * 16 + fr) * PSTR + fg * 8;
              bf[j][0] = *(const f32x4_h*)p;
              bf[j][1] = *(const f32x4_h*)(p + 4);
            }
#pragma unroll
            for (int i = 0; i < MT; ++i) {
              const int py = wave * RPW + (i >> 1), pxx = (i & 1) * 16 + fr;
              const float* p = (const float*)halo + ((py + oy) * hw + pxx + ox) * PSTR + fg * 8;
              const f32x4_h a0 = *(const f32x4_h*)p, a1 = *(const f32x4_h*)(p + 4);
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float av = e < 4 ? a0[e] : a1[e - 4];
#pragma unroll
                for (int j = 0; j < NT; ++j)
                  acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bf[j][e >> 2][e & 3], acc[i][j], 0, 0, 0);
              }
            }
          }
        }
      }
    }

    // ---- epilogue: stage fp32 accumulators, then coalesced 16-byte passes ----
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int py = wave * RPW + (i >> 1), px0 = (i & 1) * 16 + fg * 4;
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) Cs[(py * TW + px0 + e) * LDS::CSTR + j * 16 + fr] = acc[i][j][e];
    }
    __syncthreads();

    constexpr int CHN = NB / EPC;          // 16-byte chunks per pixel of the block's channel slice
    constexpr int PPP = 256 / CHN;         // pixels per pass
    const int ch = tid % CHN;
    const int nb0 = ch * EPC;              // first channel (within the block slice) of this thread
    float bias_v[EPC], scale_v[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      bias_v[e] = op.bias ? op.bias[n0 + nb0 + e] : 0.f;
      scale_v[e] = op.scale ? op.scale[n0 + nb0 + e] : 1.f;
    }
    float psum[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) psum[e] = 0.f;
    T* out = (T*)op.out;
    for (int p = tid / CHN; p < TH * TW; p += PPP) {
      const int py = p / TW, pxx = p - py * TW;
      const int oy = oy0 + py, ox = ox0 + pxx;
      const bool valid = oy < op.Ho && ox < op.Wo;
      const size_t m = ((size_t)b * op.Ho + oy) * op.Wo + ox;
      float v[EPC];
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] = Cs[p * LDS::CSTR + nb0 + e] * scale_v[e] + bias_v[e];
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
      if (op.res1) {
        const uint4 rr = *(const uint4*)((const T*)op.res1 + m * op.res1_cs + n0 + nb0);
        const T* rv = (const T*)&rr;
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] += hto_f(rv[e]);
      }
      if (op.relu) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (op.res2) {
        const uint4 rr = *(const uint4*)((const T*)op.res2 + m * op.res2_cs + n0 + nb0);
        const T* rv = (const T*)&rr;
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] += hto_f(rv[e]);
      }
      uint4 o;
      T* ov = (T*)&o;
#pragma unroll
      for (int e = 0; e < EPC; ++e) ov[e] = hfrom_f<T>(v[e]);
      *(uint4*)(out + m * op.out_cs + op.out_coff + n0 + nb0) = o;
      if (op.pool) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) psum[e] += hto_f(ov[e]);
      }
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

template <typename T, int NB, int TH>
static int launch_halo_cfg(const ConvOp& op, hipStream_t st) {
  const int tiles_x = cdiv(op.Wo, HALO_TW), tiles_y = cdiv(op.Ho, TH);
  const int ntiles = op.B * tiles_x * tiles_y * (op.N / NB);
  int grid = ntiles;
  const int cap = 256 * 4;  // persistent: a few resident blocks per CU
  if (grid > cap) grid = cap;
  hipLaunchKernelGGL((conv_halo_kernel<T, NB, TH>), dim3(grid), dim3(256), 0, st, op, tiles_x, tiles_y, ntiles);
  return (int)hipGetLastError();
}

// Returns kErrUnsupported when the op is not a halo-kernel shape (caller falls back).
int launch_conv_halo(const ConvOp& op, int dtype, hipStream_t st) {
  if (op.store == kStoreConvT2x2) return kErrUnsupported;
  if (op.Wo < 24 || op.Ho < 8) return kErrUnsupported;
  for (int s = 0; s < op.nseg; ++s) {
    const ConvSeg& g = op.seg[s];
    if (g.stride != 1 || g.kh != g.kw) return kErrUnsupported;
    if (g.kh == 3) {
      if (g.dil < 1 || g.dil > HALO_MAXPAD || g.pad != g.dil) return kErrUnsupported;
    } else if (g.kh == 1) {
      if (g.pad != 0) return kErrUnsupported;
    } else {
      return kErrUnsupported;
    }
    if (g.Hin != op.Ho || g.Win != op.Wo) return kErrUnsupported;
  }
  const int elt = dtype == kF16 ? 2 : 4;
  if (op.out && ((op.out_cs * elt) % 16 || (op.out_coff * elt) % 16)) return kErrUnsupported;
  if (op.store == kStoreHeadIllu && op.N != 32) return kErrUnsupported;
  if (dtype == kF16) {
    if (op.N == 32) return launch_halo_cfg<half_t, 32, 8>(op, st);
    if (op.N % 64 == 0) return launch_halo_cfg<half_t, 64, 8>(op, st);
  } else {
    if (op.N % 32 == 0 && op.N <= 64) return launch_halo_cfg<float, 32, 8>(op, st);
  }
  return kErrUnsupported;
}

}  // namespace upr
