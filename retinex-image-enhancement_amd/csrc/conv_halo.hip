// Halo-tiled direct convolution for gfx950 (stride-1 3x3 / 1x1 segments).
//
// The generic implicit-GEMM kernel (conv.hip) re-reads the A operand once per
// filter tap.  Here a block owns an 8 x 32 output-pixel tile of one image and
// stages, per K step (= one segment x 32-channel chunk), the input REGION the
// tile needs (tile + (k-1)*dil halo) into LDS once; every tap then reads its A
// fragments from LDS at shifted offsets.  The step's weights for all taps sit
// next to it (staged once per block when the whole K is one step).
//
// Pipeline: blocks loop over tiles (persistent grid).  The region of the NEXT
// step (possibly of the next tile) is loaded into registers — prologue
// (pre-activation BN+ReLU, 3x3 max-pool) applied there — while the current
// step's MFMAs run; fragments of tap t+1 are read from LDS while tap t's MFMAs
// issue.  Epilogue goes through LDS so every global store / residual load is a
// full 16-byte chunk of consecutive channels (NHWC rows are contiguous).
//
// MFMA fragment convention as in conv.hip: lane (r = lane&15, g = lane>>4)
// owns 8 consecutive channels [8g, 8g+8) of pixel / weight row r.
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
constexpr int HALO_MAXPAD = 2;  // 3x3 with dilation <= 2

template <typename T, int NB, int TH>
struct HaloCfg {
  static constexpr int EPC = 16 / sizeof(T);   // elements per 16-byte chunk
  static constexpr int CCH = 32 / EPC;         // chunks per 32-channel slice
  static constexpr int PSTR = 32 + EPC;        // LDS pixel stride (elements): odd # of 16-B chunks
  static constexpr int HH = TH + 2 * HALO_MAXPAD;
  static constexpr int HWX = HALO_TW + 2 * HALO_MAXPAD;
  static constexpr int HALO_ELEMS = HH * HWX * PSTR;
  static constexpr int CSTR = NB + 4;          // fp32 epilogue staging stride
  static constexpr int EPI_BYTES = TH * HALO_TW * CSTR * 4;
  static constexpr int REGION_BYTES =
      HALO_ELEMS * (int)sizeof(T) > EPI_BYTES ? HALO_ELEMS * (int)sizeof(T) : EPI_BYTES;
  static constexpr int B_ELEMS = 9 * NB * PSTR;
  static constexpr int BYTES = REGION_BYTES + B_ELEMS * (int)sizeof(T);
  static constexpr int PF = (HH * HWX * CCH + 255) / 256;  // prefetch registers (uint4) per thread
};

template <typename T, int NB, int TH>
__global__ __launch_bounds__(256) void conv_halo_kernel(ConvOp op, int tiles_x, int tiles_y, int ntiles) {
  using C = HaloCfg<T, NB, TH>;
  constexpr int EPC = C::EPC, CCH = C::CCH, PSTR = C::PSTR;
  constexpr int TW = HALO_TW;
  constexpr int RPW = TH / 4;  // tile rows per wave
  constexpr int MT = 2 * RPW;  // 16-pixel M tiles per wave
  constexpr int NT = NB / 16;  // 16-channel N tiles
  __shared__ __attribute__((aligned(16))) unsigned char smem[C::BYTES];
  T* halo = (T*)smem;
  float* Cs = (float*)smem;
  T* Bs = (T*)(smem + C::REGION_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int nblk_n = op.N / NB;
  const int HWo = op.Ho * op.Wo;
  const T* W = (const T*)op.W;

  int nsteps = 0;
  for (int s = 0; s < op.nseg; ++s) nsteps += op.seg[s].C / 32;
  const bool b_resident = nsteps == 1;

  // tile index -> (b, oy0, ox0, n0)
  auto tile_coords = [&](int tile, int& b, int& oy0, int& ox0, int& n0) {
    int t = tile;
    const int nb = t % nblk_n; t /= nblk_n;
    const int tx = t % tiles_x; t /= tiles_x;
    const int ty = t % tiles_y; t /= tiles_y;
    b = t; oy0 = ty * TH; ox0 = tx * TW; n0 = nb * NB;
  };
  // K step -> (segment, first channel)
  auto step_seg = [&](int step, int& si, int& c0) {
    si = 0;
    int s = step;
    while (s >= op.seg[si].C / 32) { s -= op.seg[si].C / 32; ++si; }
    c0 = s * 32;
  };

  uint4 pf[C::PF];
  auto load_region = [&](int step, int tile) {
    int b, oy0, ox0, n0, si, c0;
    tile_coords(tile, b, oy0, ox0, n0);
    step_seg(step, si, c0);
    const ConvSeg& sg = op.seg[si];
    const int ext = (sg.kh - 1) * sg.dil;
    const int hh = TH + ext, hw = TW + ext;
    const int nch = hh * hw * CCH;
    const T* src = (const T*)sg.src;
    if (sg.pre == kPreMaxPool3) return;  // pooled synchronously in store_region (rare, 1x1 only)
    const T* base = src + (size_t)b * sg.Hin * sg.Win * sg.cs + sg.coff + c0;
#pragma unroll
    for (int j = 0; j < C::PF; ++j) {
      const int q = tid + j * 256;
      const int px = q / CCH, ch = q - px * CCH;
      const int hy = px / hw, hx = px - hy * hw;
      const int iy = oy0 - sg.pad + hy, ix = ox0 - sg.pad + hx;
      const bool ok = q < nch && iy >= 0 && iy < sg.Hin && ix >= 0 && ix < sg.Win;
      const T* p = base + ((size_t)iy * sg.Win + ix) * sg.cs + ch * EPC;
      pf[j] = ok ? *(const uint4*)p : make_uint4(0, 0, 0, 0);
    }
  };
  // 3x3/s1/p1 max-pool of the source for a 1x1 segment (EnhancedFAM branch2, model.py:32,69)
  auto pool_region = [&](int si, int c0, int b, int oy0, int ox0) {
    const ConvSeg& sg = op.seg[si];
    const T* src = (const T*)sg.src;
    for (int q = tid; q < TH * TW * CCH; q += 256) {
      const int px = q / CCH, ch = q - px * CCH;
      const int hy = px / TW, hx = px - hy * TW;
      const int iy = oy0 + hy, ix = ox0 + hx;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (iy < sg.Hin && ix < sg.Win) {
        float mx[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) mx[e] = -INFINITY;
        for (int dy = -1; dy <= 1; ++dy) {
          const int yy = iy + dy;
          if (yy < 0 || yy >= sg.Hin) continue;
          for (int dx = -1; dx <= 1; ++dx) {
            const int xx = ix + dx;
            if (xx < 0 || xx >= sg.Win) continue;
            const uint4 w4 = *(const uint4*)(src + (((size_t)b * sg.Hin + yy) * sg.Win + xx) * sg.cs + sg.coff + c0 +
                                             ch * EPC);
            const T* wv = (const T*)&w4;
#pragma unroll
            for (int e = 0; e < EPC; ++e) mx[e] = fmaxf(mx[e], hto_f(wv[e]));
          }
        }
        T* vv = (T*)&v;
#pragma unroll
        for (int e = 0; e < EPC; ++e) vv[e] = hfrom_f<T>(mx[e]);
      }
      *(uint4*)(halo + px * PSTR + ch * EPC) = v;
    }
  };
  // prologue transform + write to LDS (same q -> slot mapping as load_region)
  auto store_region = [&](int step, int tile) {
    int si, c0;
    step_seg(step, si, c0);
    const ConvSeg& sg = op.seg[si];
    const int ext = (sg.kh - 1) * sg.dil;
    const int hh = TH + ext, hw = TW + ext;
    const int nch = hh * hw * CCH;
    int b, oy0, ox0, n0;
    tile_coords(tile, b, oy0, ox0, n0);
    if (sg.pre == kPreMaxPool3) {
      pool_region(si, c0, b, oy0, ox0);
      return;
    }
#pragma unroll
    for (int j = 0; j < C::PF; ++j) {
      const int q = tid + j * 256;
      if (q < nch) {
        const int px = q / CCH, ch = q - px * CCH;
        uint4 v = pf[j];
        if (sg.pre == kPreAffineRelu) {
          const int hy = px / hw, hx = px - hy * hw;
          const int iy = oy0 - sg.pad + hy, ix = ox0 - sg.pad + hx;
          if (iy >= 0 && iy < sg.Hin && ix >= 0 && ix < sg.Win) {  // zero padding stays zero
            const int cb = c0 + ch * EPC;
            T* vv = (T*)&v;
#pragma unroll
            for (int e = 0; e < EPC; ++e)
              vv[e] = hfrom_f<T>(fmaxf(hto_f(vv[e]) * sg.pre_scale[cb + e] + sg.pre_shift[cb + e], 0.f));
          }
        }
        *(uint4*)(halo + px * PSTR + ch * EPC) = v;
      }
    }
  };
  auto stage_b = [&](int step, int n0) {
    int si, c0;
    step_seg(step, si, c0);
    const ConvSeg& sg = op.seg[si];
    const int nbq = sg.kh * sg.kw * NB * CCH;
    for (int q = tid; q < nbq; q += 256) {
      const int row = q / CCH, ch = q - row * CCH;  // row = tap*NB + n
      const int tap = row / NB, n = row - tap * NB;
      *(uint4*)(Bs + row * PSTR + ch * EPC) =
          *(const uint4*)(W + (size_t)(n0 + n) * op.Kpad + sg.kbase + tap * sg.C + c0 + ch * EPC);
    }
  };

  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  if (b_resident) {
    int b, oy0, ox0, n0;
    tile_coords(tile, b, oy0, ox0, n0);
    // all tiles of this block share n0 only if nblk_n == 1; otherwise restage per tile (below)
    if (nblk_n == 1) stage_b(0, n0);
  }
  load_region(0, tile);

  for (; tile < ntiles; tile += gridDim.x) {
    int b, oy0, ox0, n0;
    tile_coords(tile, b, oy0, ox0, n0);

    f32x4_h acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_h{0.f, 0.f, 0.f, 0.f};

    for (int step = 0; step < nsteps; ++step) {
      __syncthreads();  // LDS free (previous step's compute / previous tile's epilogue)
      store_region(step, tile);
      if (!(b_resident && nblk_n == 1)) stage_b(step, n0);
      __syncthreads();
      // prefetch the next step's region (next tile after the last step)
      {
        const int nstep = step + 1 < nsteps ? step + 1 : 0;
        const int ntile = step + 1 < nsteps ? tile : tile + gridDim.x;
        if (ntile < ntiles) load_region(nstep, ntile);
      }
      int si, c0;
      step_seg(step, si, c0);
      const ConvSeg& sg = op.seg[si];
      const int d = sg.dil;
      auto run_taps = [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int ntap = k * k;
        const int hw = TW + (k - 1) * d;
        if constexpr (sizeof(T) == 2) {
          f16x8_h af[2][MT], bf[2][NT];
#pragma unroll
          for (int tap = 0; tap < ntap; ++tap) {
            const int r = tap / k, c = tap % k;
            const int cur = tap & 1;
#pragma unroll
            for (int j = 0; j < NT; ++j)
              bf[cur][j] = *(const f16x8_h*)(Bs + ((tap * NB) + j * 16 + fr) * PSTR + fg * 8);
#pragma unroll
            for (int i = 0; i < MT; ++i) {
              const int py = wave * RPW + (i >> 1) + r * d, pxx = (i & 1) * 16 + fr + c * d;
              af[cur][i] = *(const f16x8_h*)(halo + (py * hw + pxx) * PSTR + fg * 8);
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
              for (int j = 0; j < NT; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[cur][i], bf[cur][j], acc[i][j], 0, 0, 0);
          }
        } else {
          f32x4_h af[2][MT][2], bf[2][NT][2];
#pragma unroll
          for (int tap = 0; tap < ntap; ++tap) {
            const int r = tap / k, c = tap % k;
            const int cur = tap & 1;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
              const float* p = (const float*)Bs + ((tap * NB) + j * 16 + fr) * PSTR + fg * 8;
              bf[cur][j][0] = *(const f32x4_h*)p;
              bf[cur][j][1] = *(const f32x4_h*)(p + 4);
            }
#pragma unroll
            for (int i = 0; i < MT; ++i) {
              const int py = wave * RPW + (i >> 1) + r * d, pxx = (i & 1) * 16 + fr + c * d;
              const float* p = (const float*)halo + (py * hw + pxx) * PSTR + fg * 8;
              af[cur][i][0] = *(const f32x4_h*)p;
              af[cur][i][1] = *(const f32x4_h*)(p + 4);
            }
#pragma unroll
            for (int e = 0; e < 8; ++e)
#pragma unroll
              for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                  acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[cur][i][e >> 2][e & 3], bf[cur][j][e >> 2][e & 3],
                                                                  acc[i][j], 0, 0, 0);
          }
        }
      };
      if (sg.kh == 3) run_taps(std::integral_constant<int, 3>{});
      else run_taps(std::integral_constant<int, 1>{});
    }

    // ---- epilogue: stage fp32 accumulators, then coalesced 16-byte passes ----
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

    constexpr int CHN = NB / EPC;   // 16-byte chunks per pixel of the block's channel slice
    constexpr int PPP = 256 / CHN;  // pixels per pass
    const int ch = tid % CHN;
    const int nb0 = ch * EPC;       // first channel (within the block slice) of this thread
    float bias_v[EPC], scale_v[EPC];
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
    if (op.scale) {
#pragma unroll
      for (int e = 0; e < EPC; ++e) scale_v[e] = op.scale[n0 + nb0 + e];
    } else {
#pragma unroll
      for (int e = 0; e < EPC; ++e) scale_v[e] = 1.f;
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
      for (int e = 0; e < EPC; ++e) v[e] = Cs[p * C::CSTR + nb0 + e] * scale_v[e] + bias_v[e];
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
  using C = HaloCfg<T, NB, TH>;
  const int per_cu = C::BYTES > 80 * 1024 ? 1 : (C::BYTES > 53 * 1024 ? 2 : 3);
  int grid = 256 * per_cu;  // persistent: one wave of resident blocks
  if (grid > ntiles) grid = ntiles;
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
