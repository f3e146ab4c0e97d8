// Measured ceilings of this chip, for the bench's roofline report (not on the
// model path).  The nominal peaks (2516.6 TF/s fp16 MFMA dense, 8.0 TB/s HBM)
// are not reachable by any kernel: the fp16 MFMA clock drops under load on
// random operands (MI355X_MICROARCH.md "DVFS give-back") and a streaming copy
// reaches ~79% of the HBM spec.  These two kernels measure what is reachable,
// with the same operands and the same clock behaviour as the conv kernels:
//   * UPR_CALIB_MFMA_F16: back-to-back v_mfma_f32_16x16x32_f16 on random fp16
//     operands held in registers, 8 independent accumulators per wave (no
//     LDS, no global traffic in the loop) — an upper bound for any fp16 conv;
//   * UPR_CALIB_HBM_COPY: a 16-byte-per-lane grid-stride copy of a buffer far
//     larger than the Infinity Cache (read + write counted).
#include "upr_common.h"
#include "../../include/upr.h"

namespace upr {

__global__ __launch_bounds__(256) void calib_mfma_kernel(const half_t* __restrict__ src, float* __restrict__ sink,
                                                         int iters) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int gw = (blockIdx.x * 4 + (threadIdx.x >> 6)) & 1023;  // the source holds 1024 waves' operands
  h8 a[2], b[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    a[i] = *(const h8*)(src + ((size_t)(gw * 4 + i) * 64 + lane) * 8);
    b[i] = *(const h8*)(src + ((size_t)(gw * 4 + 2 + i) * 64 + lane) * 8);
  }
  // the accumulators are tied in place (inline asm): hipcc's own schedule of
  // this loop rotates them through v_accvgpr moves between the MFMAs
  f4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
#define UPR_CALIB_MFMA(c, x, y) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(x), "v"(y))
  for (int it = 0; it < iters; ++it) {
    UPR_CALIB_MFMA(c0, a[0], b[0]);
    UPR_CALIB_MFMA(c1, a[1], b[0]);
    UPR_CALIB_MFMA(c2, a[0], b[1]);
    UPR_CALIB_MFMA(c3, a[1], b[1]);
    UPR_CALIB_MFMA(c4, b[0], a[0]);
    UPR_CALIB_MFMA(c5, b[1], a[0]);
    UPR_CALIB_MFMA(c6, b[0], a[1]);
    UPR_CALIB_MFMA(c7, b[1], a[1]);
  }
#undef UPR_CALIB_MFMA
  asm volatile("s_nop 7\n s_nop 7\n s_nop 2" ::: "memory");  // MFMA results -> VALU reads
  const f4 s = ((c0 + c1) + (c2 + c3)) + ((c4 + c5) + (c6 + c7));
  *(f4*)(sink + ((size_t)blockIdx.x * 256 + threadIdx.x) * 4) = s;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// mode 0: grid-stride, four 16-byte loads in flight per lane before their
// stores; mode 1: the same with non-temporal loads / stores; mode 2: each
// block copies one contiguous slice, 4 x 4 KiB per loop step
__global__ __launch_bounds__(256) void calib_copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                         size_t n, int mode) {
  size_t i, end, step;
  if (mode == 2) {
    const size_t per = (n + gridDim.x - 1) / gridDim.x;
    i = (size_t)blockIdx.x * per + threadIdx.x;
    end = min(n, (size_t)(blockIdx.x + 1) * per);
    step = 256;
  } else {
    i = (size_t)blockIdx.x * 256 + threadIdx.x;
    end = n;
    step = (size_t)gridDim.x * 256;
  }
  for (; i + 3 * step < end; i += 4 * step) {
    u32x4 v[4];
    if (mode == 1) {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + i + u * step);
#pragma unroll
      for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], dst + i + u * step);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = src[i + u * step];
#pragma unroll
      for (int u = 0; u < 4; ++u) dst[i + u * step] = v[u];
    }
  }
  for (; i < end; i += step) dst[i] = src[i];
}

}  // namespace upr

using namespace upr;

extern "C" int upr_calib_run(int which, int blocks, int iters, const void* src, void* dst, size_t bytes, int reps,
                             float* ms_per_launch, void* stream) {
  if (!src || !dst || !ms_per_launch || blocks <= 0 || reps <= 0) return UPR_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (which == UPR_CALIB_MFMA_F16) {
    // src: >= 1024 waves x 4 fragments x 64 lanes x 16 B of fp16; dst: blocks x 256 x 4 floats
    if (iters <= 0 || bytes < (size_t)1024 * 4 * 64 * 16) return UPR_ERR_ARG;
  } else if (which == UPR_CALIB_HBM_COPY) {
    if (iters < 0 || iters > 2 || bytes < 16 || bytes % 16 || ((uintptr_t)src | (uintptr_t)dst) % 16) return UPR_ERR_ARG;
  } else {
    return UPR_ERR_ARG;
  }
  hipEvent_t e0, e1;
  UPR_CHECK_HIP(hipEventCreate(&e0));
  UPR_CHECK_HIP(hipEventCreate(&e1));
  UPR_CHECK_HIP(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) {
    if (which == UPR_CALIB_MFMA_F16)
      hipLaunchKernelGGL(calib_mfma_kernel, dim3(blocks), dim3(256), 0, st, (const half_t*)src, (float*)dst, iters);
    else
      hipLaunchKernelGGL(calib_copy_kernel, dim3(blocks), dim3(256), 0, st, (const u32x4*)src, (u32x4*)dst,
                         bytes / 16, iters);
  }
  UPR_CHECK_HIP(hipGetLastError());
  UPR_CHECK_HIP(hipEventRecord(e1, st));
  UPR_CHECK_HIP(hipEventSynchronize(e1));
  float ms = 0.f;
  UPR_CHECK_HIP(hipEventElapsedTime(&ms, e0, e1));
  *ms_per_launch = ms / (float)reps;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return UPR_OK;
}
