// Elementwise HBM-rate probe for the BatchNorm-backward apply pattern
// (g fp32 in, x fp16 in, dx fp32 out, dx16 fp16 out; C = 32 channels):
// variants differ only in per-thread width, rows per thread and store hints.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/ewbench tools/ewbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef _Float16 half_t;
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

struct P { const float* g; const half_t* x; float* dx; half_t* dx16; int M; int C; };

__device__ __forceinline__ float f(float g, float x, float a, float b) { return a * (g - b * x); }

// v0: the training kernel's form: 4 channels per thread, one row group per thread
__global__ __launch_bounds__(256) void v0(P p) {
  const int C4 = p.C / 4, c = (threadIdx.x % C4) * 4, rpb = 256 / C4;
  for (int m = blockIdx.x * rpb + threadIdx.x / C4; m < p.M; m += gridDim.x * rpb) {
    const float4 g = *(const float4*)(p.g + (size_t)m * p.C + c);
    const h4 x = *(const h4*)(p.x + (size_t)m * p.C + c);
    float4 r = make_float4(f(g.x, x[0], 1.1f, .3f), f(g.y, x[1], 1.1f, .3f), f(g.z, x[2], 1.1f, .3f), f(g.w, x[3], 1.1f, .3f));
    *(float4*)(p.dx + (size_t)m * p.C + c) = r;
    *(h4*)(p.dx16 + (size_t)m * p.C + c) = h4{(half_t)r.x, (half_t)r.y, (half_t)r.z, (half_t)r.w};
  }
}

// v0p: v0 with the training kernel's per-thread prologue (6 per-channel
// arrays, fp64 sums divided by M); DIV 0 multiplies by a host-side 1/M
template <int DIV>
__global__ __launch_bounds__(256) void v0p(P p, const float* mean, const float* invstd, const float* gamma,
                                           const double* acc, double invM) {
  const int C4 = p.C / 4, c = (threadIdx.x % C4) * 4, rpb = 256 / C4, C = p.C, M = p.M;
  float mu[4], is[4], sg[4], sgx[4], gis[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    mu[e] = mean[c + e];
    is[e] = invstd[c + e];
    sg[e] = DIV ? (float)(acc[c + e] / M) : (float)(acc[c + e] * invM);
    sgx[e] = DIV ? (float)(acc[C + c + e] / M) : (float)(acc[C + c + e] * invM);
    gis[e] = gamma[c + e] * is[e];
  }
  for (int m = blockIdx.x * rpb + threadIdx.x / C4; m < p.M; m += gridDim.x * rpb) {
    const float4 g = *(const float4*)(p.g + (size_t)m * p.C + c);
    const h4 x = *(const h4*)(p.x + (size_t)m * p.C + c);
    const float ga[4] = {g.x, g.y, g.z, g.w};
    float r[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = gis[e] * (ga[e] - sg[e] - ((float)x[e] - mu[e]) * is[e] * sgx[e]);
    *(float4*)(p.dx + (size_t)m * p.C + c) = make_float4(r[0], r[1], r[2], r[3]);
    *(h4*)(p.dx16 + (size_t)m * p.C + c) = h4{(half_t)r[0], (half_t)r[1], (half_t)r[2], (half_t)r[3]};
  }
}

// v1: 8 channels per thread (16-byte fp16 accesses)
template <int NT>
__global__ __launch_bounds__(256) void v1(P p) {
  const int C8 = p.C / 8, c = (threadIdx.x % C8) * 8, rpb = 256 / C8;
  for (int m = blockIdx.x * rpb + threadIdx.x / C8; m < p.M; m += gridDim.x * rpb) {
    const float4 g0 = *(const float4*)(p.g + (size_t)m * p.C + c);
    const float4 g1 = *(const float4*)(p.g + (size_t)m * p.C + c + 4);
    const h8 x = *(const h8*)(p.x + (size_t)m * p.C + c);
    const float ga[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    float r[8];
    h8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) { r[e] = f(ga[e], x[e], 1.1f, .3f); o[e] = (half_t)r[e]; }
    float4* d = (float4*)(p.dx + (size_t)m * p.C + c);
    if (NT) {
      typedef float f4 __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(f4{r[0], r[1], r[2], r[3]}, (f4*)d);
      __builtin_nontemporal_store(f4{r[4], r[5], r[6], r[7]}, (f4*)d + 1);
      __builtin_nontemporal_store(o, (h8*)(p.dx16 + (size_t)m * p.C + c));
    } else {
      d[0] = make_float4(r[0], r[1], r[2], r[3]);
      d[1] = make_float4(r[4], r[5], r[6], r[7]);
      *(h8*)(p.dx16 + (size_t)m * p.C + c) = o;
    }
  }
}

// v2: 4 channels per thread, U row groups per thread with all loads issued first
template <int U>
__global__ __launch_bounds__(256) void v2(P p) {
  const int C4 = p.C / 4, c = (threadIdx.x % C4) * 4, rpb = 256 / C4;
  const int stride = gridDim.x * rpb;
  for (int m0 = blockIdx.x * rpb + threadIdx.x / C4; m0 < p.M; m0 += stride * U) {
    float4 g[U];
    h4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = m0 + u * stride;
      if (m < p.M) { g[u] = *(const float4*)(p.g + (size_t)m * p.C + c); x[u] = *(const h4*)(p.x + (size_t)m * p.C + c); }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = m0 + u * stride;
      if (m >= p.M) break;
      float4 r = make_float4(f(g[u].x, x[u][0], 1.1f, .3f), f(g[u].y, x[u][1], 1.1f, .3f), f(g[u].z, x[u][2], 1.1f, .3f),
                             f(g[u].w, x[u][3], 1.1f, .3f));
      *(float4*)(p.dx + (size_t)m * p.C + c) = r;
      *(h4*)(p.dx16 + (size_t)m * p.C + c) = h4{(half_t)r.x, (half_t)r.y, (half_t)r.z, (half_t)r.w};
    }
  }
}

// v3: 8 channels per thread, 2 row groups per thread, loads first
__global__ __launch_bounds__(256) void v3(P p) {
  const int C8 = p.C / 8, c = (threadIdx.x % C8) * 8, rpb = 256 / C8;
  const int stride = gridDim.x * rpb;
  for (int m0 = blockIdx.x * rpb + threadIdx.x / C8; m0 < p.M; m0 += 2 * stride) {
    float4 g[2][2];
    h8 x[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = m0 + u * stride;
      if (m < p.M) {
        g[u][0] = *(const float4*)(p.g + (size_t)m * p.C + c);
        g[u][1] = *(const float4*)(p.g + (size_t)m * p.C + c + 4);
        x[u] = *(const h8*)(p.x + (size_t)m * p.C + c);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = m0 + u * stride;
      if (m >= p.M) break;
      const float ga[8] = {g[u][0].x, g[u][0].y, g[u][0].z, g[u][0].w, g[u][1].x, g[u][1].y, g[u][1].z, g[u][1].w};
      float r[8];
      h8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) { r[e] = f(ga[e], x[u][e], 1.1f, .3f); o[e] = (half_t)r[e]; }
      float4* d = (float4*)(p.dx + (size_t)m * p.C + c);
      d[0] = make_float4(r[0], r[1], r[2], r[3]);
      d[1] = make_float4(r[4], r[5], r[6], r[7]);
      *(h8*)(p.dx16 + (size_t)m * p.C + c) = o;
    }
  }
}

// copy ceiling: fp32 in -> fp32 out, 16 B per thread
__global__ __launch_bounds__(256) void vcopy(const float4* a, float4* b, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) b[i] = a[i];
}

int main() {
  const int M = 8 * 512 * 512, C = 32;
  const size_t n = (size_t)M * C;
  float *g, *dx; half_t *x, *dx16;
  hipMalloc(&g, n * 4); hipMalloc(&dx, n * 4); hipMalloc(&x, n * 2); hipMalloc(&dx16, n * 2);
  hipMemset(g, 0, n * 4); hipMemset(x, 0, n * 2);
  P p{g, x, dx, dx16, M, C};
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = n * 12.0;
  auto run = [&](const char* name, auto launch, double b) {
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(e0);
    const int R = 20;
    for (int i = 0; i < R; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    ms /= R;
    printf("%-28s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, b / (ms * 1e-3) / 1e12);
  };
  const int g4 = (int)(n / 4 / 256), g8 = (int)(n / 8 / 256);
  run("v0 4ch 1row", [&] { hipLaunchKernelGGL(v0, dim3(g4 > 65536 ? 65536 : g4), dim3(256), 0, 0, p); }, bytes);
  float* par; double* acc;
  hipMalloc(&par, 4096 * 4); hipMalloc(&acc, 4096 * 8);
  hipMemset(par, 0, 4096 * 4); hipMemset(acc, 0, 4096 * 8);
  run("v0p div", [&] { hipLaunchKernelGGL(v0p<1>, dim3(g4 > 65536 ? 65536 : g4), dim3(256), 0, 0, p, par, par + 1024, par + 2048, acc, 1.0 / M); }, bytes);
  run("v0p mul", [&] { hipLaunchKernelGGL(v0p<0>, dim3(g4 > 65536 ? 65536 : g4), dim3(256), 0, 0, p, par, par + 1024, par + 2048, acc, 1.0 / M); }, bytes);
  run("v0p div grid/4", [&] { hipLaunchKernelGGL(v0p<1>, dim3(g4 / 4), dim3(256), 0, 0, p, par, par + 1024, par + 2048, acc, 1.0 / M); }, bytes);
  run("v0p mul grid/4", [&] { hipLaunchKernelGGL(v0p<0>, dim3(g4 / 4), dim3(256), 0, 0, p, par, par + 1024, par + 2048, acc, 1.0 / M); }, bytes);
  run("v1 8ch", [&] { hipLaunchKernelGGL(v1<0>, dim3(g8), dim3(256), 0, 0, p); }, bytes);
  run("v1 8ch nt", [&] { hipLaunchKernelGGL(v1<1>, dim3(g8), dim3(256), 0, 0, p); }, bytes);
  for (int k : {4, 8, 16, 32}) {
    char nm[64];
    snprintf(nm, 64, "v1 8ch grid cus*%d", k);
    run(nm, [&] { hipLaunchKernelGGL(v1<0>, dim3(cus * k), dim3(256), 0, 0, p); }, bytes);
    snprintf(nm, 64, "v2<4> grid cus*%d", k);
    run(nm, [&] { hipLaunchKernelGGL(v2<4>, dim3(cus * k), dim3(256), 0, 0, p); }, bytes);
    snprintf(nm, 64, "v3 grid cus*%d", k);
    run(nm, [&] { hipLaunchKernelGGL(v3, dim3(cus * k), dim3(256), 0, 0, p); }, bytes);
  }
  run("v2<2> full", [&] { hipLaunchKernelGGL(v2<2>, dim3(g4 / 2), dim3(256), 0, 0, p); }, bytes);
  run("v3 full", [&] { hipLaunchKernelGGL(v3, dim3(g8 / 2), dim3(256), 0, 0, p); }, bytes);
  const long long nc = (long long)(n / 4);  // g -> dx, 8 B per element
  run("copy f32 (same bytes)", [&] { hipLaunchKernelGGL(vcopy, dim3(cus * 16), dim3(256), 0, 0, (const float4*)g, (float4*)dx, nc); }, nc * 32.0);
  run("copy f32 full grid", [&] { hipLaunchKernelGGL(vcopy, dim3((int)(nc / 256)), dim3(256), 0, 0, (const float4*)g, (float4*)dx, nc); }, nc * 32.0);
  hipError_t e = hipGetLastError();
  printf("err %s\n", hipGetErrorString(e));
  return 0;
}
