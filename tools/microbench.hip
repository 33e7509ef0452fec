// Micro-benchmarks for per-packet costs in k_execute (diagnostic tool, not the product).
// Build: hipcc --offload-arch=gfx950 -O3 -I../include tools/microbench.hip -o tools/microbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#include "sgn_workload.h"

__global__ void k_digest(uint64_t* out, int iters, uint64_t* clk) {
  uint64_t h = threadIdx.x + 1;
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++) h = sgn_digest3(h, 946684800000000000ULL + i, 17, 12345 + i);
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  out[threadIdx.x] = h;
  if (threadIdx.x == 0) {
    clk[0] = c1 - c0;
    clk[1] = r1 - r0;
  }
}

__global__ void k_xoshiro(uint64_t* out, int iters, uint64_t* clk) {
  uint64_t a = threadIdx.x + 1, b = 2, c = 3, d = 4;
  double acc = 0;
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++) {
    const uint64_t res = ((a + d) << 23 | (a + d) >> 41) + a;
    const uint64_t t = b << 17;
    c ^= a;
    d ^= b;
    b ^= c;
    a ^= d;
    c ^= t;
    d = (d << 45) | (d >> 19);
    const double x = (double)(res >> 11) * 0x1.0p-53;
    acc += x >= 0.99 ? 1.0 : 0.0;
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  out[threadIdx.x] = a ^ (uint64_t)acc;
  if (threadIdx.x == 0) {
    clk[0] = c1 - c0;
    clk[1] = r1 - r0;
  }
}

// dependent global loads (pointer chase) to read latency
__global__ void k_chase(const uint32_t* next, int iters, uint64_t* clk, uint32_t* sink) {
  uint32_t p = 0;
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++) p = next[p];
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  sink[0] = p;
  clk[0] = c1 - c0;
  clk[1] = r1 - r0;
}

int main() {
  uint64_t *out, *clk;
  hipMalloc(&out, 64 * 8);
  hipMalloc(&clk, 16);
  uint64_t h[2];
  const int iters = 10000;
  for (int lanes : {1, 64}) {
    hipLaunchKernelGGL(k_digest, 1, lanes, 0, 0, out, iters, clk);
    hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    printf("digest3 lanes=%d: %.1f memtime/iter, %.1f ns/iter, memtime/ns=%.3f\n", lanes,
           (double)h[0] / iters, h[1] * 10.0 / iters, (double)h[0] / (h[1] * 10.0));
    hipLaunchKernelGGL(k_xoshiro, 1, lanes, 0, 0, out, iters, clk);
    hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    printf("xoshiro+f64 lanes=%d: %.1f memtime/iter, %.1f ns/iter\n", lanes, (double)h[0] / iters,
           h[1] * 10.0 / iters);
  }
  // pointer chase over 256 MB (HBM) and 1 MB (L2)
  for (size_t bytes : {(size_t)1 << 20, (size_t)256 << 20}) {
    const size_t n = bytes / 4;
    uint32_t* hn = (uint32_t*)malloc(bytes);
    const size_t stride = 4099;  // words: defeats the prefetch of neighbouring lines
    for (size_t i = 0; i < n; i++) hn[i] = (uint32_t)((i + stride) % n);
    uint32_t *dn, *sink;
    hipMalloc(&dn, bytes);
    hipMalloc(&sink, 4);
    hipMemcpy(dn, hn, bytes, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_chase, 1, 1, 0, 0, dn, 2000, clk, sink);
    hipLaunchKernelGGL(k_chase, 1, 1, 0, 0, dn, 2000, clk, sink);
    hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    printf("chase %zu MB: %.1f memtime/load, %.1f ns/load\n", bytes >> 20, h[0] / 2000.0,
           h[1] * 10.0 / 2000.0);
    hipFree(dn);
    hipFree(sink);
    free(hn);
  }
  return 0;
}
