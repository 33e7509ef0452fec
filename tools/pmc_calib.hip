// Calibration of FETCH_SIZE / WRITE_SIZE (rocprofv3) for the engine's access widths on gfx950
// (MI355X_MICROARCH.md: only 16-B/lane streaming reads and stores are calibrated). Each kernel
// touches N distinct random 128-B lines of a 2 GiB buffer (far beyond L2 + Infinity Cache), one
// access per lane; the bytes requested per access are known, so counter bytes / N gives the
// fabric bytes one access of that kind costs. Diagnostic tool, not the product.
// Build: hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint64_t line_of(uint64_t i, uint64_t nlines) {
  uint64_t x = i * 0x9E3779B97F4A7C15ULL;
  x ^= x >> 29;
  return x % nlines;
}
// 0: 8-B device-scope atomic load (ld_dev), 1: 16-B plain load, 2: 32-B record (two 16-B),
// 3: 128-B line as 8 lanes x 16 B (coalesced), 4: 8-B device-scope store (st_dev),
// 5: 16-B plain store, 6: 32-B device-scope record store (4 x st_dev 8 B)
__global__ void k(uint64_t* buf, uint64_t nlines, uint64_t n, int mode, uint64_t* sink) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t acc = 0;
  if (mode == 3) {
    const uint64_t ln = line_of(i / 8, nlines);
    const uint4 v = ((const uint4*)(buf + ln * 16))[i % 8];
    acc = v.x ^ v.w;
  } else {
    const uint64_t ln = line_of(i, nlines);
    uint64_t* p = buf + ln * 16;
    if (mode == 0) acc = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (mode == 1) { const uint4 v = *(const uint4*)p; acc = v.x ^ v.z; }
    if (mode == 2) { const uint4 v = ((const uint4*)p)[0], w = ((const uint4*)p)[1]; acc = v.x ^ w.z; }
    if (mode == 4) __hip_atomic_store(p, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (mode == 5) *(uint4*)p = make_uint4((uint32_t)i, 1, 2, 3);
    if (mode == 6)
      for (int q = 0; q < 4; q++) __hip_atomic_store(p + q, i + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (acc == 0x123456789ULL) sink[0] = acc;
}

int main() {
  const uint64_t bytes = 2ULL << 30, nlines = bytes / 128, n = 1 << 22;
  uint64_t *buf, *sink;
  hipMalloc(&buf, bytes);
  hipMalloc(&sink, 64);
  hipMemset(buf, 1, bytes);
  const char* names[] = {"ld_dev 8B", "load 16B", "record 32B", "line 8x16B", "st_dev 8B", "store 16B", "st_dev record 32B"};
  const double req[] = {8, 16, 32, 16, 8, 16, 32};
  for (int mode = 0; mode < 7; mode++) {
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, buf, nlines, n, mode, sink);
    hipDeviceSynchronize();
    printf("mode %d %-18s accesses %llu requested bytes/access %.0f\n", mode, names[mode], (unsigned long long)n, req[mode]);
  }
  return 0;
}
