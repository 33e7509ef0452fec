// Cycles per screened xoshiro256++ draw (the TGEN kernel's loss loop, send_batch) for ONE wave
// of a CU while the CU's other waves do something else (diagnostic tool, not the product):
// one 512-thread workgroup per CU, wave 0 runs the loop on `busy` lanes, waves 1..7 run a
// background pattern until wave 0 is done (an LDS flag):
//   0 idle, 1 poll a global word with device-scope loads and s_sleep (a barrier wait),
//   2 the same loop on every lane (VALU), 3 a dependent global-load chain (a gather),
//   4 LDS traffic (an event sort), 5 scalar loads + SALU (the event loop's control).
// Build: hipcc --offload-arch=gfx950 -O3 tools/rng_situ_bench.hip -o tools/rng_situ_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

__device__ __forceinline__ uint32_t lo32(uint64_t x) { return (uint32_t)x; }
__device__ __forceinline__ uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
__device__ __forceinline__ uint64_t mk64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
template <int K>
__device__ __forceinline__ uint64_t rotl64c(uint64_t x) {
  if constexpr (K < 32)
    return mk64(__builtin_amdgcn_alignbit(lo32(x), hi32(x), 32 - K), __builtin_amdgcn_alignbit(hi32(x), lo32(x), 32 - K));
  else
    return mk64(__builtin_amdgcn_alignbit(hi32(x), lo32(x), 64 - K), __builtin_amdgcn_alignbit(lo32(x), hi32(x), 64 - K));
}
__device__ __forceinline__ uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
  return mk64(__builtin_amdgcn_bitop3_b32(lo32(a), lo32(b), lo32(c), 0x96),
              __builtin_amdgcn_bitop3_b32(hi32(a), hi32(b), hi32(c), 0x96));
}
__device__ __forceinline__ void step(uint64_t& s0, uint64_t& s1, uint64_t& s2, uint64_t& s3) {
  const uint64_t t = s1 << 17;
  const uint64_t n1 = xor3_64(s1, s2, s0);
  const uint64_t n0 = xor3_64(s0, s3, s1);
  const uint64_t n2 = xor3_64(s2, s0, t);
  s3 = rotl64c<45>(s3 ^ s1);
  s0 = n0;
  s1 = n1;
  s2 = n2;
}
__device__ __forceinline__ uint32_t next_hi(uint64_t& s0, uint64_t& s1, uint64_t& s2, uint64_t& s3) {
  const uint64_t a = s0 + s3;
  const uint32_t r = __builtin_amdgcn_alignbit(hi32(a), lo32(a), 9) + hi32(s0);
  step(s0, s1, s2, s3);
  return r;
}
__device__ __forceinline__ uint32_t screened(uint64_t& s0, uint64_t& s1, uint64_t& s2, uint64_t& s3, int n,
                                             uint32_t Th) {
  uint32_t sent = 0;
  for (int j = 0; j + 8 <= n; j += 8) {
    const uint32_t h0 = next_hi(s0, s1, s2, s3), h1 = next_hi(s0, s1, s2, s3), h2 = next_hi(s0, s1, s2, s3),
                   h3 = next_hi(s0, s1, s2, s3), h4 = next_hi(s0, s1, s2, s3), h5 = next_hi(s0, s1, s2, s3),
                   h6 = next_hi(s0, s1, s2, s3), h7 = next_hi(s0, s1, s2, s3);
    const uint32_t m = max(max(max(h0, h1), max(h2, h3)), max(max(h4, h5), max(h6, h7)));
    sent += (m + 1 >= Th) ? 7u : 8u;
  }
  return sent;
}

__global__ __launch_bounds__(512) void k(uint64_t* res, int n, uint32_t busy, uint32_t Th, int bg,
                                         uint64_t* clk, uint32_t* word, const uint32_t* chain) {
  __shared__ volatile uint32_t done;
  __shared__ uint32_t scratch[1024];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x == 0) done = 0;
  __syncthreads();
  uint64_t s0 = threadIdx.x * 0x9E3779B97F4A7C15ull + 1, s1 = 2 + blockIdx.x, s2 = 3, s3 = 4;
  uint64_t acc = 0;
  if (wv == 0) {
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    if (lane < busy) acc = screened(s0, s1, s2, s3, n, Th);
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
      done = 1;
      clk[blockIdx.x] = c1 - c0;
    }
  } else {
    uint32_t p = (blockIdx.x * 8 + wv) * 64 + lane;
    int it = 0;
    while (!done && it < (1 << 20)) {
      it++;
      if (bg == 1) {
        acc += __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_sleep(16);
      } else if (bg == 2) {
        acc += screened(s0, s1, s2, s3, 64, Th);
      } else if (bg == 3) {
        for (int q = 0; q < 8; q++) p = __hip_atomic_load(&chain[p & ((1u << 22) - 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc += p;
      } else if (bg == 4) {
        for (int q = 0; q < 16; q++) {
          atomicAdd(&scratch[(p + q * 37) & 1023], 1u);
          acc += scratch[(p * 3 + q) & 1023];
        }
      } else if (bg == 5) {
        for (int q = 0; q < 16; q++) acc += __builtin_amdgcn_readfirstlane((int)word[(q + it) & 255]);
      } else {
        break;
      }
    }
  }
  res[blockIdx.x * 512 + threadIdx.x] = acc ^ s0;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2048;
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint64_t *res, *clk;
  uint32_t *word, *chain;
  hipMalloc(&res, (size_t)cus * 512 * 8);
  hipMalloc(&clk, cus * 8);
  hipMalloc(&word, 4096);
  hipMemset(word, 0, 4096);
  hipMalloc(&chain, (size_t)4 << 22);
  {
    uint32_t* h = (uint32_t*)malloc((size_t)4 << 22);
    uint32_t x = 12345;
    for (uint32_t i = 0; i < (1u << 22); i++) {
      x = x * 1664525u + 1013904223u;
      h[i] = x;
    }
    hipMemcpy(chain, h, (size_t)4 << 22, hipMemcpyHostToDevice);
    free(h);
  }
  const uint32_t Th = 0xFFFFF000u;  // (loss ~ 2^-20: the screen never fires)
  const char* names[] = {"idle", "poll (device-scope load + s_sleep 16)", "VALU (the same loop, 64 lanes)",
                         "dependent global loads", "LDS atomics + reads", "scalar loads + readfirstlane"};
  std::vector<uint64_t> hc(cus);
  for (uint32_t busy : {3u, 64u})
    for (int bg = 0; bg < 6; bg++) {
      double best = 1e30, med = 0;
      for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k, dim3(cus), dim3(512), 0, 0, res, n, busy, Th, bg, clk, word, chain);
        hipDeviceSynchronize();
        hipMemcpy(hc.data(), clk, cus * 8, hipMemcpyDeviceToHost);
        std::vector<uint64_t> v(hc);
        std::sort(v.begin(), v.end());
        med = (double)v[cus / 2] / n;
        best = std::min(best, med);
      }
      printf("busy lanes %2u, other 7 waves: %-40s %.1f cycles per draw (median CU)\n", busy, names[bg], best);
    }
  return 0;
}
