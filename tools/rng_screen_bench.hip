// Cycles per xoshiro256++ draw + loss test on gfx950 (diagnostic tool, not the product):
// the product's form (64-bit output, one 64-bit compare per draw, eight per test) against a
// screened form: per draw only the output's high word without the low word's carry, eight
// high words folded with v_max3, and an exact redo of the eight draws from a saved state
// when the screen fires (probability ~ 8 x loss).
// Build: hipcc --offload-arch=gfx950 -O3 tools/rng_screen_bench.hip -o tools/rng_screen_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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
__device__ __forceinline__ uint64_t out(uint64_t s0, uint64_t s3) { return rotl64c<23>(s0 + s3) + s0; }
__device__ __forceinline__ uint64_t next(uint64_t& s0, uint64_t& s1, uint64_t& s2, uint64_t& s3) {
  const uint64_t r = out(s0, s3);
  step(s0, s1, s2, s3);
  return r;
}
// the output's high word without the carry out of the low word: the true high word is this
// or this + 1
__device__ __forceinline__ uint32_t out_hi_nc(uint64_t s0, uint64_t s3) {
  const uint64_t a = s0 + s3;
  return __builtin_amdgcn_alignbit(hi32(a), lo32(a), 9) + hi32(s0);
}
__device__ __forceinline__ uint32_t next_hi(uint64_t& s0, uint64_t& s1, uint64_t& s2, uint64_t& s3) {
  const uint32_t r = out_hi_nc(s0, s3);
  step(s0, s1, s2, s3);
  return r;
}
__device__ __forceinline__ uint32_t max3(uint32_t a, uint32_t b, uint32_t c) { return max(max(a, b), c); }  // v_max3_u32

template <int V>
__global__ void k(uint64_t* res, int n, uint32_t busy, uint64_t Tx, uint64_t* clk) {
  uint64_t s0 = threadIdx.x * 0x9E3779B97F4A7C15ull + 1, s1 = 2 + blockIdx.x, s2 = 3, s3 = 4;
  uint32_t sent = 0, lost = 0, slow = 0;
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x < busy) {
    if constexpr (V == 0) {
      for (int j = 0; j + 8 <= n; j += 8) {
        const uint64_t x0 = next(s0, s1, s2, s3), x1 = next(s0, s1, s2, s3), x2 = next(s0, s1, s2, s3),
                       x3 = next(s0, s1, s2, s3), x4 = next(s0, s1, s2, s3), x5 = next(s0, s1, s2, s3),
                       x6 = next(s0, s1, s2, s3), x7 = next(s0, s1, s2, s3);
        if ((x0 >= Tx) | (x1 >= Tx) | (x2 >= Tx) | (x3 >= Tx) | (x4 >= Tx) | (x5 >= Tx) | (x6 >= Tx) | (x7 >= Tx)) {
          const uint32_t L = (x0 >= Tx) + (x1 >= Tx) + (x2 >= Tx) + (x3 >= Tx) + (x4 >= Tx) + (x5 >= Tx) +
                             (x6 >= Tx) + (x7 >= Tx);
          lost += L;
          sent += 8 - L;
          slow++;
        } else {
          sent += 8;
        }
      }
    } else {
      // screen: every draw with true high word < Th is kept; true high <= nc + 1
      const uint32_t Th = hi32(Tx);
      for (int j = 0; j + 8 <= n; j += 8) {
        const uint64_t a0 = s0, a1 = s1, a2 = s2, a3 = s3;
        const uint32_t h0 = next_hi(s0, s1, s2, s3), h1 = next_hi(s0, s1, s2, s3), h2 = next_hi(s0, s1, s2, s3),
                       h3 = next_hi(s0, s1, s2, s3), h4 = next_hi(s0, s1, s2, s3), h5 = next_hi(s0, s1, s2, s3),
                       h6 = next_hi(s0, s1, s2, s3), h7 = next_hi(s0, s1, s2, s3);
        const uint32_t m = max(max3(h0, h1, h2), max3(max3(h3, h4, h5), h6, h7));
        if (m + 1 >= Th || m == 0xFFFFFFFFu) {  // (m + 1 wraps at the top)
          uint64_t b0 = a0, b1 = a1, b2 = a2, b3 = a3;
          uint32_t L = 0;
          for (int q = 0; q < 8; q++) L += next(b0, b1, b2, b3) >= Tx;
          lost += L;
          sent += 8 - L;
          slow++;
        } else {
          sent += 8;
        }
      }
    }
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x < busy)
    res[(blockIdx.x * 64 + threadIdx.x) * 4] = s0 ^ s1 ^ s2 ^ s3,
    res[(blockIdx.x * 64 + threadIdx.x) * 4 + 1] = sent, res[(blockIdx.x * 64 + threadIdx.x) * 4 + 2] = lost,
    res[(blockIdx.x * 64 + threadIdx.x) * 4 + 3] = slow;
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = c1 - c0;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  uint64_t *res, *clk;
  hipMalloc(&res, 64 * 1024 * 32);
  hipMalloc(&clk, 8);
  uint64_t h0[4 * 64], h1[4 * 64];
  // loss 1 %: T = 0.99 * 2^53, Tx = T << 11; loss 0.01 %
  for (double loss : {0.01, 0.0001}) {
    const uint64_t Tx = (uint64_t)((1.0 - loss) * 9007199254740992.0) << 11;
    for (uint32_t busy : {1u, 64u})
      for (int waves : {1, 1024}) {
        double cyc[2];
        for (int V = 0; V < 2; V++) {
          for (int rep = 0; rep < 2; rep++) {
            if (V == 0) hipLaunchKernelGGL(k<0>, dim3(waves), dim3(64), 0, 0, res, n, busy, Tx, clk);
            else hipLaunchKernelGGL(k<1>, dim3(waves), dim3(64), 0, 0, res, n, busy, Tx, clk);
            hipDeviceSynchronize();
          }
          uint64_t c;
          hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
          cyc[V] = (double)c / n;
          hipMemcpy(V ? h1 : h0, res, sizeof(h0), hipMemcpyDeviceToHost);
        }
        bool same = true;
        for (uint32_t i = 0; i < busy; i++)
          for (int w = 0; w < 3; w++) same &= h0[i * 4 + w] == h1[i * 4 + w];
        printf("loss=%.4f busy=%2u waves=%4d: product %.1f  screened %.1f cycles/draw  (slow batches %lu / %d)  same=%d\n",
               loss, busy, waves, cyc[0], cyc[1], (unsigned long)h1[3], n / 8, (int)same);
      }
  }
  return 0;
}
