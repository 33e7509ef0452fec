// Cycles per xoshiro256++ draw + loss test on gfx950 (diagnostic tool, not the product):
// the compiler's 64-bit form against the alignbit / bitop3 form, one busy lane and 64.
// Build: hipcc --offload-arch=gfx950 -O3 tools/rng_bench.hip -o tools/rng_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
__device__ __forceinline__ uint64_t mk(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
template <int K>
__device__ __forceinline__ uint64_t rotc(uint64_t x) {
  const uint32_t l = (uint32_t)x, h = (uint32_t)(x >> 32);
  if constexpr (K < 32) return mk(__builtin_amdgcn_alignbit(l, h, 32 - K), __builtin_amdgcn_alignbit(h, l, 32 - K));
  else return mk(__builtin_amdgcn_alignbit(h, l, 64 - K), __builtin_amdgcn_alignbit(l, h, 64 - K));
}
__device__ __forceinline__ uint64_t x3(uint64_t a, uint64_t b, uint64_t c) {
  return mk(__builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x96),
            __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x96));
}
template <int V>
__device__ __forceinline__ uint64_t next(uint64_t& s0, uint64_t& s1, uint64_t& s2, uint64_t& s3) {
  if constexpr (V == 0) {
    const uint64_t r = rotl(s0 + s3, 23) + s0, t = s1 << 17;
    s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t; s3 = rotl(s3, 45);
    return r;
  } else {
    const uint64_t r = rotc<23>(s0 + s3) + s0, t = s1 << 17;
    const uint64_t n1 = x3(s1, s2, s0), n0 = x3(s0, s3, s1), n2 = x3(s2, s0, t);
    s3 = rotc<45>(s3 ^ s1); s0 = n0; s1 = n1; s2 = n2;
    return r;
  }
}
// all-32-bit form: state as 8 words, 64-bit adds as add / add-with-carry
struct S8 { uint32_t l0, h0, l1, h1, l2, h2, l3, h3; };
__device__ __forceinline__ uint32_t bx3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ void add64(uint32_t al, uint32_t ah, uint32_t bl, uint32_t bh, uint32_t& rl, uint32_t& rh) {
  unsigned c;
  rl = __builtin_addc(al, bl, 0u, &c);
  rh = ah + bh + c;
}
__device__ __forceinline__ void next32(S8& s, uint32_t& xl, uint32_t& xh) {
  uint32_t al, ah;
  add64(s.l0, s.h0, s.l3, s.h3, al, ah);
  const uint32_t rl = __builtin_amdgcn_alignbit(al, ah, 9), rh = __builtin_amdgcn_alignbit(ah, al, 9);
  add64(rl, rh, s.l0, s.h0, xl, xh);
  const uint32_t tl = s.l1 << 17, th = __builtin_amdgcn_alignbit(s.h1, s.l1, 15);
  const uint32_t n1l = bx3(s.l1, s.l2, s.l0), n1h = bx3(s.h1, s.h2, s.h0);
  const uint32_t n0l = bx3(s.l0, s.l3, s.l1), n0h = bx3(s.h0, s.h3, s.h1);
  const uint32_t n2l = bx3(s.l2, s.l0, tl), n2h = bx3(s.h2, s.h0, th);
  const uint32_t ul = s.l3 ^ s.l1, uh = s.h3 ^ s.h1;
  s.l3 = __builtin_amdgcn_alignbit(uh, ul, 19);
  s.h3 = __builtin_amdgcn_alignbit(ul, uh, 19);
  s.l0 = n0l; s.h0 = n0h; s.l1 = n1l; s.h1 = n1h; s.l2 = n2l; s.h2 = n2h;
}
__device__ __forceinline__ bool ge64(uint32_t xl, uint32_t xh, uint64_t T) {
  return xh > (uint32_t)(T >> 32) || (xh == (uint32_t)(T >> 32) && xl >= (uint32_t)T);
}
__global__ void k2(uint64_t* out, int n, uint32_t busy, uint64_t Tx, uint64_t* clk) {
  S8 s{threadIdx.x + 1, 0, 2, 0, 3, 0, 4, 0};
  uint32_t sent = 0, lost = 0;
  const uint32_t Th = (uint32_t)(Tx >> 32);
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x < busy) {
    int j = 0;
    for (; j + 4 <= n; j += 4) {
      uint32_t al, ah, bl, bh, cl, ch, dl, dh;
      next32(s, al, ah); next32(s, bl, bh); next32(s, cl, ch); next32(s, dl, dh);
      const uint32_t m = max(max(ah, bh), max(ch, dh));
      if (m >= Th) {
        const int L = ge64(al, ah, Tx) + ge64(bl, bh, Tx) + ge64(cl, ch, Tx) + ge64(dl, dh, Tx);
        lost += L;
        sent += 4 - L;
      } else {
        sent += 4;
      }
    }
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = s.l0 ^ s.h1 ^ s.l2 ^ s.h3 ^ sent ^ ((uint64_t)lost << 32);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = c1 - c0;
}

template <int V>
__global__ void k(uint64_t* out, int n, uint32_t busy, uint64_t Tx, uint64_t* clk) {
  uint64_t s0 = threadIdx.x + 1, s1 = 2, s2 = 3, s3 = 4;
  uint32_t sent = 0, lost = 0;
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x < busy) {
    int j = 0;
    for (; j + 4 <= n; j += 4) {
      const uint64_t a = next<V>(s0, s1, s2, s3), b = next<V>(s0, s1, s2, s3), c = next<V>(s0, s1, s2, s3),
                     d = next<V>(s0, s1, s2, s3);
      if ((a >= Tx) | (b >= Tx) | (c >= Tx) | (d >= Tx)) {
        lost += (a >= Tx) + (b >= Tx) + (c >= Tx) + (d >= Tx);
        sent += (a < Tx) + (b < Tx) + (c < Tx) + (d < Tx);
      } else {
        sent += 4;
      }
    }
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3 ^ sent ^ ((uint64_t)lost << 32);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = c1 - c0;
}

int main() {
  uint64_t *out, *clk;
  hipMalloc(&out, 64 * 1024 * 8);
  hipMalloc(&clk, 8);
  const int n = 4096;
  for (int V = 0; V < 3; V++)
    for (uint32_t busy : {1u, 64u})
      for (int waves : {1, 1024}) {
        for (int rep = 0; rep < 2; rep++) {
          if (V == 0) hipLaunchKernelGGL(k<0>, dim3(waves), dim3(64), 0, 0, out, n, busy, 0xFF00000000000000ull, clk);
          else if (V == 1) hipLaunchKernelGGL(k<1>, dim3(waves), dim3(64), 0, 0, out, n, busy, 0xFF00000000000000ull, clk);
          else hipLaunchKernelGGL(k2, dim3(waves), dim3(64), 0, 0, out, n, busy, 0xFF00000000000000ull, clk);
          hipDeviceSynchronize();
        }
        uint64_t c;
        hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
        printf("variant %s busy=%2u waves=%4d: %.1f cycles/draw\n", V == 2 ? "32-bit words" : V ? "alignbit+bitop3" : "plain", busy, waves,
               (double)c / n);
      }
  return 0;
}
