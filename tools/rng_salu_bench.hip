// Cycles per xoshiro256++ draw + loss test on gfx950, VALU (the engine's form, the state in
// the busy lane's VGPRs) against SALU (the busy lane's state read into SGPRs and stepped by
// the scalar unit, which issues beside other waves' VALU work), alone and with other waves
// on the same CU doing VALU work (diagnostic tool, not the product).
// Build: hipcc --offload-arch=gfx950 -O3 tools/rng_salu_bench.hip -o tools/rng_salu_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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
__device__ __forceinline__ uint64_t vnext(uint64_t& s0, uint64_t& s1, uint64_t& s2, uint64_t& s3) {
  const uint64_t r = rotc<23>(s0 + s3) + s0, t = s1 << 17;
  const uint64_t n1 = x3(s1, s2, s0), n0 = x3(s0, s3, s1), n2 = x3(s2, s0, t);
  s3 = rotc<45>(s3 ^ s1); s0 = n0; s1 = n1; s2 = n2;
  return r;
}
// scalar form (plain 64-bit C: the operands are wave-uniform, so it compiles to s_*_b64)
__device__ __forceinline__ uint64_t snext(uint64_t& s0, uint64_t& s1, uint64_t& s2, uint64_t& s3) {
  const uint64_t a = s0 + s3;
  const uint64_t r = ((a << 23) | (a >> 41)) + s0, t = s1 << 17;
  s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t; s3 = (s3 << 45) | (s3 >> 19);
  return r;
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int lane) {
  return mk((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane), (uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), lane));
}

// mode 0: VALU draws in lane 0; mode 1: SALU draws of lane 0's stream. Block 0 measures; the
// other blocks (noise) run VALU-heavy loops for `noise` iterations.
__global__ void k(uint64_t* out, int n, int mode, int noise, uint64_t Tx, uint64_t* clk) {
  uint64_t s0 = threadIdx.x + 1 + blockIdx.x, s1 = 2, s2 = 3, s3 = 4;
  if (blockIdx.x != 0) {  // noise: dependent VALU chains in every lane
    uint64_t acc = 0;
    for (int i = 0; i < noise; i++) acc += vnext(s0, s1, s2, s3);
    out[blockIdx.x * 64 + threadIdx.x] = acc;
    return;
  }
  __builtin_amdgcn_s_sleep(100);  // let the noise waves start
  uint32_t sent = 0, lost = 0;
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  if (mode == 0) {
    if (threadIdx.x == 0) {
      for (int j = 0; j + 8 <= n; j += 8) {
        const uint64_t a = vnext(s0, s1, s2, s3), b = vnext(s0, s1, s2, s3), c = vnext(s0, s1, s2, s3), d = vnext(s0, s1, s2, s3);
        const uint64_t e = vnext(s0, s1, s2, s3), f = vnext(s0, s1, s2, s3), g = vnext(s0, s1, s2, s3), h = vnext(s0, s1, s2, s3);
        if ((a >= Tx) | (b >= Tx) | (c >= Tx) | (d >= Tx) | (e >= Tx) | (f >= Tx) | (g >= Tx) | (h >= Tx)) lost++;
        else sent += 8;
      }
    }
  } else {
    uint64_t a0 = rl64(s0, 0), a1 = rl64(s1, 0), a2 = rl64(s2, 0), a3 = rl64(s3, 0);
    uint32_t ss = 0, sl = 0;
    for (int j = 0; j + 8 <= n; j += 8) {
      bool any = false;
#pragma unroll
      for (int u = 0; u < 8; u++) any |= snext(a0, a1, a2, a3) >= Tx;
      if (any) sl++;
      else ss += 8;
    }
    if (threadIdx.x == 0) {
      s0 = a0; s1 = a1; s2 = a2; s3 = a3;
      sent = ss;
      lost = sl;
    }
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = s0 ^ s1 ^ s2 ^ s3 ^ sent ^ ((uint64_t)lost << 32);
  if (threadIdx.x == 0) clk[0] = c1 - c0;
}

int main(int argc, char** argv) {
  uint64_t *out, *clk;
  hipMalloc(&out, 64 * 8192 * 8);
  hipMalloc(&clk, 8);
  const int n = argc > 1 ? atoi(argv[1]) : 4096;  // draws per launch (88: one server's round)
  for (int mode = 0; mode < 2; mode++)
    for (int blocks : {1, 2048, 4096}) {
      for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, out, n, mode, 3 * n, 0xFF00000000000000ull, clk);
        hipDeviceSynchronize();
      }
      uint64_t c;
      hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
      printf("%s draws, %4d workgroups (%.0f per CU): %.1f cycles/draw\n", mode ? "SALU" : "VALU", blocks,
             blocks / 256.0, (double)c / n);
    }
  return 0;
}
