// routes.hip — the routing table (NetworkGraph::compute_shortest_paths,
// network/graph/mod.rs:181-226, and get_direct_paths, :228-250) on gfx950.
//
// Shadow runs one petgraph Dijkstra per used source with the lexicographic cost
// (latency u64, then loss f32) and the non-associative f32 fold
//   loss' = 1f - (1f - loss) * (1f - edge_loss)            (graph/mod.rs:316-325).
// Because the fold is isotone and latencies are strictly positive, Dijkstra's result is
// the lexicographic minimum over all paths; it is computed here in two exact phases:
//   1. latency: blocked min-plus Floyd-Warshall over all V graph nodes, 64x64 u64 tiles
//      staged through LDS (VALU/LDS-bound, no MFMA: min-plus is not multiply-accumulate);
//   2. loss: per used source, a Bellman-Ford sweep over the *tight* arcs
//      (d[s][u] + lat(u,v) == d[s][v]) to the fixed point
//      loss[v] = min over tight u->v of fold(loss[u], p(u,v)), loss[s] = 0, with every f32
//      operation rounded individually (__fsub_rn/__fmul_rn; Rust never contracts).
//      A Floyd-Warshall over (lat, loss) pairs would combine sub-path aggregates and is
//      NOT bit-exact (fold(fold(fold(0,.1),.2),.3) != fold(fold(0,.1),fold(.2,.3))).
// Then each used node's (n,n) entry is replaced by its single self-loop edge
// (graph/mod.rs:209-215).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <unordered_map>

#include "sgn_internal.h"

namespace sgn {

constexpr int FW_T = 64;
constexpr uint64_t FW_INF = 1ULL << 62;  // sums of two stay below 2^63

__global__ void fw_init(uint64_t* D, uint32_t Vp) {
  const uint64_t n = (uint64_t)Vp * Vp;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = i / Vp, c = i % Vp;
    D[i] = r == c ? 0 : FW_INF;
  }
}

__global__ void fw_edges(uint64_t* D, uint32_t Vp, const uint32_t* eu, const uint32_t* ev,
                         const uint64_t* el, uint32_t E, int directed) {
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < E; k += gridDim.x * blockDim.x) {
    const uint32_t u = eu[k], v = ev[k];
    if (u == v) continue;  // the zero-length path always beats a self-loop
    atomicMin((unsigned long long*)&D[(uint64_t)u * Vp + v], (unsigned long long)el[k]);
    if (!directed)
      atomicMin((unsigned long long*)&D[(uint64_t)v * Vp + u], (unsigned long long)el[k]);
  }
}

// thread (ty, tx) of 256 owns rows ty + 16a and columns tx + 16b, a, b in 0..3
#define FW_LOAD_TILE(dst, bi, bj)                                                  \
  for (int a = 0; a < 4; a++)                                                      \
    for (int b = 0; b < 4; b++)                                                    \
      dst[ty + 16 * a][tx + 16 * b] =                                              \
          D[(uint64_t)((bi) * FW_T + ty + 16 * a) * Vp + (bj) * FW_T + tx + 16 * b];

// The dependent tiles (pivot, panels) run as 1024-thread workgroups, 2x2 entries per thread
// in registers (thread (ty, tx) of 32x32 owns rows ty + 32a, columns tx + 32b): at step k the
// owners of the tile's row k / column k publish them to a double-buffered LDS row / column
// (one barrier per step) and every thread updates its entries from the published values.
// Row k and column k do not change at step k (the pivot's diagonal is 0), so the published
// values are exactly those the in-place algorithm would read. 16 waves per workgroup keep
// the SIMDs busy through each step's dependent chain.
__global__ __launch_bounds__(1024) void fw_phase1(uint64_t* D, uint32_t Vp, int kb) {
  __shared__ uint64_t rowb[2][FW_T], colb[2][FW_T];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  uint64_t c[2][2];
  for (int a = 0; a < 2; a++)
    for (int b = 0; b < 2; b++)
      c[a][b] = D[(uint64_t)(kb * FW_T + ty + 32 * a) * Vp + kb * FW_T + tx + 32 * b];
  for (int k = 0; k < FW_T; k++) {
    const int h = k & 1;
    if (ty == (k & 31))
#pragma unroll
      for (int b = 0; b < 2; b++) rowb[h][tx + 32 * b] = c[k >> 5][b];
    if (tx == (k & 31))
#pragma unroll
      for (int a = 0; a < 2; a++) colb[h][ty + 32 * a] = c[a][k >> 5];
    __syncthreads();
    const uint64_t u0 = rowb[h][tx], u1 = rowb[h][tx + 32];
    const uint64_t l0 = colb[h][ty], l1 = colb[h][ty + 32];
    c[0][0] = min(c[0][0], l0 + u0);
    c[0][1] = min(c[0][1], l0 + u1);
    c[1][0] = min(c[1][0], l1 + u0);
    c[1][1] = min(c[1][1], l1 + u1);
  }
  for (int a = 0; a < 2; a++)
    for (int b = 0; b < 2; b++)
      D[(uint64_t)(kb * FW_T + ty + 32 * a) * Vp + kb * FW_T + tx + 32 * b] = c[a][b];
}

// row panel (kb, j) and column panel (i, kb) against the finished pivot tile
// ROW: C[i][j] = min(C, P[i][k] + C[k][j]) publishes its row k each step;
// column: C[i][j] = min(C, C[i][k] + P[k][j]) publishes its column k
template <bool ROW>
__device__ __forceinline__ void fw_panel(uint64_t (&c)[2][2], uint64_t (*P)[FW_T + 1],
                                         uint64_t (*pub)[FW_T], int tx, int ty) {
  for (int k = 0; k < FW_T; k++) {
    const int h = k & 1;
    if (ROW) {
      if (ty == (k & 31))
#pragma unroll
        for (int b = 0; b < 2; b++) pub[h][tx + 32 * b] = c[k >> 5][b];
    } else if (tx == (k & 31)) {
#pragma unroll
      for (int a = 0; a < 2; a++) pub[h][ty + 32 * a] = c[a][k >> 5];
    }
    __syncthreads();
    const uint64_t u0 = ROW ? pub[h][tx] : P[k][tx], u1 = ROW ? pub[h][tx + 32] : P[k][tx + 32];
    const uint64_t l0 = ROW ? P[ty][k] : pub[h][ty], l1 = ROW ? P[ty + 32][k] : pub[h][ty + 32];
    c[0][0] = min(c[0][0], l0 + u0);
    c[0][1] = min(c[0][1], l0 + u1);
    c[1][0] = min(c[1][0], l1 + u0);
    c[1][1] = min(c[1][1], l1 + u1);
  }
}

__global__ __launch_bounds__(1024) void fw_phase2(uint64_t* D, uint32_t Vp, int kb, int nb) {
  __shared__ uint64_t P[FW_T][FW_T + 1];
  __shared__ uint64_t pub[2][FW_T];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  int idx = blockIdx.x;
  const bool row = idx < nb - 1;
  if (!row) idx -= nb - 1;
  const int other = idx < kb ? idx : idx + 1;
  const int bi = row ? kb : other, bj = row ? other : kb;
  for (int a = 0; a < 2; a++)
    for (int b = 0; b < 2; b++)
      P[ty + 32 * a][tx + 32 * b] = D[(uint64_t)(kb * FW_T + ty + 32 * a) * Vp + kb * FW_T + tx + 32 * b];
  uint64_t c[2][2];
  for (int a = 0; a < 2; a++)
    for (int b = 0; b < 2; b++)
      c[a][b] = D[(uint64_t)(bi * FW_T + ty + 32 * a) * Vp + bj * FW_T + tx + 32 * b];
  __syncthreads();
  if (row)
    fw_panel<true>(c, P, pub, tx, ty);
  else
    fw_panel<false>(c, P, pub, tx, ty);
  for (int a = 0; a < 2; a++)
    for (int b = 0; b < 2; b++)
      D[(uint64_t)(bi * FW_T + ty + 32 * a) * Vp + bj * FW_T + tx + 32 * b] = c[a][b];
}

// all remaining tiles: C = min(C, A (bi,kb) (+) B (kb,bj)), k order irrelevant
__global__ __launch_bounds__(256) void fw_phase3(uint64_t* D, uint32_t Vp, int kb, int nb) {
  __shared__ uint64_t A[FW_T][FW_T + 1];
  __shared__ uint64_t B[FW_T][FW_T];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m = nb - 1;
  const int lin = blockIdx.x;
  const int i0 = lin / m, j0 = lin % m;
  const int bi = i0 < kb ? i0 : i0 + 1;
  const int bj = j0 < kb ? j0 : j0 + 1;
  FW_LOAD_TILE(A, bi, kb);
  for (int a = 0; a < 4; a++)
    for (int b = 0; b < 4; b++)
      B[ty + 16 * a][tx + 16 * b] =
          D[(uint64_t)(kb * FW_T + ty + 16 * a) * Vp + bj * FW_T + tx + 16 * b];
  uint64_t c[4][4];
  for (int a = 0; a < 4; a++)
    for (int b = 0; b < 4; b++)
      c[a][b] = D[(uint64_t)(bi * FW_T + ty + 16 * a) * Vp + bj * FW_T + tx + 16 * b];
  __syncthreads();
#pragma unroll 4
  for (int k = 0; k < FW_T; k++) {
    uint64_t bk[4];
#pragma unroll
    for (int b = 0; b < 4; b++) bk[b] = B[k][tx + 16 * b];
#pragma unroll
    for (int a = 0; a < 4; a++) {
      const uint64_t aik = A[ty + 16 * a][k];
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const uint64_t s = aik + bk[b];
        c[a][b] = s < c[a][b] ? s : c[a][b];
      }
    }
  }
  for (int a = 0; a < 4; a++)
    for (int b = 0; b < 4; b++)
      D[(uint64_t)(bi * FW_T + ty + 16 * a) * Vp + bj * FW_T + tx + 16 * b] = c[a][b];
}

// ---- latency phase, fast form: min-plus squaring on saturating u32 ----
// D <- min(D, D (+) D) until nothing changes: after k squarings D holds the shortest paths of
// up to 2^k hops, so at most ceil(log2 V) + 1 passes, each an independent tiled min-plus
// product (no dependent pivot chain: the whole chip works on every pass). Entries are u32
// with a saturating add (v_add_u32 clamp): every finite entry is the length of a real path
// and a true shortest path never saturates (its sub-path sums are <= its length), so the
// result is exact whenever every used pair ends below 2^32 - 1; otherwise (a path of 4.29 s
// or more, or a disconnected pair) the build redoes the phase with the u64 Floyd-Warshall
// above. In place: a tile may read entries another workgroup already lowered this pass,
// which are still real path lengths, so the fixed point is the same.
constexpr uint32_t SQ_INF = 0xFFFFFFFFu;
constexpr uint32_t kFx = 0xC0000000u;  // -2^30: the fused sweep's excluded pairs (loss_sweep_dense)
constexpr int SQ_T = 64, SQ_K = 32;

__global__ void sq_init(uint32_t* D, uint32_t Vp) {
  const uint64_t n = (uint64_t)Vp * Vp;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    D[i] = (i / Vp == i % Vp) ? 0u : SQ_INF;
}

__global__ void sq_edges(uint32_t* D, uint32_t Vp, const uint32_t* eu, const uint32_t* ev, const uint64_t* el,
                         uint32_t E, int directed) {
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < E; k += gridDim.x * blockDim.x) {
    const uint32_t u = eu[k], v = ev[k];
    if (u == v) continue;  // the zero-length path always beats a self-loop
    const uint32_t l = (uint32_t)el[k];  // < 2^32 - 1 (checked on the host)
    atomicMin(&D[(uint64_t)u * Vp + v], l);
    if (!directed) atomicMin(&D[(uint64_t)v * Vp + u], l);
  }
}

// One pass, 64 x 64 output tile per workgroup of 256 threads, 4 x 4 consecutive entries per
// thread; K in steps of 32 through LDS (A transposed so both operands are 16-byte reads).
// flag[it] = 1 if anything changed; the pass returns at once when pass it - 1 changed nothing.
// rt0: the first row tile of this launch (a shard's block of rows, gridDim.y tiles)
__global__ __launch_bounds__(256) void sq_pass(uint32_t* D, uint32_t Vp, uint32_t* flag, int it, uint32_t rt0) {
  if (it > 0 && __hip_atomic_load(&flag[it - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  __shared__ __attribute__((aligned(16))) uint32_t As[SQ_K][SQ_T + 4];
  __shared__ __attribute__((aligned(16))) uint32_t Bs[SQ_K][SQ_T + 4];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const uint64_t r0 = (uint64_t)(blockIdx.y + rt0) * SQ_T, c0 = (uint64_t)blockIdx.x * SQ_T;
  uint32_t acc[4][4], orig[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint4 v = *(const uint4*)&D[(r0 + ty * 4 + i) * Vp + c0 + tx * 4];
    acc[i][0] = orig[i][0] = v.x;
    acc[i][1] = orig[i][1] = v.y;
    acc[i][2] = orig[i][2] = v.z;
    acc[i][3] = orig[i][3] = v.w;
  }
  for (uint32_t k0 = 0; k0 < Vp; k0 += SQ_K) {
    // A = D[r0 .. +64][k0 .. +32] transposed into As[k][m]; B = D[k0 .. +32][c0 .. +64]
    for (int e = threadIdx.x; e < SQ_T * SQ_K / 4; e += 256) {
      const int m = e >> 3, kq = (e & 7) * 4;
      const uint4 a = *(const uint4*)&D[(r0 + m) * Vp + k0 + kq];
      As[kq][m] = a.x;
      As[kq + 1][m] = a.y;
      As[kq + 2][m] = a.z;
      As[kq + 3][m] = a.w;
      const int kb = e >> 4, nq = (e & 15) * 4;
      *(uint4*)&Bs[kb][nq] = *(const uint4*)&D[(k0 + kb) * Vp + c0 + nq];
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < SQ_K; k++) {
      const uint4 a = *(const uint4*)&As[k][ty * 4];
      const uint4 b = *(const uint4*)&Bs[k][tx * 4];
      const uint32_t av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t s2 = __builtin_elementwise_add_sat(av[i], bv[j]);
          acc[i][j] = s2 < acc[i][j] ? s2 : acc[i][j];
        }
    }
    __syncthreads();
  }
  bool ch = false;
#pragma unroll
  for (int i = 0; i < 4; i++) {
#pragma unroll
    for (int j = 0; j < 4; j++) ch |= acc[i][j] != orig[i][j];
    *(uint4*)&D[(r0 + ty * 4 + i) * Vp + c0 + tx * 4] = make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
  }
  if (__ballot(ch) && (threadIdx.x & 63) == 0) flag[it] = 1;
}

// sq_init + sq_edges for a graph whose arcs are in tail order (CSR): one workgroup per row u
// builds d[u][.] in LDS (the diagonal 0, each arc's latency by LDS atomic min: parallel
// arcs keep the shortest) and writes it whole — no global atomics, one coalesced row write.
// NL, EI (the fused form of the loss sweep: no parallel arcs): the same row negated, with kFx on
// the diagonal and where there is no arc, and each arc's index (dense_arcs' matrices). NDT
// (undirected graphs: the matrix is symmetric, so row u is column u): the sweep's transposed
// used-source entries of row u, NDT[u][j] = -d[usrc[j]][u], as ndt_build<true> makes them.
__global__ __launch_bounds__(256) void sq_rows(uint32_t* D, uint32_t Vp, uint32_t V, const uint32_t* rowptr,
                                               const uint32_t* auv, const uint64_t* al, uint32_t* NL, uint32_t* EI,
                                               uint32_t* NDT, const uint32_t* usrc, uint32_t ns, uint32_t Up,
                                               uint32_t* z0, uint32_t n0, uint32_t* z1, uint32_t n1) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* row = (uint32_t*)smem;
  const uint32_t u = blockIdx.x;
  // (block 0 clears the squaring's flag words and, in the fused form, the tight counts: two
  // buffer fills less on the build's path)
  if (u == 0) {
    for (uint32_t i = threadIdx.x; z0 && i < n0; i += blockDim.x) z0[i] = 0;
    for (uint32_t i = threadIdx.x; z1 && i < n1; i += blockDim.x) z1[i] = 0;
  }
  for (uint32_t v = threadIdx.x; v < Vp; v += blockDim.x) row[v] = v == u ? 0u : SQ_INF;
  __syncthreads();
  if (u < V)
    for (uint32_t e = rowptr[u] + threadIdx.x; e < rowptr[u + 1]; e += blockDim.x) {
      const uint32_t v = auv[e] >> 16;
      atomicMin(&row[v], (uint32_t)al[e]);  // (< 2^32 - 1: the fast form's bound)
      if (EI) EI[(uint64_t)u * Vp + v] = e;
    }
  __syncthreads();
  for (uint32_t v = 4 * threadIdx.x; v < Vp; v += 4 * blockDim.x) {
    const uint4 r = *(const uint4*)&row[v];
    *(uint4*)&D[(uint64_t)u * Vp + v] = r;
    if (NL) {
      const uint32_t rv[4] = {r.x, r.y, r.z, r.w};
      uint32_t nv[4];
#pragma unroll
      for (int k = 0; k < 4; k++) nv[k] = v + k == u || rv[k] == SQ_INF ? kFx : 0u - rv[k];
      *(uint4*)&NL[(uint64_t)u * Vp + v] = make_uint4(nv[0], nv[1], nv[2], nv[3]);
    }
  }
  if (NDT)
    for (uint32_t j = threadIdx.x; j < Up; j += blockDim.x) {
      uint32_t x = kFx;
      if (j < ns) {
        const uint32_t sj = usrc[j];
        if (sj != u) x = 0u - row[sj];
      }
      NDT[(uint64_t)u * Up + j] = x;
    }
}

// All squaring passes in ONE launch (one shard): a 1024-thread workgroup per 64 x 64 output tile
// (looping over tiles when they outnumber the CUs) whose four 256-thread slices each take a
// quarter of K (16 waves per CU: sq_pass's 256 tiles left one wave per SIMD and ran at ~1/3 of
// the VALU rate), the slices' minima folded in LDS; each slice's next K step is loaded into
// registers while the current one is computed. A pass ends at a grid barrier (every workgroup
// resident: the grid is at most one workgroup per CU; stores drained, agent release, counter,
// agent acquire), and the launch ends after the first pass that changed nothing — a graph whose
// edges already are its shortest paths (config C's Tor graph) pays one pass and one barrier
// instead of ceil(log2 V) + 1 launches. *err: a barrier timed out (the host redoes the phase
// with sq_pass).
constexpr int SQR_SL = 4;                                   // K slices per workgroup
constexpr size_t SQR_LDS = 2ull * SQR_SL * SQ_K * (SQ_T + 4) * 4;  // As + Bs per slice
__global__ __launch_bounds__(1024) void sq_run(uint32_t* D, uint32_t Vp, uint32_t* flag, uint32_t max_pass,
                                               uint32_t* err, uint32_t* bar, const uint32_t* skip) {
  // (skip: the fused first pass's change word — 0: the matrix is already closed, and this launch
  // is its one pass that changed nothing; flag[0] stays 0)
  if (skip && *skip == 0) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef uint32_t Tile[SQ_K][SQ_T + 4];
  Tile* As = (Tile*)smem;
  Tile* Bs = As + SQR_SL;
  uint32_t* red = (uint32_t*)smem;  // [64][64] after a tile's K loop (As[0..1] are free then)
  __shared__ uint32_t go;
  const uint32_t sl = threadIdx.x >> 8, t = threadIdx.x & 255;
  const int tx = t & 15, ty = t >> 4;
  const uint32_t nt = Vp / SQ_T, ntiles = nt * nt;
  const uint32_t nsteps = Vp / SQ_K, per = (nsteps + SQR_SL - 1) / SQR_SL;
  const uint32_t s_first = sl * per;
  for (uint32_t it = 0; it < max_pass; it++) {
    bool ch = false;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      const uint64_t r0 = (uint64_t)(tile / nt) * SQ_T, c0 = (uint64_t)(tile % nt) * SQ_T;
      uint32_t acc[4][4], orig[4][4];
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = orig[i][j] = SQ_INF;
      if (sl == 0)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint4 v = *(const uint4*)&D[(r0 + ty * 4 + i) * Vp + c0 + tx * 4];
          acc[i][0] = orig[i][0] = v.x;
          acc[i][1] = orig[i][1] = v.y;
          acc[i][2] = orig[i][2] = v.z;
          acc[i][3] = orig[i][3] = v.w;
        }
      // step s's operands, thread t's share: A = D[r0 .. +64][k0 .. +32] (rows t / 8 and
      // t / 8 + 32), B = D[k0 .. +32][c0 .. +64] (rows t / 16 and t / 16 + 16)
      const uint32_t* pa = D + (r0 + (t >> 3)) * Vp + (t & 7) * 4;
      const uint32_t* pb = D + (uint64_t)(t >> 4) * Vp + c0 + (t & 15) * 4;
      const uint64_t a2 = 32ull * Vp, b2 = 16ull * Vp;
      uint4 ra0 = {}, ra1 = {}, rb0 = {}, rb1 = {};
#define SQR_LOAD(s)                                               \
  do {                                                            \
    const uint64_t k0_ = (uint64_t)(s) * SQ_K;                    \
    ra0 = *(const uint4*)(pa + k0_);                              \
    ra1 = *(const uint4*)(pa + a2 + k0_);                         \
    rb0 = *(const uint4*)(pb + k0_ * Vp);                         \
    rb1 = *(const uint4*)(pb + b2 + k0_ * Vp);                    \
  } while (0)
      if (s_first < nsteps) SQR_LOAD(s_first);
      for (uint32_t s = 0; s < per; s++) {  // (every slice takes the same number of barriers)
        const bool have = s_first + s < nsteps;
        __syncthreads();  // the previous step's LDS reads (or the last tile's fold) are done
        if (have) {
          const int m = t >> 3, kq = (t & 7) * 4;
          As[sl][kq][m] = ra0.x;
          As[sl][kq + 1][m] = ra0.y;
          As[sl][kq + 2][m] = ra0.z;
          As[sl][kq + 3][m] = ra0.w;
          As[sl][kq][m + 32] = ra1.x;
          As[sl][kq + 1][m + 32] = ra1.y;
          As[sl][kq + 2][m + 32] = ra1.z;
          As[sl][kq + 3][m + 32] = ra1.w;
          *(uint4*)&Bs[sl][t >> 4][(t & 15) * 4] = rb0;
          *(uint4*)&Bs[sl][(t >> 4) + 16][(t & 15) * 4] = rb1;
        }
        __syncthreads();
        if (have && s + 1 < per && s_first + s + 1 < nsteps) SQR_LOAD(s_first + s + 1);
        if (have) {
#pragma unroll 8
          for (int k = 0; k < SQ_K; k++) {
            const uint4 a = *(const uint4*)&As[sl][k][ty * 4];
            const uint4 b = *(const uint4*)&Bs[sl][k][tx * 4];
            const uint32_t av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
              for (int j = 0; j < 4; j++) {
                const uint32_t s2 = __builtin_elementwise_add_sat(av[i], bv[j]);
                acc[i][j] = s2 < acc[i][j] ? s2 : acc[i][j];
              }
          }
        }
      }
#undef SQR_LOAD
      // fold the slices: slice 0 (which started from the tile's entries) writes, the rest min in
      __syncthreads();
      if (sl == 0)
#pragma unroll
        for (int i = 0; i < 4; i++)
          *(uint4*)&red[(ty * 4 + i) * SQ_T + tx * 4] = make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
      __syncthreads();
      if (sl != 0)
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (acc[i][j] < SQ_INF) atomicMin(&red[(ty * 4 + i) * SQ_T + tx * 4 + j], acc[i][j]);
      __syncthreads();
      if (sl == 0)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint4 r = *(const uint4*)&red[(ty * 4 + i) * SQ_T + tx * 4];
          if (r.x != orig[i][0] || r.y != orig[i][1] || r.z != orig[i][2] || r.w != orig[i][3]) {
            *(uint4*)&D[(r0 + ty * 4 + i) * Vp + c0 + tx * 4] = r;
            ch = true;
          }
        }
    }
    // the pass's barrier: every storing wave drains, one lane releases and arrives
    if (__ballot(ch) && (threadIdx.x & 63) == 0)
      __hip_atomic_store(&flag[it], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t target = (it + 1) * gridDim.x;
      uint32_t sp = 0;
      while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++sp < (1u << 24))
        __builtin_amdgcn_s_sleep(2);
      if (sp >= (1u << 24)) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      go = __hip_atomic_load(&flag[it], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 &&
           __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
    }
    __syncthreads();
    if (!go) break;
  }
}

// Latency phase for sparse graphs: one workgroup per used source relaxes the arc list over
// its distance row in LDS (u64, 64-bit LDS atomic min) until a sweep changes nothing —
// Bellman-Ford, exact (integer latencies, all positive), a few sweeps of a short list instead
// of V^3 min-plus work. Only used sources' rows of D are written (all that is read).
__global__ __launch_bounds__(512) void bf_pass(uint64_t* D, uint32_t Vp, const uint32_t* usrc, const uint32_t* auv,
                                               const uint64_t* al, uint32_t E2, uint32_t* iters) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  unsigned long long* Dr = (unsigned long long*)smem;
  uint32_t* ch = (uint32_t*)(Dr + Vp);
  const uint32_t s = usrc[blockIdx.x];
  for (uint32_t v = threadIdx.x; v < Vp; v += blockDim.x) Dr[v] = v == s ? 0ULL : FW_INF;
  uint32_t it = 0;
  while (true) {
    if (threadIdx.x == 0) *ch = 0;
    __syncthreads();
    bool changed = false;
    for (uint32_t e = threadIdx.x; e < E2; e += blockDim.x) {
      const uint32_t uv = auv[e];
      const unsigned long long du = Dr[uv & 0xFFFFu];
      if (du >= FW_INF) continue;
      const unsigned long long nd = du + al[e];  // < 2^63: FW_INF = 2^62 bounds both terms
      if (nd < Dr[uv >> 16] && nd < atomicMin(&Dr[uv >> 16], nd)) changed = true;
    }
    if (changed) *ch = 1;
    __syncthreads();
    it++;
    if (!*ch) break;
    __syncthreads();
  }
  for (uint32_t v = threadIdx.x; v < Vp; v += blockDim.x) D[(uint64_t)s * Vp + v] = Dr[v];
  if (threadIdx.x == 0) iters[blockIdx.x] = it;
}

// D32 -> the u64 matrix the loss pass and the extraction read (2^32 - 1 -> "no path")
__global__ void sq_widen(const uint32_t* D32, uint64_t* D, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = D32[i];
    D[i] = v == SQ_INF ? FW_INF : v;
  }
}

// Tight arcs for S sources at once (u32 latency form): a workgroup holds the S sources'
// distance rows interleaved in LDS (row[u * S + k] = d[source k][u], so one arc's S tests are
// two 4S-byte reads; arcs are 8 bytes: u | v << 16 and the u32 latency) and sweeps one P-th of the arc list; each arc load now serves S sources
// instead of one (the single-source sweep re-read the whole arc list once per source, from
// L2 / MALL). Tight arcs go to a per-source list in global memory (arc indices).
// b + nl + nd as one v_add3_u32 (nd a scalar register: gfx950 VOP3 reads one SGPR); written
// out because the compiler re-associates the sum into an add and a sub
__device__ __forceinline__ uint32_t add3_vvs(uint32_t b, uint32_t nl, uint32_t nd) {
  uint32_t r;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(nl), "s"(nd));
  return r;
}

template <int S>
__device__ __forceinline__ void sweep_arc(const uint32_t* row, uint32_t g0, uint32_t uv, uint32_t l, uint32_t e,
                                          uint32_t capg, uint32_t* tcnt, uint32_t* tlist) {
  if (l == SQ_INF) return;  // 2^32 - 1 ns or more: no u32 path is that long, never tight
  const uint32_t* du = row + (uv & 0xFFFFu) * S;
  const uint32_t* dv = row + (uv >> 16) * S;
#pragma unroll
  for (int k = 0; k < S; k += 4) {
    const uint4 x = *(const uint4*)(du + k), y = *(const uint4*)(dv + k);
    const uint32_t a[4] = {x.x, x.y, x.z, x.w}, b[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (a[j] == SQ_INF || (uint64_t)a[j] + l != (uint64_t)b[j]) continue;
      const uint32_t src = g0 + k + j;
      const uint32_t pos = atomicAdd(&tcnt[src], 1u);
      if (pos < capg) tlist[(uint64_t)src * capg + pos] = e;
    }
  }
}

template <int S>
__global__ __launch_bounds__(512) void loss_sweep(const uint32_t* D32, uint32_t Vp, const uint32_t* usrc,
                                                  uint32_t U, const uint32_t* auv, const uint32_t* al32,
                                                  uint32_t E2, uint32_t capg, uint32_t* tcnt,
                                                  uint32_t* tlist) {
  static_assert(S % 4 == 0, "rows are read 4 sources at a time");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* row = (uint32_t*)smem;  // [Vp][S]
  const uint32_t g0 = blockIdx.x * S;
  for (uint32_t i = threadIdx.x; i < Vp * S; i += blockDim.x) {
    const uint32_t u = i / S, k = i % S;
    row[i] = g0 + k < U ? D32[(uint64_t)usrc[g0 + k] * Vp + u] : SQ_INF;
  }
  __syncthreads();
  // this workgroup's share of the arc list in 4-arc quads; two quads per thread in flight
  const uint32_t E4 = E2 / 4;
  const uint32_t per = (E4 + gridDim.y - 1) / gridDim.y;
  const uint32_t q0 = blockIdx.y * per, q1 = min(E4, q0 + per);
  const uint4* a4 = (const uint4*)auv;
  const uint4* l4 = (const uint4*)al32;
  for (uint32_t q = q0 + threadIdx.x; q < q1; q += 2 * blockDim.x) {
    const uint32_t q2 = q + blockDim.x;
    const bool two = q2 < q1;
    const uint4 a = a4[q], l = l4[q];
    uint4 b = make_uint4(0, 0, 0, 0), m = make_uint4(SQ_INF, SQ_INF, SQ_INF, SQ_INF);
    if (two) {
      b = a4[q2];
      m = l4[q2];
    }
    sweep_arc<S>(row, g0, a.x, l.x, 4 * q, capg, tcnt, tlist);
    sweep_arc<S>(row, g0, a.y, l.y, 4 * q + 1, capg, tcnt, tlist);
    sweep_arc<S>(row, g0, a.z, l.z, 4 * q + 2, capg, tcnt, tlist);
    sweep_arc<S>(row, g0, a.w, l.w, 4 * q + 3, capg, tcnt, tlist);
    sweep_arc<S>(row, g0, b.x, m.x, 4 * q2, capg, tcnt, tlist);
    sweep_arc<S>(row, g0, b.y, m.y, 4 * q2 + 1, capg, tcnt, tlist);
    sweep_arc<S>(row, g0, b.z, m.z, 4 * q2 + 2, capg, tcnt, tlist);
    sweep_arc<S>(row, g0, b.w, m.w, 4 * q2 + 3, capg, tcnt, tlist);
  }
  if (blockIdx.y == gridDim.y - 1)
    for (uint32_t e = 4 * E4 + threadIdx.x; e < E2; e += blockDim.x)
      sweep_arc<S>(row, g0, auv[e], al32[e], e, capg, tcnt, tlist);
}

// The same sweep over the arc list in tail order (CSR: rowptr[u] .. rowptr[u + 1] are u's arcs,
// dense graphs): a wave takes one tail u at a time, so its S distances d[s][u] are one LDS
// broadcast read kept in registers, and the lanes' heads v are consecutive (conflict-free
// reads of d[s][v]); a workgroup sweeps a range of tails. The test is d[s][v] - d[s][u] == l
// with d[s][v] >= d[s][u] (u32; an arc of 2^32 - 1 ns or more is never tight).
#ifndef SGN_SWEEP_Q
#define SGN_SWEEP_Q 16
#endif
constexpr uint32_t kSweepQ = SGN_SWEEP_Q;  // arcs per lane in flight per step
constexpr uint32_t SWEEP_HCAP = 256;       // filter hits a wave lists before checking them exactly
template <int S>
__global__ __launch_bounds__(512) void loss_sweep_csr(const uint32_t* D32, uint32_t Vp, const uint32_t* usrc,
                                                      uint32_t U, uint32_t V, const uint32_t* rowptr,
                                                      const uint32_t* auv, const uint32_t* al32, uint32_t capg,
                                                      uint32_t* tcnt, uint32_t* tlist) {
  static_assert(S % 4 == 0, "rows are read 4 sources at a time");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // S/4 planes of [Vp][4]: a lane's 16-byte read of 4 sources' d[.][v] sits at a 16-byte
  // stride from its neighbour's (conflict-free; one [Vp][S] row put the lanes 4S bytes apart)
  uint32_t* row = (uint32_t*)smem;
  const uint32_t g0 = blockIdx.x * S;
  // (all S loads of a column in flight, then one 16-byte LDS write per plane; a source past U
  // reads source 0's row and keeps INF)
  const uint32_t* src[S];
#pragma unroll
  for (int k = 0; k < S; k++) src[k] = D32 + (uint64_t)usrc[g0 + k < U ? g0 + k : 0] * Vp;
  for (uint32_t u = threadIdx.x; u < Vp; u += blockDim.x) {
    uint32_t x[S];
#pragma unroll
    for (int k = 0; k < S; k++) x[k] = src[k][u];
#pragma unroll
    for (int k = 0; k < S; k += 4)
      *(uint4*)(row + (k >> 2) * Vp * 4 + u * 4) =
          make_uint4(g0 + k < U ? x[k] : SQ_INF, g0 + k + 1 < U ? x[k + 1] : SQ_INF,
                     g0 + k + 2 < U ? x[k + 2] : SQ_INF, g0 + k + 3 < U ? x[k + 3] : SQ_INF);
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // a wave's filter hits of one 256-arc step, checked exactly after the step (after the rows)
  uint32_t* hits = (uint32_t*)smem + (size_t)Vp * S + wave * SWEEP_HCAP;
  const uint32_t u0 = (uint32_t)((uint64_t)V * blockIdx.y / gridDim.y);
  const uint32_t u1 = (uint32_t)((uint64_t)V * (blockIdx.y + 1) / gridDim.y);
  for (uint32_t u = u0 + wave; u < u1; u += nw) {
    uint32_t du[S], ndu[S];  // wave-uniform (u is): scalar operands of the filter below
#pragma unroll
    for (int k = 0; k < S; k += 4) {
      const uint4 x = *(const uint4*)(row + (k >> 2) * Vp * 4 + u * 4);
      du[k] = __builtin_amdgcn_readfirstlane(x.x);
      du[k + 1] = __builtin_amdgcn_readfirstlane(x.y);
      du[k + 2] = __builtin_amdgcn_readfirstlane(x.z);
      du[k + 3] = __builtin_amdgcn_readfirstlane(x.w);
    }
#pragma unroll
    for (int k = 0; k < S; k++) ndu[k] = 0u - du[k];
    // kSweepQ arcs per lane in flight (e, e + 64, ...): the sweep waits on the arc loads (PMC,
    // round 4: 84 % of its wave cycles waiting with one arc per lane)
    const uint32_t e_beg = rowptr[u], e1 = rowptr[u + 1];
    for (uint32_t e0 = e_beg + lane; e0 - lane < e1; e0 += 64 * kSweepQ) {
      uint32_t uv[kSweepQ], l[kSweepQ];
#pragma unroll
      for (int q = 0; q < (int)kSweepQ; q++) {  // (clamped, unconditional loads: all in flight at once;
        // 32-bit byte offsets from the scalar bases)
        const uint32_t off = min(e0 + 64 * q, e1 - 1) * 4u;
        uv[q] = *(const uint32_t*)((const char*)auv + off);
        l[q] = *(const uint32_t*)((const char*)al32 + off);
      }
      uint32_t nh = 0;  // (wave-uniform)
      // the exact test of the listed hits (it also drops the clamped lanes past the tail's last
      // arc, and arcs of 2^32 - 1 ns or more)
      auto check = [&](uint32_t n) {
        for (uint32_t h = lane; h < n; h += 64) {
          const uint32_t e = hits[h];
          if (e >= e1) continue;
          const uint32_t lq = al32[e];
          if (lq == SQ_INF) continue;
          const uint32_t v = auv[e] >> 16;
#pragma unroll
          for (int k = 0; k < S; k++) {
            const uint32_t bk = row[(k >> 2) * Vp * 4 + v * 4 + (k & 3)];
            if (du[k] == SQ_INF || bk < du[k] || bk - du[k] != lq) continue;
            const uint32_t src = g0 + k;
            const uint32_t pos = atomicAdd(&tcnt[src], 1u);
            if (pos < capg) tlist[(uint64_t)src * capg + pos] = e;
          }
        }
      };
#pragma unroll
      for (int q = 0; q < (int)kSweepQ; q++) {
        const uint32_t v = uv[q] >> 16;
        uint32_t b[S];
#pragma unroll
        for (int k = 0; k < S; k += 4) {
          const uint4 y = *(const uint4*)(row + (k >> 2) * Vp * 4 + v * 4);
          b[k] = y.x;
          b[k + 1] = y.y;
          b[k + 2] = y.z;
          b[k + 3] = y.w;
        }
        // branch-free filter: b - l - du (one v_add3 with -l and the scalar -du) is 0 for every
        // tight (source, arc) pair (and, rarely, for a wrapped one). About one pair in a
        // thousand is tight, yet ~40 % of wave steps hold a hit in some lane: hits are listed
        // (ballot + mbcnt, no divergence) and checked exactly after the step, lane-parallel
        const uint32_t nl = 0u - l[q];
        uint32_t acc = add3_vvs(b[0], nl, ndu[0]);
#pragma unroll
        for (int k = 1; k < S; k++) acc = min(acc, add3_vvs(b[k], nl, ndu[k]));
        const uint64_t m = __ballot(acc == 0);
        if (m) {
          if (acc == 0) hits[nh + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = e0 + 64 * q;
          nh += (uint32_t)__popcll(m);
          if (nh > SWEEP_HCAP - 64) {  // (a full list is checked now: room for the next arc's 64)
            check(nh);
            nh = 0;
          }
        }
      }
      if (nh) check(nh);
    }
  }
}

// Dense graphs (at least half of all arcs present, no parallel arcs; round 6): the same tight
// test as a dense sweep over (source, tail, head) with nothing from LDS in its inner loop. In
// loss_sweep_csr every (source, arc) pair reads d[s][v] from LDS (4 B a pair: the LDS return path
// and the VALU were both near their limits). Here a lane owns one head v and keeps the S
// sources' d[s][v] in registers for the whole launch; a wave walks a range of tails u, and per
// tail the lane loads one word, the arc's latency L[u][v] from the dense latency matrix
// (coalesced over the wave's heads), while the S values -d[s][u] are scalar loads (NDT: the used
// sources' distance columns, transposed and negated). Per pair: one v_add3_u32 and half a
// v_min3. Arcs are looked up through a dense (tail, head) -> arc index matrix, so the tight
// lists hold the same arc indices as the CSR form, and the fold reads them alike.
// A source's own out-arcs (tail u = s) are taken apart (the first tail range's workgroups test
// them from registers before the sweep): on graphs whose edges are
// their own shortest paths (config C's Tor graph) they are nearly all of the tight pairs, and
// in the sweep they would fill every lane's hit list at the few tails that are sources.
// The fused form (kF, complete graphs with every latency below 2^29 ns): the sweep runs on the
// matrix of direct arcs BEFORE the squaring. It is the squaring's first pass restricted to the
// used sources: its filter d[s][v] - l(u,v) - d[s][u], read as a signed number, is positive
// exactly when the arc (u, v) shortens s's path to v, and zero when it is tight. The sweep folds
// it by a signed max: no positive value anywhere means every used source's row of direct arcs
// is already closed (Bellman's condition on every arc, so the rows are the shortest paths) and
// the tight lists are final; the squaring launch then returns at once (one pass that changed
// nothing) and the loss phase only folds. Otherwise the change word is set, the squaring runs
// as usual and the loss phase sweeps the final matrix (same form: its entries only shrank).
// Excluded pairs carry -2^30 (`kFx`) instead of -SQ_INF, so their signed value stays negative.
constexpr uint32_t kDenseQ = 8;  // tails whose latency loads are in flight at once
// filter hits a wave lists before checking them exactly: room for one more batch of kDenseQ tails
// after any fill below the threshold, so the list is checked once per batch at most (one copy
// of the check in the code: a copy per unrolled tail made the kernel 19 k lines)
constexpr uint32_t DENSE_HCAP = 2 * 64 * kDenseQ;  // (kDenseQ hit lists per batch: Q tails x H heads)

// NL32[u][v] = minus the arc's u32 latency (the filter's operand as it is used; entries without
// an arc keep the fill: 1 = -SQ_INF, or kFx in the fused form), EI[u][v] = its index (no
// parallel arcs)
__global__ void dense_arcs(const uint32_t* auv, const uint32_t* al32, uint32_t E2, uint32_t Vp, uint32_t* NL32,
                           uint32_t* EI) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < E2; e += gridDim.x * blockDim.x) {
    const uint32_t uv = auv[e];
    const size_t i = (size_t)(uv & 0xFFFFu) * Vp + (uv >> 16);
    NL32[i] = 0u - al32[e];
    EI[i] = e;
  }
}

// NDT[u][j] = -d[usrc[j]][u] (u32), through a 64 x 64 LDS tile (rows of D32 read along u, NDT
// written along j). 1 (= -SQ_INF: the filter never passes it, the exact test rejects it; kFx in
// the fused form) for the padding sources j >= ns and for u = usrc[j] (the sweep's own-arc step takes
// those arcs). gate: run only if *gate != 0 (the fused pass found a change); zero: the tight
// counts to clear first (the loss phase's sweep after a change).
template <bool kF>
__global__ __launch_bounds__(256) void ndt_build(const uint32_t* D32, uint32_t Vp, const uint32_t* usrc, uint32_t ns,
                                                 uint32_t* NDT, uint32_t Up, const uint32_t* gate, uint32_t* zero) {
  if (gate && *gate == 0) return;
  if (zero)
    for (uint32_t i = (blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x; i < ns; i += gridDim.x * gridDim.y * 256)
      zero[i] = 0;
  __shared__ uint32_t tile[64][65];
  const uint32_t j0 = blockIdx.x * 64, u0 = blockIdx.y * 64, c = threadIdx.x & 63;
#pragma unroll
  for (uint32_t jj = threadIdx.x >> 6; jj < 64; jj += 4) {
    const uint32_t j = j0 + jj, u = u0 + c;
    uint32_t x = kF ? kFx : 1u;
    if (j < ns && u < Vp) {
      const uint32_t s = usrc[j];
      if (u != s) x = 0u - D32[(size_t)s * Vp + u];
    }
    tile[jj][c] = x;
  }
  __syncthreads();
  for (uint32_t uu = threadIdx.x >> 6; uu < 64; uu += 4) {
    const uint32_t u = u0 + uu, j = j0 + c;
    if (u < Vp && j < Up) NDT[(size_t)u * Up + j] = tile[c][uu];
  }
}

// 16 scalar words in one s_load_dwordx16 issued now and waited for later (swait16): the compiler
// waits for its own scalar loads at their first use with lgkmcnt(0), which exposed the whole
// latency at every tail (the first build ran at 60 % of VALU issue, PMC)
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ u32x16 sload16(const uint32_t* p) {
  u32x16 r;
  asm volatile("s_load_dwordx16 %0, %1, 0x0" : "=s"(r) : "s"(p));
  return r;
}

// grid (ceil(ns / S), ceil(Vp / (256 H)), tail ranges); 256 threads, thread t owns the H heads
// v0 + t + 256 h. The filter folds the sources in groups of 8, so a hit names the groups to test
// exactly. Per tail the S values -d[s][u] are loaded one tail ahead (asm: issued before the
// tail's work, waited for after it) and serve H heads per lane.
template <int S, int H, bool kF>
__global__ __launch_bounds__(256) void loss_sweep_dense(const uint32_t* __restrict__ D32, uint32_t Vp,
                                                        const uint32_t* __restrict__ usrc, uint32_t U, uint32_t V,
                                                        const uint32_t* __restrict__ NDT, uint32_t Up,
                                                        const uint32_t* __restrict__ NL32,
                                                        const uint32_t* __restrict__ EI, uint32_t capg,
                                                        uint32_t* __restrict__ tcnt, uint32_t* __restrict__ tlist,
                                                        const uint32_t* gate, uint32_t* chg) {
  if (gate && *gate == 0) return;
  static_assert(S % 16 == 0 && S <= 32, "sources per tail come in 16-word scalar loads");
  static_assert(H == 1 || H == 2, "heads per lane");
  constexpr int NG = S / 16, NV = S / 16;  // filter groups of 16 sources = the scalar loads
  constexpr uint32_t Q = kDenseQ / H;  // tails per batch (Q * H latency loads in flight)
  __shared__ uint32_t hits[4][DENSE_HCAP];
  __shared__ uint32_t srow[S];  // the sources' row offsets in D32 (for the exact test)
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // XCD-aware order: blocks id, id + 8, ... share an XCD (MI355X_MICROARCH.md), so each XCD takes a
  // contiguous run of (source tile, head block, tail range) with the source tile fastest — the
  // tiles that read one block of NL32 run together on one XCD and find it in that XCD's L2
  const uint32_t nblk = gridDim.x * gridDim.y * gridDim.z;
  const uint32_t id = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const uint32_t xq = nblk >> 3, xr = nblk & 7, xc = id & 7;
  const uint32_t lin = xc * xq + min(xc, xr) + (id >> 3);
  const uint32_t bx = lin % gridDim.x, by = (lin / gridDim.x) % gridDim.y, bz = lin / (gridDim.x * gridDim.y);
  const uint32_t g0 = bx * S, v0 = by * 256 * H;
  uint32_t vc[H];  // (heads past V: the exact test drops them)
#pragma unroll
  for (int h = 0; h < H; h++) vc[h] = min(v0 + t + 256 * h, Vp - 1);
  if (t < S) srow[t] = usrc[g0 + t < U ? g0 + t : 0] * Vp;
  __syncthreads();
  uint32_t dv[H][S];
#pragma unroll
  for (int k = 0; k < S; k++)
#pragma unroll
    for (int h = 0; h < H; h++)
      dv[h][k] = g0 + k < U && (!kF || v0 + t + 256 * h < V) ? D32[srow[k] + vc[h]] : kF ? 0u : SQ_INF;
  const uint32_t u0 = (uint32_t)((uint64_t)V * bz / gridDim.z);
  const uint32_t u1 = (uint32_t)((uint64_t)V * (bz + 1) / gridDim.z);
  // the sources' own out-arcs (tail u = s, excluded from the sweep below: NDT holds -SQ_INF or
  // kFx there), source k by the workgroups of tail range k mod (tail ranges): d[s][v] is in
  // registers, one append per wave and (source, head) with a tight lane
  {
#pragma unroll
    for (int k = 0; k < S; k++) {
      if (g0 + k >= U) break;
      if ((uint32_t)k % gridDim.z != bz) continue;
      const uint32_t sr = srow[k], sn = sr / Vp, du = D32[sr + sn];
#pragma unroll
      for (int h = 0; h < H; h++) {
        const uint32_t v = v0 + t + 256 * h;
        bool tight = false;
        if (v < V && du != SQ_INF) {
          const uint32_t lq = 0u - NL32[sr + v], bk = dv[h][k];
          tight = lq != SQ_INF && bk >= du && bk - du == lq;
        }
        const uint64_t m = __ballot(tight);
        if (!m) continue;
        const uint32_t first = (uint32_t)__builtin_ctzll(m);
        uint32_t base = 0;
        if (lane == first) base = atomicAdd(&tcnt[g0 + k], (uint32_t)__popcll(m));
        base = __shfl(base, (int)first, 64);
        if (tight) {
          const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (pos < capg) tlist[(uint64_t)(g0 + k) * capg + pos] = EI[sr + v];
        }
      }
    }
  }
  // the exact test of the listed hits, lane-parallel; an entry is u << 13 | groups << 9 | head
  // offset, and a group's 16 values of d[s][u] and d[s][v] are loaded at once
  auto check = [&](uint32_t n) {
    for (uint32_t i = lane; i < n; i += 64) {
      const uint32_t ent = hits[wave][i], u = ent >> 13, gm = (ent >> 9) & 15u, v = v0 + (ent & 511u);
      if (v >= V) continue;
      const uint32_t lq = 0u - NL32[(size_t)u * Vp + v];
      if (lq == SQ_INF) continue;  // no arc (or one of 2^32 - 1 ns or more: never tight)
      const uint32_t* nd = NDT + (size_t)u * Up + g0;
      for (int gi = 0; gi < NG; gi++) {
        if (!((gm >> gi) & 1u)) continue;
        uint32_t nk[16], bk[16];
#pragma unroll
        for (int k = 0; k < 16; k += 4) {
          const uint4 x = *(const uint4*)(nd + 16 * gi + k);
          nk[k] = x.x;
          nk[k + 1] = x.y;
          nk[k + 2] = x.z;
          nk[k + 3] = x.w;
        }
#pragma unroll
        for (int k = 0; k < 16; k++) bk[k] = D32[srow[16 * gi + k] + v];
#pragma unroll
        for (int k = 0; k < 16; k++) {
          const uint32_t src = g0 + 16 * gi + k, du = 0u - nk[k];
          if (src >= U || du == SQ_INF || bk[k] < du || bk[k] - du != lq) continue;
          const uint32_t pos = atomicAdd(&tcnt[src], 1u);
          if (pos < capg) tlist[(uint64_t)src * capg + pos] = EI[(size_t)u * Vp + v];
        }
      }
    }
  };
  // (32-bit byte offsets from the scalar base: Vp <= 8192 keeps NL32 under 4 GB)
  auto lrow = [&](uint32_t u, int h) {
    return *(const uint32_t*)((const char*)NL32 + (min(u, u1 - 1) * Vp + vc[h]) * 4u);
  };
  auto ndrow = [&](uint32_t u) { return NDT + (size_t)min(u, u1 - 1) * Up + g0; };
  uint32_t lc[Q][H];
#pragma unroll
  for (int q = 0; q < (int)Q; q++)
#pragma unroll
    for (int h = 0; h < H; h++) lc[q][h] = lrow(u0 + q, h);
  u32x16 cur[NV];
#pragma unroll
  for (int i = 0; i < NV; i++) cur[i] = sload16(ndrow(u0) + 16 * i);
  if constexpr (NV == 1) asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(cur[0]));
  else asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(cur[0]), "+s"(cur[NV - 1]));
  uint32_t nh = 0;  // (wave-uniform)
  bool grew = false;  // (kF) some arc shortens some source's path
  for (uint32_t ub = u0; ub < u1; ub += Q) {
    uint32_t ln[Q][H];  // the next batch's latencies, loaded while this one computes
#pragma unroll
    for (int q = 0; q < (int)Q; q++)
#pragma unroll
      for (int h = 0; h < H; h++) ln[q][h] = lrow(ub + Q + q, h);
#pragma unroll
    for (int q = 0; q < (int)Q; q++) {
      const uint32_t u = ub + q;
      if (u >= u1) break;
      u32x16 nxt[NV];  // the next tail's -d[s][u], in flight during this tail's work
#pragma unroll
      for (int i = 0; i < NV; i++) nxt[i] = sload16(ndrow(u + 1) + 16 * i);
      uint32_t amin[H], a[H][NG];
#pragma unroll
      for (int h = 0; h < H; h++) {
        const uint32_t nl = lc[q][h];  // (NL32 holds -latency)
#pragma unroll
        for (int gi = 0; gi < NG; gi++) {
          uint32_t acc = add3_vvs(dv[h][16 * gi], nl, cur[gi][0]);
#pragma unroll
          for (int k = 1; k < 16; k++) {
            const uint32_t x = add3_vvs(dv[h][16 * gi + k], nl, cur[gi][k]);
            acc = kF ? (uint32_t)max((int32_t)acc, (int32_t)x) : min(acc, x);
          }
          a[h][gi] = acc;
        }
        amin[h] = a[h][0];
#pragma unroll
        for (int gi = 1; gi < NG; gi++) amin[h] = kF ? (uint32_t)max((int32_t)amin[h], (int32_t)a[h][gi]) : min(amin[h], a[h][gi]);
        if constexpr (kF) grew |= (int32_t)amin[h] > 0;
      }
#pragma unroll
      for (int h = 0; h < H; h++) {
        const uint64_t m = __ballot(amin[h] == 0);
        if (m) {
          if (amin[h] == 0) {
            uint32_t gm = 0;
#pragma unroll
            for (int gi = 0; gi < NG; gi++) gm |= a[h][gi] == 0 ? 1u << gi : 0u;
            hits[wave][nh + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                (u << 13) | (gm << 9) | (t + 256 * h);
          }
          nh += (uint32_t)__popcll(m);
        }
      }
      // the next tail's scalars have arrived (the wait follows this tail's filter: amin)
      uint32_t am = amin[0];
#pragma unroll
      for (int h = 1; h < H; h++) am = min(am, amin[h]);
      if constexpr (NV == 1) asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(nxt[0]) : "v"(am));
      else asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(nxt[0]), "+s"(nxt[NV - 1]) : "v"(am));
#pragma unroll
      for (int i = 0; i < NV; i++) cur[i] = nxt[i];
    }
#pragma unroll
    for (int q = 0; q < (int)Q; q++)
#pragma unroll
      for (int h = 0; h < H; h++) lc[q][h] = ln[q][h];
    if (nh > DENSE_HCAP - 64 * kDenseQ || (nh && ub + Q >= u1)) {
      check(nh);
      nh = 0;
    }
  }
  if constexpr (kF) {
    if (chg && __ballot(grew) && lane == 0) atomicOr(chg, 1u);
  }
}

// The loss fold of one used source over its tight list (from loss_sweep): the list into LDS,
// then the fixed point as in loss_pass. (tcnt > capg: the caller reruns loss_pass instead.)
__global__ __launch_bounds__(256) void loss_fold(uint32_t Vp, const uint32_t* usrc, const uint32_t* auv,
                                                 const float* ap, const uint32_t* tcnt, const uint32_t* tlist,
                                                 uint32_t capg, uint32_t cap, float* Lout, uint32_t* iters) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* L = (float*)smem;
  uint32_t* tuv = (uint32_t*)(L + Vp);
  float* tp = (float*)(tuv + cap);
  uint32_t* ctl = (uint32_t*)(tp + cap);
  const uint32_t s = usrc[blockIdx.x];
  const uint32_t nt = min(tcnt[blockIdx.x], capg);
  const bool in_lds = nt <= cap;
  for (uint32_t v = threadIdx.x; v < Vp; v += blockDim.x) L[v] = 2.0f;
  if (in_lds)
    for (uint32_t i = threadIdx.x; i < nt; i += blockDim.x) {
      const uint32_t e = tlist[(uint64_t)blockIdx.x * capg + i];
      tuv[i] = auv[e];
      tp[i] = ap[e];
    }
  __syncthreads();
  if (threadIdx.x == 0) L[s] = 0.0f;
  uint32_t it = 0;
  while (true) {
    __syncthreads();
    if (threadIdx.x == 0) ctl[0] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nt; i += blockDim.x) {
      uint32_t uv;
      float pe;
      if (in_lds) {
        uv = tuv[i];
        pe = tp[i];
      } else {
        const uint32_t e = tlist[(uint64_t)blockIdx.x * capg + i];
        uv = auv[e];
        pe = ap[e];
      }
      const float lu = L[uv & 0xFFFFu];
      if (lu > 1.0f) continue;
      const float cand = __fsub_rn(1.0f, __fmul_rn(__fsub_rn(1.0f, lu), __fsub_rn(1.0f, pe)));
      const uint32_t cb = __float_as_uint(cand);
      float* lv = &L[uv >> 16];
      if (cb < __float_as_uint(*lv)) {
        const uint32_t old = atomicMin((unsigned int*)lv, cb);
        if (cb < old) ctl[0] = 1;
      }
    }
    __syncthreads();
    it++;
    if (!ctl[0]) break;
  }
  for (uint32_t v = threadIdx.x; v < Vp; v += blockDim.x) Lout[(uint64_t)blockIdx.x * Vp + v] = L[v];
  if (threadIdx.x == 0) iters[blockIdx.x] = it | (in_lds ? 0u : 0x80000000u);
}

// Tight-arc loss fold, one workgroup per used source. The arcs that are tight for the
// source (d[s][u] + lat(u,v) == d[s][v]) are found in ONE sweep over the arc list and kept in
// LDS (packed u | v << 16 and the arc's loss); the fixed point then iterates over that short
// list only. A source with more tight arcs than the LDS list holds falls back to sweeping the
// global arc list each iteration. The fixed point is the same in any order (min of an isotone
// fold), so the LDS list order (atomic appends) does not matter.
// LDS: D row (u64 x Vp), loss row (f32 x Vp), tight list (2 x u32 x cap), 3 counters.
__global__ __launch_bounds__(512) void loss_pass(const uint64_t* D, uint32_t Vp,
                                                 const uint32_t* usrc, const uint32_t* auv,
                                                 const uint64_t* al, const float* ap, uint32_t E2,
                                                 uint32_t cap, float* Lout, uint32_t* iters) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t* Dr = (uint64_t*)smem;
  float* L = (float*)(Dr + Vp);
  uint32_t* tuv = (uint32_t*)(L + Vp);
  float* tp = (float*)(tuv + cap);
  uint32_t* ctl = (uint32_t*)(tp + cap);  // [0] tight count, [1] changed
  const uint32_t s = usrc[blockIdx.x];
  for (uint32_t v = threadIdx.x; v < Vp; v += blockDim.x) {
    Dr[v] = D[(uint64_t)s * Vp + v];
    L[v] = 2.0f;  // "no path yet": larger than any loss in [0, 1]
  }
  if (threadIdx.x == 0) ctl[0] = 0;
  __syncthreads();
  if (threadIdx.x == 0) L[s] = 0.0f;  // the source's score is PathProperties::default()
  // one sweep: the source's tight arcs into LDS. Four arcs per thread per step with 16-byte
  // loads, two steps in flight: the sweep is bound by how many loads each thread keeps
  // outstanding, not by bytes.
  auto tight = [&](uint32_t uv, uint64_t l, uint32_t e) {
    const uint64_t du = Dr[uv & 0xFFFFu];
    if (du >= FW_INF || du + l != Dr[uv >> 16]) return;
    const uint32_t k = atomicAdd(&ctl[0], 1u);
    if (k < cap) {
      tuv[k] = uv;
      tp[k] = ap[e];
    }
  };
  const uint32_t E4 = E2 / 4;
  const uint4* auv4 = (const uint4*)auv;
  const ulonglong2* al2 = (const ulonglong2*)al;
  for (uint32_t q = threadIdx.x; q < E4; q += 2 * blockDim.x) {
    const uint32_t q2 = q + blockDim.x;
    const bool two = q2 < E4;
    const uint4 a = auv4[q];
    const ulonglong2 l0 = al2[2 * q], l1 = al2[2 * q + 1];
    uint4 b = make_uint4(0, 0, 0, 0);
    ulonglong2 m0 = make_ulonglong2(0, 0), m1 = make_ulonglong2(0, 0);
    if (two) {
      b = auv4[q2];
      m0 = al2[2 * q2];
      m1 = al2[2 * q2 + 1];
    }
    tight(a.x, l0.x, 4 * q);
    tight(a.y, l0.y, 4 * q + 1);
    tight(a.z, l1.x, 4 * q + 2);
    tight(a.w, l1.y, 4 * q + 3);
    if (two) {
      tight(b.x, m0.x, 4 * q2);
      tight(b.y, m0.y, 4 * q2 + 1);
      tight(b.z, m1.x, 4 * q2 + 2);
      tight(b.w, m1.y, 4 * q2 + 3);
    }
  }
  for (uint32_t e = 4 * E4 + threadIdx.x; e < E2; e += blockDim.x) tight(auv[e], al[e], e);
  __syncthreads();
  const uint32_t nt = ctl[0];
  const bool in_lds = nt <= cap;
  uint32_t it = 0;
  while (true) {
    __syncthreads();
    if (threadIdx.x == 0) ctl[1] = 0;
    __syncthreads();
    const uint32_t n = in_lds ? nt : E2;
    for (uint32_t e = threadIdx.x; e < n; e += blockDim.x) {
      uint32_t uv;
      float pe;
      if (in_lds) {
        uv = tuv[e];
        pe = tp[e];
      } else {
        uv = auv[e];
        const uint64_t du = Dr[uv & 0xFFFFu];
        if (du >= FW_INF || du + al[e] != Dr[uv >> 16]) continue;
        pe = ap[e];
      }
      const float lu = L[uv & 0xFFFFu];
      if (lu > 1.0f) continue;
      const float cand = __fsub_rn(1.0f, __fmul_rn(__fsub_rn(1.0f, lu), __fsub_rn(1.0f, pe)));
      const uint32_t cb = __float_as_uint(cand);
      float* lv = &L[uv >> 16];
      if (cb < __float_as_uint(*lv)) {
        const uint32_t old = atomicMin((unsigned int*)lv, cb);
        if (cb < old) ctl[1] = 1;
      }
    }
    __syncthreads();
    it++;
    if (!ctl[1]) break;
  }
  for (uint32_t v = threadIdx.x; v < Vp; v += blockDim.x) Lout[(uint64_t)blockIdx.x * Vp + v] = L[v];
  if (threadIdx.x == 0) iters[blockIdx.x] = it | (in_lds ? 0u : 0x80000000u);
}

// The U x U table straight into the engine's device buffers: latency from D, loss from the
// loss rows, each used node's (n,n) entry replaced by its single self-loop edge
// (graph/mod.rs:209-215). One workgroup per used source row of [row0, row1): the row's
// {first disconnected column, min latency, max latency} go to rowres[3 i ..] with plain
// stores (no same-address atomics across thousands of waves: that serialised the old form
// at ~88 atomics/us on one word), and extract_fold reduces the rows into res.
template <bool k32>  // the distances as the u32 squaring left them (SQ_INF: no u32 path) or u64
__global__ __launch_bounds__(256) void extract(const void* __restrict__ Dv, uint32_t Vp,
                                               const float* __restrict__ Lrows, const uint32_t* __restrict__ uidx,
                                               uint32_t U, const uint64_t* self_lat, const float* self_loss,
                                               uint64_t* lat, float* loss, uint64_t* rowres, uint32_t row0) {
  __shared__ uint64_t sh[3][4];
  const uint32_t i = row0 + blockIdx.x;
  const uint64_t base = (uint64_t)i * U;
  const uint64_t* drow = (const uint64_t*)Dv + (uint64_t)uidx[i] * Vp;
  const uint32_t* drow32 = (const uint32_t*)Dv + (uint64_t)uidx[i] * Vp;
  const float* lrow = Lrows + (uint64_t)i * Vp;
  uint64_t mn = ~0ULL, mx = 0;
  uint32_t bad = 0xFFFFFFFFu;
  for (uint32_t j = threadIdx.x; j < U; j += blockDim.x) {
    uint64_t l;
    float p;
    if (i == j) {
      l = self_lat[i];
      p = self_loss[i];
    } else {
      const uint32_t c = uidx[j];
      if constexpr (k32) {
        const uint32_t d = drow32[c];
        l = d == SQ_INF ? FW_INF : d;
      } else {
        l = drow[c];
      }
      p = lrow[c];
      if (l >= FW_INF && j < bad) bad = j;
    }
    lat[base + j] = l;
    loss[base + j] = p;
    mn = l < mn ? l : mn;
    mx = l > mx ? l : mx;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64);
    const uint32_t c = __shfl_xor(bad, off, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
    bad = c < bad ? c : bad;
  }
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[0][w] = bad == 0xFFFFFFFFu ? ~0ULL : base + bad;
    sh[1][w] = mn;
    sh[2][w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t b0 = sh[0][0], m0 = sh[1][0], x0 = sh[2][0];
    for (uint32_t k = 1; k < (blockDim.x >> 6); k++) {
      b0 = sh[0][k] < b0 ? sh[0][k] : b0;
      m0 = sh[1][k] < m0 ? sh[1][k] : m0;
      x0 = sh[2][k] > x0 ? sh[2][k] : x0;
    }
    rowres[3 * (uint64_t)i] = b0;
    rowres[3 * (uint64_t)i + 1] = m0;
    rowres[3 * (uint64_t)i + 2] = x0;
  }
}
// rows [row0, row1) of rowres into res = {first disconnected pair index, min, max}: one
// workgroup, three atomics (res also carries the other shard blocks' results)
__global__ __launch_bounds__(256) void extract_fold(const uint64_t* rowres, uint32_t row0, uint32_t row1,
                                                    unsigned long long* res) {
  __shared__ uint64_t sh[3][4];
  uint64_t b = ~0ULL, mn = ~0ULL, mx = 0;
  for (uint32_t i = row0 + threadIdx.x; i < row1; i += blockDim.x) {
    const uint64_t x = rowres[3 * (uint64_t)i], y = rowres[3 * (uint64_t)i + 1], z = rowres[3 * (uint64_t)i + 2];
    b = x < b ? x : b;
    mn = y < mn ? y : mn;
    mx = z > mx ? z : mx;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t x = __shfl_xor(b, off, 64), y = __shfl_xor(mn, off, 64), z = __shfl_xor(mx, off, 64);
    b = x < b ? x : b;
    mn = y < mn ? y : mn;
    mx = z > mx ? z : mx;
  }
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[0][w] = b;
    sh[1][w] = mn;
    sh[2][w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t k = 1; k < (blockDim.x >> 6); k++) {
      b = sh[0][k] < b ? sh[0][k] : b;
      mn = sh[1][k] < mn ? sh[1][k] : mn;
      mx = sh[2][k] > mx ? sh[2][k] : mx;
    }
    if (b != ~0ULL) atomicMin(&res[0], (unsigned long long)b);
    atomicMin(&res[1], (unsigned long long)mn);
    atomicMax(&res[2], (unsigned long long)mx);
  }
}

}  // namespace sgn

using namespace sgn;

namespace {

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) hipFree(p);
  }
};

template <typename T>
int upload(sgn_ctx* ctx, DevBuf& b, const T* src, size_t n) {
  SGN_HIP(ctx, hipMalloc(&b.p, std::max<size_t>(n, 1) * sizeof(T)));
  if (n) SGN_HIP(ctx, hipMemcpy(b.p, src, n * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

}  // namespace

// The host mirror of the device table, copied on first use by a CPU-side consumer
// (sgn_route_get, sgn_routes_copy, worker_getLatency); the engine never needs it.
int sgn::ensure_host_routes(sgn_ctx* ctx) {
  if (ctx->h_routes) return 0;
  const size_t n = (size_t)ctx->U * ctx->U;
  ctx->h_lat.resize(n);
  ctx->h_loss.resize(n);
  SGN_HIP(ctx, hipMemcpy(ctx->h_lat.data(), ctx->d_lat, n * 8, hipMemcpyDeviceToHost));
  SGN_HIP(ctx, hipMemcpy(ctx->h_loss.data(), ctx->d_loss, n * 4, hipMemcpyDeviceToHost));
  ctx->h_routes = true;
  return 0;
}

extern "C" int sgn_routes_build(sgn_ctx* ctx, const sgn_graph* g, const uint32_t* used,
                                uint32_t U, int32_t use_shortest_path) {
  if (!ctx || !g || (!used && U)) return SGN_EINVAL;
  if (U == 0) return set_error(ctx, SGN_EINVAL, "no used nodes");
  if (g->n_nodes == 0) return set_error(ctx, SGN_EINVAL, "graph has no nodes");
  SGN_HIP(ctx, hipSetDevice(ctx->device));
  const uint32_t V = g->n_nodes, E = g->n_edges;
  std::unordered_map<uint32_t, uint32_t> idx;  // GML id -> NodeIndex (last wins, mod.rs:159)
  idx.reserve(V * 2);
  for (uint32_t i = 0; i < V; i++) idx[g->node_id[i]] = i;
  std::vector<uint32_t> uidx(U), es(E), ed(E);
  for (uint32_t i = 0; i < U; i++) {
    auto it = idx.find(used[i]);
    if (it == idx.end())
      return set_error(ctx, SGN_EINVAL, "used node " + std::to_string(used[i]) + " is not in the graph");
    uidx[i] = it->second;
  }
  for (uint32_t k = 0; k < E; k++) {
    auto a = idx.find(g->edge_src[k]);
    auto b = idx.find(g->edge_dst[k]);
    if (a == idx.end()) return set_error(ctx, SGN_EINVAL, "Edge source " + std::to_string(g->edge_src[k]) + " doesn't exist");
    if (b == idx.end()) return set_error(ctx, SGN_EINVAL, "Edge target " + std::to_string(g->edge_dst[k]) + " doesn't exist");
    if (g->edge_latency_ns[k] == 0) return set_error(ctx, SGN_EINVAL, "Edge 'latency' must not be 0");
    if (g->edge_latency_ns[k] >= (1ULL << 60)) return set_error(ctx, SGN_ERANGE, "edge latency too large");
    const float p = g->edge_loss[k];
    if (!(p >= 0.0f && p <= 1.0f)) return set_error(ctx, SGN_EINVAL, "Edge 'packet_loss' is not in the range [0,1]");
    es[k] = a->second;
    ed[k] = b->second;
  }
  // exactly-one-edge lookup (get_edge_weight, graph/mod.rs:254-287; undirected counts both
  // orientations, a self-loop once)
  auto key = [](uint32_t a, uint32_t b) { return ((uint64_t)a << 32) | b; };
  std::unordered_map<uint64_t, std::pair<uint32_t, uint32_t>> pairs;  // (count, first edge)
  const bool need_pairs = !use_shortest_path;
  std::vector<uint32_t> self_count(V, 0), self_edge(V, 0);
  for (uint32_t k = 0; k < E; k++) {
    if (es[k] == ed[k]) {
      if (self_count[es[k]]++ == 0) self_edge[es[k]] = k;
    }
    if (need_pairs) {
      auto add = [&](uint64_t kk) {
        auto& e = pairs[kk];
        if (e.first++ == 0) e.second = k;
      };
      add(key(es[k], ed[k]));
      if (!g->directed && es[k] != ed[k]) add(key(ed[k], es[k]));
    }
  }
  auto edge_msg = [&](uint32_t c, uint32_t a, uint32_t b) {
    return std::string(c == 0 ? "No edge connecting node " : "More than one edge connecting node ") +
           std::to_string(g->node_id[a]) + " to " + std::to_string(g->node_id[b]);
  };
  std::vector<uint64_t> lat;  // direct paths only (the shortest-path table stays on the device)
  std::vector<float> loss;
  hipEvent_t e0, e1, e2, e3;
  SGN_HIP(ctx, hipEventCreate(&e0));
  SGN_HIP(ctx, hipEventCreate(&e1));
  SGN_HIP(ctx, hipEventCreate(&e2));
  SGN_HIP(ctx, hipEventCreate(&e3));
  struct EvGuard {
    hipEvent_t* e;
    ~EvGuard() {
      for (int i = 0; i < 4; i++) hipEventDestroy(e[i]);
    }
  };
  hipEvent_t evs[4] = {e0, e1, e2, e3};
  EvGuard guard{evs};
  sgn_routes_timing tm{};
  tm.tile = FW_T;
  if (!use_shortest_path) {
    lat.resize((size_t)U * U);
    loss.resize((size_t)U * U);
    for (uint32_t i = 0; i < U; i++)
      for (uint32_t j = 0; j < U; j++) {
        auto it = pairs.find(key(uidx[i], uidx[j]));
        const uint32_t c = it == pairs.end() ? 0 : it->second.first;
        if (c != 1) return set_error(ctx, SGN_EINVAL, edge_msg(c, uidx[i], uidx[j]));
        const uint32_t k = it->second.second;
        lat[(size_t)i * U + j] = g->edge_latency_ns[k];
        loss[(size_t)i * U + j] = g->edge_loss[k];
      }
  } else {
    for (uint32_t i = 0; i < U; i++)
      if (self_count[uidx[i]] != 1)
        return set_error(ctx, SGN_EINVAL, edge_msg(self_count[uidx[i]], uidx[i], uidx[i]));
    const uint32_t nb = (V + FW_T - 1) / FW_T;
    const uint32_t Vp = nb * FW_T;
    const size_t lds = (size_t)Vp * 12 + 16;
    if (lds > 160 * 1024)
      return set_error(ctx, SGN_ERANGE, "graph too large for the LDS loss pass (V > 13632)");
    // directed arcs (undirected edges both ways), self-loops excluded; u | v << 16 packed
    // (V <= 13632 here: the LDS bound above)
    std::vector<uint32_t> auv;
    std::vector<uint64_t> al;
    std::vector<float> ap;
    auv.reserve(2 * (size_t)E);
    for (uint32_t k = 0; k < E; k++) {
      if (es[k] == ed[k]) continue;
      auv.push_back(es[k] | (ed[k] << 16)); al.push_back(g->edge_latency_ns[k]); ap.push_back(g->edge_loss[k]);
      if (!g->directed) {
        auv.push_back(ed[k] | (es[k] << 16)); al.push_back(g->edge_latency_ns[k]); ap.push_back(g->edge_loss[k]);
      }
    }
    const uint32_t E2 = (uint32_t)auv.size();
    // dense graphs (the multi-source loss sweep): the arcs in tail order, with CSR offsets
    // (every consumer of the arc list is order-free: relaxation and the loss folds reach the same
    // fixed point); SGN_APSP_SWEEP_ARCS=1 keeps the edge order and the per-arc sweep (A/B)
    const bool csr = E2 >= 32ull * Vp && !getenv("SGN_APSP_SWEEP_ARCS");
    std::vector<uint32_t> rowptr;
    if (csr) {
      rowptr.assign(V + 1, 0);
      for (uint32_t e = 0; e < E2; e++) rowptr[(auv[e] & 0xFFFFu) + 1]++;
      for (uint32_t u = 0; u < V; u++) rowptr[u + 1] += rowptr[u];
      std::vector<uint32_t> pos(rowptr.begin(), rowptr.end() - 1), auv2(E2);
      std::vector<uint64_t> al2(E2);
      std::vector<float> ap2(E2);
      for (uint32_t e = 0; e < E2; e++) {
        const uint32_t k = pos[auv[e] & 0xFFFFu]++;
        auv2[k] = auv[e];
        al2[k] = al[e];
        ap2[k] = ap[e];
      }
      auv.swap(auv2);
      al.swap(al2);
      ap.swap(ap2);
    }
    std::vector<uint64_t> sl(U);
    std::vector<float> sp(U);
    for (uint32_t i = 0; i < U; i++) {
      sl[i] = g->edge_latency_ns[self_edge[uidx[i]]];
      sp[i] = g->edge_loss[self_edge[uidx[i]]];
    }
    // tight-arc list capacity: 4 per node (a source's tight arcs are its shortest-path DAG:
    // about one per node plus ties), at least 4 k, within what LDS holds next to the rows
    const uint32_t cap = (uint32_t)std::min<size_t>(std::max<size_t>(4096, 4 * (size_t)Vp),
                                                    (160 * 1024 - lds - 16) / 8);
    const size_t lds2 = lds + (size_t)cap * 8 + 16;
    DevBuf dD, deu, dev, del, dauv, dal, dap, dus, dL, dit, dsl, dsp, dres, drowres, drp;
    int rc;
    if (csr && (rc = upload(ctx, drp, rowptr.data(), V + 1))) return rc;
    if ((rc = upload(ctx, deu, es.data(), E)) || (rc = upload(ctx, dev, ed.data(), E)) ||
        (rc = upload(ctx, del, g->edge_latency_ns, E)) || (rc = upload(ctx, dauv, auv.data(), E2)) ||
        (rc = upload(ctx, dal, al.data(), E2)) || (rc = upload(ctx, dap, ap.data(), E2)) ||
        (rc = upload(ctx, dus, uidx.data(), U)) || (rc = upload(ctx, dsl, sl.data(), U)) ||
        (rc = upload(ctx, dsp, sp.data(), U)))
      return rc;
    const unsigned long long res0[3] = {~0ULL, ~0ULL, 0ULL};
    if ((rc = upload(ctx, dres, res0, 3))) return rc;
    SGN_HIP(ctx, hipMalloc(&dD.p, (size_t)Vp * Vp * 8));
    SGN_HIP(ctx, hipMalloc(&dL.p, (size_t)U * Vp * 4));
    SGN_HIP(ctx, hipMalloc(&dit.p, (size_t)U * 4));
    SGN_HIP(ctx, hipMalloc(&drowres.p, (size_t)U * 3 * 8));
    // the engine's table (replaces any previous one)
    if (ctx->d_lat) hipFree(ctx->d_lat);
    if (ctx->d_loss) hipFree(ctx->d_loss);
    ctx->d_lat = nullptr;
    ctx->d_loss = nullptr;
    ctx->routes_ready = false;
    SGN_HIP(ctx, hipMalloc(&ctx->d_lat, (size_t)U * U * 8));
    SGN_HIP(ctx, hipMalloc(&ctx->d_loss, (size_t)U * U * 4));
    hipStream_t st = ctx->stream;
    uint64_t* D = (uint64_t*)dD.p;
    uint64_t max_edge = 0;
    for (uint32_t k = 0; k < E; k++)
      if (es[k] != ed[k]) max_edge = std::max(max_edge, g->edge_latency_ns[k]);
    // latency phase: sparse graphs relax per source (Bellman-Ford in LDS, u64, exact);
    // otherwise u32 min-plus squaring when edges fit (exact unless a used pair ends at
    // 2^32 - 1 or above: then the u64 Floyd-Warshall redoes it), else Floyd-Warshall
    const bool bf = E2 < 32ull * Vp && Vp * 8 + 16 <= 64 * 1024 && !getenv("SGN_APSP_FW") &&
                    !getenv("SGN_APSP_SQ");
    bool fast = !bf && max_edge < SQ_INF && !getenv("SGN_APSP_FW");
    DevBuf dD32, dflag;
    const uint32_t max_pass = 34;
    if (fast) {
      SGN_HIP(ctx, hipMalloc(&dD32.p, (size_t)Vp * Vp * 4));
      SGN_HIP(ctx, hipMalloc(&dflag.p, (max_pass + 3) * 4));  // + sq_run's timeout word, barrier counter, the
                                                              // fused pass's change word
    }
    // the loss phase's form and buffers (allocated here, outside the timed build)
    const uint32_t capg = std::max<uint32_t>(4096, 4 * Vp);
    const size_t lds_fold = (size_t)Vp * 4 + (size_t)cap * 8 + 16;
    // 0 one-source kernel, 1 multi-source arc sweep (not for sparse graphs: their arc list is
    // re-read from L2 cheaply source by source)
    int lform = fast && !getenv("SGN_APSP_LOSS1") && lds_fold <= 160 * 1024 && E2 >= 32ull * Vp ? 1 : 0;
    int kS = 0;  // sources per sweep workgroup: the largest whose rows fit its LDS
    if (lform == 1) {
      // (16 sources per workgroup in tail order share each arc's loads and addressing over twice
      // the sources, but measured slower at config C's V = 1000: 179 vs 132 us, its 64 KB of rows
      // leave 2 workgroups per CU; SGN_APSP_SWEEP_S=16 selects it, A/B)
      const int smax = getenv("SGN_APSP_SWEEP_S") ? atoi(getenv("SGN_APSP_SWEEP_S")) : 8;
      for (int k : {16, 8, 4}) {
        const size_t b = (size_t)Vp * k * 4 + (csr ? 8 * SWEEP_HCAP * 4 : 0);  // rows (+ hit lists)
        if (b > 160 * 1024 || k > smax || (k == 16 && !csr)) continue;
        const void* f = csr ? (k == 16 ? (const void*)loss_sweep_csr<16>
                               : k == 8 ? (const void*)loss_sweep_csr<8> : (const void*)loss_sweep_csr<4>)
                            : (k == 8 ? (const void*)loss_sweep<8> : (const void*)loss_sweep<4>);
        if (b <= 64 * 1024 ||
            hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)b) == hipSuccess) {
          kS = k;
          break;
        }
        (void)hipGetLastError();
      }
      if (!kS) lform = 0;
    }
    const size_t lds_sw = (size_t)Vp * kS * 4 + (csr ? 8 * SWEEP_HCAP * 4 : 0);
    // the dense form of the sweep (loss_sweep_dense): at least half of all arcs present, at most
    // one arc per (tail, head) — the dense index matrix holds one — and Vp <= 8192 (two Vp^2
    // u32 matrices); SGN_APSP_DENSE=0 keeps the CSR sweep (A/B), SGN_APSP_DENSE_S picks the
    // sources per workgroup
    bool dense = false;
    int kDS = 16, kDH = 2;  // sources per workgroup, heads per lane
    if (lform == 1 && csr && Vp <= 8192 && 2ull * E2 >= (uint64_t)V * (V - 1) &&
        !(getenv("SGN_APSP_DENSE") && atoi(getenv("SGN_APSP_DENSE")) == 0)) {
      std::vector<uint32_t> seen(V, ~0u);
      dense = true;
      for (uint32_t u = 0; u < V && dense; u++)
        for (uint32_t e = rowptr[u]; e < rowptr[u + 1]; e++) {
          const uint32_t v = auv[e] >> 16;
          if (seen[v] == u) {
            dense = false;
            break;
          }
          seen[v] = u;
        }
      if (getenv("SGN_APSP_DENSE_S")) kDS = atoi(getenv("SGN_APSP_DENSE_S")) == 32 ? 32 : 16;
      if (getenv("SGN_APSP_DENSE_H")) kDH = atoi(getenv("SGN_APSP_DENSE_H")) == 1 ? 1 : 2;
      if (kDS == 32) kDH = 1;
    }
    const uint32_t Upd = (U + kDS - 1) / kDS * kDS;  // NDT's row length
    // the fused form (loss_sweep_dense<.., true> before the squaring): complete graphs whose
    // latencies stay below 2^29 ns (signed sums), one shard; SGN_APSP_FUSED=0 turns it off (A/B)
    const bool fused_ok = dense && kDS == 16 && kDH == 2 && E2 == (uint64_t)V * (V - 1) && max_edge < (1ull << 29) &&
                          !(getenv("SGN_APSP_FUSED") && atoi(getenv("SGN_APSP_FUSED")) == 0);
    bool fused = false;
    DevBuf dtc, dtl, dal32, dNL32, dEI, dNDT;
    if (dense) {
      SGN_HIP(ctx, hipMalloc(&dNL32.p, (size_t)Vp * Vp * 4));
      SGN_HIP(ctx, hipMalloc(&dEI.p, (size_t)Vp * Vp * 4));
      SGN_HIP(ctx, hipMalloc(&dNDT.p, (size_t)Vp * Upd * 4));
    }
    if (lform) {
      SGN_HIP(ctx, hipMalloc(&dtc.p, (size_t)U * 4));
      SGN_HIP(ctx, hipMalloc(&dtl.p, (size_t)U * capg * 4));
    }
    if (lform == 1) {
      std::vector<uint32_t> al32(E2);
      for (uint32_t e = 0; e < E2; e++) al32[e] = al[e] >= SQ_INF ? SQ_INF : (uint32_t)al[e];
      if ((rc = upload(ctx, dal32, al32.data(), E2))) return rc;
    }
    DevBuf dbfit;
    if (bf) SGN_HIP(ctx, hipMalloc(&dbfit.p, (size_t)U * 4));
    // Sharded build. With an RCCL communicator (sgn_comm_init before the build)
    // every shard computes a contiguous block of the used sources' rows — and in the squaring
    // form a block of row tiles per pass, exchanged after each pass — and the table's blocks are
    // exchanged at the end, so every shard holds the whole table; all shards must call
    // sgn_routes_build with the same graph. The u64 Floyd-Warshall (a chain of pivot steps)
    // runs whole on every shard. The split is used from kApspShardMinU used nodes on: below it
    // the whole build takes ~1 ms on one GPU and the per-pass and final exchanges cost more
    // than the share of work they save (replicated is acceptable at V <= 2k);
    // SGN_APSP_SHARDED=1 forces the split, SGN_APSP_REPLICATED=1 forbids it.
    // SGN_APSP_VSHARDS=n without a communicator (a test hook): one process runs the n blocks
    // in turn over one buffer, which checks the block arithmetic on one GPU.
    uint32_t nsh = 1, me = 0;
    bool rccl = false;
    constexpr uint32_t kApspShardMinU = 2048;
    if (ctx->comm && ctx->nranks > 1 && !getenv("SGN_APSP_REPLICATED") &&
        (U >= kApspShardMinU || getenv("SGN_APSP_SHARDED"))) {
      nsh = ctx->nranks;
      me = ctx->rank;
      rccl = true;
    } else if (const char* v = getenv("SGN_APSP_VSHARDS")) {
      nsh = (uint32_t)std::max(1, std::min(atoi(v), 1024));
    }
    const uint32_t sh_first = rccl ? me : 0, sh_last = rccl ? me + 1 : nsh;
    std::vector<uint64_t> soff(nsh + 1), toff(nsh + 1);  // used-source blocks, row-tile blocks
    for (uint32_t r = 0; r <= nsh; r++) {
      soff[r] = (uint64_t)U * r / nsh;
      toff[r] = (uint64_t)nb * r / nsh;
    }
    tm.shards = nsh;
    tm.shard_sources = (uint32_t)(soff[sh_last] - soff[sh_first]);
    // one shard: all squaring passes in one launch (sq_run), unless its barrier ever timed out
    // (the grid not resident: another context holds CUs) or SGN_APSP_SQ_PASSES=1 (A/B)
    bool sq_one = nsh == 1 && !getenv("SGN_APSP_SQ_PASSES");
    uint32_t n_cu = 0;
    {
      int c = 0;
      if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || c <= 0) c = 0;
      n_cu = (uint32_t)c;
      if (!n_cu || hipFuncSetAttribute((const void*)sq_run, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)SQR_LDS) != hipSuccess) {
        (void)hipGetLastError();
        sq_one = false;
      }
    }
    // the dense sweep over used sources [s0, s0 + ns): NDT, the sources' own out-arcs, the sweep
    // (kf: the fused form; gate: run only if the fused pass found a change; chg: its change word)
    auto dense_block = [&](uint32_t s0, uint32_t ns, bool kf, const uint32_t* gate, uint32_t* chg, bool zero,
                           bool ndt_ready) {
      const uint32_t* d32 = (const uint32_t*)dD32.p;
      const uint32_t* us = (const uint32_t*)dus.p + s0;
      uint32_t* tcs = (uint32_t*)dtc.p + s0;
      uint32_t* tls = (uint32_t*)dtl.p + (size_t)s0 * capg;
      const uint32_t gx = (ns + kDS - 1) / kDS, gy = (Vp + 256 * kDH - 1) / (256 * kDH);
      const uint32_t wg = getenv("SGN_APSP_DENSE_WG") ? (uint32_t)atoi(getenv("SGN_APSP_DENSE_WG")) : 4096u;
      const uint32_t gz = std::max<uint32_t>(1, std::min<uint32_t>(std::max<uint32_t>(1, V / 16), (wg + gx * gy - 1) / (gx * gy)));
      if (!ndt_ready)
        hipLaunchKernelGGL(kf ? ndt_build<true> : ndt_build<false>, dim3((Upd + 63) / 64, (Vp + 63) / 64), dim3(256), 0,
                           st, d32, Vp, us, ns, (uint32_t*)dNDT.p, Upd, gate, zero ? tcs : nullptr);
      auto f = kf ? loss_sweep_dense<16, 2, true>
                  : kDS == 16 ? (kDH == 2 ? loss_sweep_dense<16, 2, false> : loss_sweep_dense<16, 1, false>)
                              : loss_sweep_dense<32, 1, false>;
      hipLaunchKernelGGL(f, dim3(gx, gy, gz), dim3(256), 0, st, d32, Vp, us, ns, V, (const uint32_t*)dNDT.p, Upd,
                         (const uint32_t*)dNL32.p, (const uint32_t*)dEI.p, capg, tcs, tls, gate, chg);
    };
    bool wide = true;  // D (u64) holds the distances; false: only D32 (u32 squaring)
  latency_phase:
    SGN_HIP(ctx, hipEventRecord(e0, st));
    wide = true;
    if (bf) {  // per source: a shard's block needs no exchange until the table
      for (uint32_t r = sh_first; r < sh_last; r++) {
        const uint32_t s0 = (uint32_t)soff[r], ns = (uint32_t)(soff[r + 1] - s0);
        if (ns)
          hipLaunchKernelGGL(bf_pass, dim3(ns), dim3(512), (size_t)Vp * 8 + 16, st, D, Vp,
                             (const uint32_t*)dus.p + s0, (const uint32_t*)dauv.p, (const uint64_t*)dal.p, E2,
                             (uint32_t*)dbfit.p + s0);
      }
    } else if (fast) {
      uint32_t* D32 = (uint32_t*)dD32.p;
      if (!csr) SGN_HIP(ctx, hipMemsetAsync(dflag.p, 0, (max_pass + 3) * 4, st));  // (sq_rows clears them)
      // the fused form: the tight sweep on the direct arcs, which is also the first squaring pass
      // for the used sources (sq_run returns at once if it found no change); sq_rows writes the
      // sweep's negated latency and arc-index matrices beside the rows
      fused = fused_ok && csr && sq_one && nsh == 1;
      uint32_t* chgw = (uint32_t*)dflag.p + max_pass + 2;
      if (csr) {
        hipLaunchKernelGGL(sq_rows, dim3(Vp), dim3(256), (size_t)Vp * 4, st, D32, Vp, V, (const uint32_t*)drp.p,
                           (const uint32_t*)dauv.p, (const uint64_t*)dal.p, fused ? (uint32_t*)dNL32.p : nullptr,
                           fused ? (uint32_t*)dEI.p : nullptr, fused && !g->directed ? (uint32_t*)dNDT.p : nullptr,
                           (const uint32_t*)dus.p, U, Upd, (uint32_t*)dflag.p, max_pass + 3,
                           fused ? (uint32_t*)dtc.p : nullptr, U);
      } else {
        hipLaunchKernelGGL(sq_init, dim3(2048), dim3(256), 0, st, D32, Vp);
        hipLaunchKernelGGL(sq_edges, dim3(std::max<uint32_t>(1, std::min<uint32_t>(4096, (E + 255) / 256))), dim3(256), 0,
                           st, D32, Vp, (const uint32_t*)deu.p, (const uint32_t*)dev.p, (const uint64_t*)del.p, E,
                           (int)g->directed);
      }
      if (fused) {  // (sq_rows cleared the tight counts)
        dense_block(0, U, true, nullptr, chgw, false, !g->directed);
      }
      // ceil(log2 Vp) passes cover every simple path; one more confirms the fixed point
      uint32_t passes = 1;
      while ((1u << (passes - 1)) < Vp) passes++;
      passes = std::min(passes + 1, max_pass);
      if (sq_one)
        hipLaunchKernelGGL(sq_run, dim3(std::min<uint32_t>(nb * nb, n_cu)), dim3(1024), SQR_LDS, st, D32, Vp,
                           (uint32_t*)dflag.p, passes, (uint32_t*)dflag.p + max_pass, (uint32_t*)dflag.p + max_pass + 1,
                           (const uint32_t*)(fused ? chgw : nullptr));
      for (uint32_t it = 0; it < passes && !sq_one; it++) {
        for (uint32_t r = sh_first; r < sh_last; r++) {
          const uint32_t t0 = (uint32_t)toff[r], nt = (uint32_t)(toff[r + 1] - t0);
          if (nt)
            hipLaunchKernelGGL(sq_pass, dim3(nb, nt), dim3(256), 0, st, D32, Vp, (uint32_t*)dflag.p, (int)it, t0);
        }
        if (rccl) {  // every shard's new rows to all, and whether any shard changed a row
          if ((rc = comm_bcast_blocks(ctx, D32, (size_t)SQ_T * Vp * 4, toff)) ||
              (rc = comm_allreduce_max_u32(ctx, (uint32_t*)dflag.p + it, 1)))
            return rc;
          uint32_t f = 0;
          SGN_HIP(ctx, hipMemcpyAsync(&f, (uint32_t*)dflag.p + it, 4, hipMemcpyDeviceToHost, st));
          SGN_HIP(ctx, hipStreamSynchronize(st));
          if (!f) break;
        }
      }
      wide = false;  // (the tight forms and the extraction read the u32 matrix; sq_widen only for
                     // the one-source loss pass)
    } else {
      hipLaunchKernelGGL(fw_init, dim3(2048), dim3(256), 0, st, D, Vp);
      hipLaunchKernelGGL(fw_edges, dim3(std::max<uint32_t>(1, std::min<uint32_t>(4096, (E + 255) / 256))), dim3(256), 0, st,
                         D, Vp, (const uint32_t*)deu.p, (const uint32_t*)dev.p, (const uint64_t*)del.p, E,
                         (int)g->directed);
      for (uint32_t kb = 0; kb < nb; kb++) {
        hipLaunchKernelGGL(fw_phase1, dim3(1), dim3(1024), 0, st, D, Vp, (int)kb);
        if (nb > 1) {
          hipLaunchKernelGGL(fw_phase2, dim3(2 * (nb - 1)), dim3(1024), 0, st, D, Vp, (int)kb, (int)nb);
          hipLaunchKernelGGL(fw_phase3, dim3((nb - 1) * (nb - 1)), dim3(256), 0, st, D, Vp, (int)kb, (int)nb);
        }
      }
    }
    SGN_HIP(ctx, hipGetLastError());
    SGN_HIP(ctx, hipEventRecord(e1, st));
    // loss phase (u32 form): tight arcs of kS used sources per arc load (dense and mid-density
    // graphs), then a per-source fold in LDS. Sparse graphs, the u64 form, a list overflow, or
    // SGN_APSP_LOSS1 take the one-source kernel.
    int form = lform;
  loss_phase:
    if (!form && !wide) {  // the one-source loss pass reads the u64 matrix
      hipLaunchKernelGGL(sq_widen, dim3(2048), dim3(256), 0, st, (const uint32_t*)dD32.p, D, (uint64_t)Vp * Vp);
      wide = true;
    }
    if (form) {
      const uint32_t* gate = fused ? (const uint32_t*)dflag.p + max_pass + 2 : nullptr;
      // (the fused pass's lists stand unless it found a change; then ndt_build clears the counts)
      if (!fused) SGN_HIP(ctx, hipMemsetAsync(dtc.p, 0, (size_t)U * 4, st));
      if (dense && !fused) {
        SGN_HIP(ctx, hipMemsetD32Async((hipDeviceptr_t)dNL32.p, 1, (size_t)Vp * Vp, st));  // (1 = -SQ_INF: no arc)
        hipLaunchKernelGGL(dense_arcs, dim3(std::max<uint32_t>(1, std::min<uint32_t>(4096, (E2 + 255) / 256))),
                           dim3(256), 0, st, (const uint32_t*)dauv.p, (const uint32_t*)dal32.p, E2, Vp,
                           (uint32_t*)dNL32.p, (uint32_t*)dEI.p);
      }
      for (uint32_t r = sh_first; r < sh_last; r++) {
        const uint32_t s0 = (uint32_t)soff[r], ns = (uint32_t)(soff[r + 1] - s0);
        if (!ns) continue;
        const uint32_t groups = (ns + kS - 1) / kS;
        const uint32_t parts = std::max<uint32_t>(1, std::min<uint32_t>(64, (2048 + groups - 1) / groups));
        const dim3 grid(groups, std::min<uint32_t>(parts, std::max<uint32_t>(1, E2 / 4096)));
        const uint32_t* d32 = (const uint32_t*)dD32.p;
        const uint32_t* a32 = (const uint32_t*)dal32.p;
        const uint32_t* us = (const uint32_t*)dus.p + s0;
        uint32_t* tcs = (uint32_t*)dtc.p + s0;
        uint32_t* tls = (uint32_t*)dtl.p + (size_t)s0 * capg;
        if (dense) {
          dense_block(s0, ns, fused, gate, nullptr, fused, false);
        } else if (csr && kS == 16)
          hipLaunchKernelGGL(loss_sweep_csr<16>, grid, dim3(512), lds_sw, st, d32, Vp, us, ns, V,
                             (const uint32_t*)drp.p, (const uint32_t*)dauv.p, a32, capg, tcs, tls);
        else if (csr && kS == 8)
          hipLaunchKernelGGL(loss_sweep_csr<8>, grid, dim3(512), lds_sw, st, d32, Vp, us, ns, V,
                             (const uint32_t*)drp.p, (const uint32_t*)dauv.p, a32, capg, tcs, tls);
        else if (csr)
          hipLaunchKernelGGL(loss_sweep_csr<4>, grid, dim3(512), lds_sw, st, d32, Vp, us, ns, V,
                             (const uint32_t*)drp.p, (const uint32_t*)dauv.p, a32, capg, tcs, tls);
        else if (kS == 8)
          hipLaunchKernelGGL(loss_sweep<8>, grid, dim3(512), lds_sw, st, d32, Vp, us, ns,
                             (const uint32_t*)dauv.p, a32, E2, capg, tcs, tls);
        else
          hipLaunchKernelGGL(loss_sweep<4>, grid, dim3(512), lds_sw, st, d32, Vp, us, ns,
                             (const uint32_t*)dauv.p, a32, E2, capg, tcs, tls);
        hipLaunchKernelGGL(loss_fold, dim3(ns), dim3(256), lds_fold, st, Vp, us, (const uint32_t*)dauv.p,
                           (const float*)dap.p, (const uint32_t*)tcs, (const uint32_t*)tls, capg, cap,
                           (float*)dL.p + (size_t)s0 * Vp, (uint32_t*)dit.p + s0);
      }
      SGN_HIP(ctx, hipGetLastError());
      SGN_HIP(ctx, hipEventRecord(e2, st));
    } else {
      for (uint32_t r = sh_first; r < sh_last; r++) {
        const uint32_t s0 = (uint32_t)soff[r], ns = (uint32_t)(soff[r + 1] - s0);
        if (ns)
          hipLaunchKernelGGL(loss_pass, dim3(ns), dim3(512), lds2, st, D, Vp, (const uint32_t*)dus.p + s0,
                             (const uint32_t*)dauv.p, (const uint64_t*)dal.p, (const float*)dap.p, E2, cap,
                             (float*)dL.p + (size_t)s0 * Vp, (uint32_t*)dit.p + s0);
      }
      SGN_HIP(ctx, hipGetLastError());
      SGN_HIP(ctx, hipEventRecord(e2, st));
    }
    // a source with more tight pairs than its list holds: the phase is redone the one-source
    // way. One shard checks after the extraction (no host round trip inside the timed build:
    // ~40 us at config C); sharded builds check first, so every shard enters the table's
    // exchange below exactly once.
    std::vector<uint32_t> tc(form ? U : 0);
    auto tight_over = [&]() {
      for (uint32_t x : tc)
        if (x > capg) return true;
      return false;
    };
    if (form && rccl) {
      SGN_HIP(ctx, hipMemcpyAsync(tc.data(), dtc.p, (size_t)U * 4, hipMemcpyDeviceToHost, st));
      SGN_HIP(ctx, hipStreamSynchronize(st));
      if (tight_over()) {
        form = 0;
        goto loss_phase;
      }
    }
    for (uint32_t r = sh_first; r < sh_last; r++)
      if (soff[r + 1] > soff[r]) {
        hipLaunchKernelGGL(wide ? extract<false> : extract<true>, dim3((uint32_t)(soff[r + 1] - soff[r])), dim3(256), 0, st,
                           wide ? (const void*)D : (const void*)dD32.p, Vp,
                           (const float*)dL.p, (const uint32_t*)dus.p, U, (const uint64_t*)dsl.p,
                           (const float*)dsp.p, ctx->d_lat, ctx->d_loss, (uint64_t*)drowres.p, (uint32_t)soff[r]);
        hipLaunchKernelGGL(extract_fold, dim3(1), dim3(256), 0, st, (const uint64_t*)drowres.p,
                           (uint32_t)soff[r], (uint32_t)soff[r + 1], (unsigned long long*)dres.p);
      }
    SGN_HIP(ctx, hipGetLastError());
    if (rccl) {  // the table's blocks to every shard; res = {min bad pair, min, max} over shards
      if ((rc = comm_bcast_blocks(ctx, ctx->d_lat, (size_t)U * 8, soff)) ||
          (rc = comm_bcast_blocks(ctx, ctx->d_loss, (size_t)U * 4, soff)) ||
          (rc = comm_allreduce_minmax(ctx, (uint64_t*)dres.p, 2, 1)))
        return rc;
    }
    unsigned long long res[3];
    SGN_HIP(ctx, hipMemcpyAsync(res, dres.p, sizeof(res), hipMemcpyDeviceToHost, st));
    SGN_HIP(ctx, hipEventRecord(e3, st));
    if (form && !rccl) SGN_HIP(ctx, hipMemcpyAsync(tc.data(), dtc.p, (size_t)U * 4, hipMemcpyDeviceToHost, st));
    std::vector<uint32_t> its(U);
    SGN_HIP(ctx, hipMemcpyAsync(its.data(), dit.p, (size_t)U * 4, hipMemcpyDeviceToHost, st));
    SGN_HIP(ctx, hipStreamSynchronize(st));
    if (form && !rccl && tight_over()) {
      form = 0;
      SGN_HIP(ctx, hipMemcpy(dres.p, res0, sizeof(res0), hipMemcpyHostToDevice));
      goto loss_phase;
    }
    tm.loss_multi = form ? (uint32_t)(dense ? kDS : kS) : 0u;
    tm.loss_dense = form && dense ? 1u : 0u;
    float ms_fw = 0, ms_loss = 0, ms_total = 0;
    hipEventElapsedTime(&ms_fw, e0, e1);
    hipEventElapsedTime(&ms_loss, e1, e2);
    hipEventElapsedTime(&ms_total, e0, e3);
    tm.latency_ms = ms_fw;
    tm.loss_ms = ms_loss;
    tm.total_ms = ms_total;
    uint32_t mi = 0, n_global = 0;
    for (uint32_t v : its) {
      mi = std::max(mi, v & 0x7FFFFFFFu);
      n_global += v >> 31;
    }
    tm.loss_iters = mi;
    tm.n_tight_edges = E2;
    if (n_global)
      fprintf(stderr, "libsgn: %u sources had more tight arcs than the LDS list (%u): global sweeps\n",
              n_global, cap);
    uint32_t sq_passes = 0;
    if (fast) {
      std::vector<uint32_t> fl(max_pass + 3);
      SGN_HIP(ctx, hipMemcpy(fl.data(), dflag.p, (max_pass + 3) * 4, hipMemcpyDeviceToHost));
      tm.loss_fused = fused && fl[max_pass + 2] == 0 ? 1u : 0u;
      if (sq_one && fl[max_pass]) {  // sq_run's grid barrier timed out: redo with sq_pass launches
        fprintf(stderr, "libsgn: APSP squaring grid not resident; one launch per pass\n");
        sq_one = false;
        SGN_HIP(ctx, hipMemcpy(dres.p, res0, sizeof(res0), hipMemcpyHostToDevice));
        goto latency_phase;
      }
      while (sq_passes < max_pass && fl[sq_passes]) sq_passes++;
      sq_passes++;  // the pass that found the fixed point
    }
    if (res[0] != ~0ULL && fast) {
      // a used pair without a finite u32 path: disconnected, or a path of 2^32 - 1 ns or more;
      // the u64 Floyd-Warshall decides
      fast = false;
      lform = 0;  // the tight forms read the u32 matrix
      SGN_HIP(ctx, hipMemcpy(dres.p, res0, sizeof(res0), hipMemcpyHostToDevice));
      goto latency_phase;
    }
    tm.tile = bf ? 0u : fast ? (uint32_t)SQ_T : (uint32_t)FW_T;
    tm.latency_passes = fast ? sq_passes : nb;
    tm.latency_u64 = fast ? 0u : 1u;
    tm.latency_bf = bf ? 1u : 0u;
    if (bf) {
      std::vector<uint32_t> bi(U);
      SGN_HIP(ctx, hipMemcpy(bi.data(), dbfit.p, (size_t)U * 4, hipMemcpyDeviceToHost));
      tm.latency_passes = *std::max_element(bi.begin(), bi.end());
    }
    if (res[0] != ~0ULL) {
      const uint64_t i = res[0] / U, j = res[0] % U;
      return set_error(ctx, SGN_EINVAL, "used nodes " + std::to_string(used[i]) + " -> " +
                                            std::to_string(used[j]) + " are not connected");
    }
    ctx->lat_min = res[1];
    ctx->lat_max = res[2];
    ctx->h_lat.clear();
    ctx->h_loss.clear();
    ctx->h_routes = false;  // host mirror made on demand (sgn_route_get & co.)
    ctx->U = U;
    ctx->used_ids.assign(used, used + U);
    ctx->rt_timing = tm;
    ctx->routes_ready = true;
    ctx->hosts_ready = false;  // hosts map onto used nodes: re-register
    return 0;
  }
  // direct paths (use_shortest_path: false): the host table, uploaded for the engine
  ctx->lat_min = *std::min_element(lat.begin(), lat.end());
  ctx->lat_max = *std::max_element(lat.begin(), lat.end());
  ctx->h_routes = true;
  if (ctx->d_lat) hipFree(ctx->d_lat);
  if (ctx->d_loss) hipFree(ctx->d_loss);
  ctx->d_lat = nullptr;
  ctx->d_loss = nullptr;
  SGN_HIP(ctx, hipMalloc(&ctx->d_lat, (size_t)U * U * 8));
  SGN_HIP(ctx, hipMalloc(&ctx->d_loss, (size_t)U * U * 4));
  SGN_HIP(ctx, hipMemcpy(ctx->d_lat, lat.data(), (size_t)U * U * 8, hipMemcpyHostToDevice));
  SGN_HIP(ctx, hipMemcpy(ctx->d_loss, loss.data(), (size_t)U * U * 4, hipMemcpyHostToDevice));
  ctx->U = U;
  ctx->used_ids.assign(used, used + U);
  ctx->h_lat.swap(lat);
  ctx->h_loss.swap(loss);
  ctx->rt_timing = tm;
  ctx->routes_ready = true;
  ctx->hosts_ready = false;  // hosts map onto used nodes: re-register
  return 0;
}

uint64_t sgn::layout_sig_routes() { return kLayoutSig; }
