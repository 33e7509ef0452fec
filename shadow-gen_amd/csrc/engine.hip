// engine.hip — the per-round packet path of Shadow on gfx950.
//
// One wave of 64 lanes per host group (64 consecutive hosts, lane = host). A simulation
// round (core/manager.rs:541-656) for a group is exec_group():
//   gather   the group's calendar slabs of the window's buckets -> LDS (device-scope loads);
//            runs due later in the last bucket move to the spare slab set
//   order    counting sort of the due event runs by destination lane, rank sort inside each
//            lane's segment by (time, src host, src event id) (core/work/event.rs:84-183)
//   execute  every lane runs Host::execute (host/host.rs:762-830) over its segment merged
//            with its three local event slots: router/CoDel, relays and token buckets,
//            Worker::send_packet (loss draws from the host's Xoshiro256++), emitting event
//            runs into the destinations' calendar slabs
//   edge     minimum next event, bucket bookkeeping, Controller::manager_finished_current_
//            round (controller.rs:88-112) — run by the last wave to arrive
// Kernels: k_rounds (single shard, persistent: up to 128 rounds per launch with an atomic
// grid barrier per round), k_execute (one round per launch: sgn_round, multi-shard) with
// k_import after the RCCL exchange (comm.cpp; its last block advances the window), k_inject
// (sgn_submit), k_rng (sgn_rng_*). The window lives in device memory (Ctrl), so rounds run
// back to back without a host round trip.
//
// Bit-exactness notes: all time/byte/event-id arithmetic is u64 integer; the only floating
// point is (a) reliability = (f64)(1.0f - loss) vs the f64 draw (x >> 11) * 2^-53
// (core/worker.rs:363-371, exact on any IEEE device), and (b) the CoDel control law
// round(1e8 / sqrt(count)) in f64 (router/codel_queue.rs:285-298), which relies on
// correctly rounded f64 sqrt/div (checked on the GPU by tests/test_gpu_parity.py).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <tuple>

#include "sgn_internal.h"
#include "sgn_workload.h"

// Cost experiments only (tools/build_exp.sh builds them as separate libraries; results are
// not parity-valid): digests off, loss draws off.
#ifdef SGN_EXP_NODIGEST
#define sgn_drun_add_seq(...) ((void)0)
#define sgn_drun_add_same(...) ((void)0)
#define sgn_drun_flush_seq(...) ((void)0)
#define sgn_drun_flush_same(...) ((void)0)
#define sgn_digest3(h, ...) (h)
#endif

// Diagnostic build (libsgn_diag.so, -DSGN_DIAG): per-lane counts of the work kinds that
// carry dependent global-memory round trips, reported through sgn_debug_stamps.
#ifdef SGN_DIAG
#define DG(i) ((void)0)  // per-lane work counts: off (registers; see DGT sections)
#define DGT_BEGIN(v) const uint64_t v = __builtin_amdgcn_s_memtime()
// wave time in a section: added by the section's lowest active lane only (the lanes in a
// section entered it together), so the wave's sum over lanes is the section's wave time
#define DGT_END(i, v)                                                                  \
  do {                                                                                 \
    const uint64_t dgt_t = __builtin_amdgcn_s_memtime();                               \
    if ((uint32_t)(__ffsll((long long)__ballot(1)) - 1) == (threadIdx.x & 63))         \
      dgt[i] += (uint32_t)(dgt_t - (v));                                               \
  } while (0)
#else
#define DG(i) ((void)0)
#define DGT_BEGIN(v) ((void)0)
#define DGT_END(i, v) ((void)0)
#endif
enum { DG_RO = 0, DG_RI, DG_APP, DG_BATCH, DG_HDLOAD, DG_FQLOAD, DG_RMISS, DG_POPRUN, DG_N };
// diagnostic timers: cycles while this lane was inside ...
enum { DGT_SEND = 0, DGT_FWDOUT, DGT_FWDIN, DGT_POP, DGT_APP, DGT_LOAD,
       DGT_HDLD, DGT_FHLD, DGT_RTLD, DGT_SVLD, DGT_SLAB,
       DGT_DRAWS,   // (counts, not cycles) loss draws of this lane's trains
       DGT_RENTRY,  // ... and the wave's entries into the draw loop (its lowest lane counts)
       DGT_LLANE,   // (counts) this lane's entries with a long train (more than kTrainWait draws)
       DGT_LENTRY,  // ... and the wave's entries in which some lane draws a long train
       DGT_CQALLOC, DGT_CQFREE, DGT_TBRM, DGT_DELIV,  // CoDel page alloc / free, token bucket, delivery
       DGT_N };
#ifdef SGN_DIAG
#define DGT_WAIT() asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory")
#else
#define DGT_WAIT() ((void)0)
#endif

namespace sgn {

enum : uint32_t { RELAY_IDLE = 0, RELAY_PENDING = 1, RELAY_FORWARDING = 2 };

constexpr uint64_t CODEL_TARGET = 10000000ULL;      // codel_queue.rs:23
constexpr uint64_t CODEL_INTERVAL = 100000000ULL;   // codel_queue.rs:28
constexpr uint64_t SIMTIME_MAX = 17500059273709551614ULL;

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) {
  return (x << k) | (x >> (64 - k));
}
// xoshiro256++'s operations on 32-bit halves for gfx950's VALU: a 64-bit rotate is two
// v_alignbit_b32 (the compiler's shift pair + or takes three), and a ^ b ^ c is one
// v_bitop3_b32 per half (LUT 0x96) where the compiler emits two v_xor_b32.
__device__ __forceinline__ uint32_t lo32(uint64_t x) { return (uint32_t)x; }
__device__ __forceinline__ uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
__device__ __forceinline__ uint64_t mk64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
template <int K>  // rotate left by K, 0 < K < 64, K != 32
__device__ __forceinline__ uint64_t rotl64c(uint64_t x) {
  static_assert(K > 0 && K < 64 && K != 32, "rotate amount");
  if constexpr (K < 32)
    return mk64(__builtin_amdgcn_alignbit(lo32(x), hi32(x), 32 - K), __builtin_amdgcn_alignbit(hi32(x), lo32(x), 32 - K));
  else
    return mk64(__builtin_amdgcn_alignbit(hi32(x), lo32(x), 64 - K), __builtin_amdgcn_alignbit(lo32(x), hi32(x), 64 - K));
}
__device__ __forceinline__ uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
  return mk64(__builtin_amdgcn_bitop3_b32(lo32(a), lo32(b), lo32(c), 0x96),
              __builtin_amdgcn_bitop3_b32(hi32(a), hi32(b), hi32(c), 0x96));
}
// one xoshiro256++ step (rand_xoshiro 0.7.0 Xoshiro256PlusPlus::next_u64) on state s0..s3
__device__ __forceinline__ void xoshiro_step(uint64_t& s0, uint64_t& s1, uint64_t& s2, uint64_t& s3) {
  // s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= s1 << 17 (old s1); s3 = rotl(s3, 45)
  const uint64_t t = s1 << 17;
  const uint64_t n1 = xor3_64(s1, s2, s0);
  const uint64_t n0 = xor3_64(s0, s3, s1);
  const uint64_t n2 = xor3_64(s2, s0, t);
  s3 = rotl64c<45>(s3 ^ s1);
  s0 = n0;
  s1 = n1;
  s2 = n2;
}
__device__ __forceinline__ uint64_t xoshiro_out(uint64_t s0, uint64_t s3) { return rotl64c<23>(s0 + s3) + s0; }
__device__ __forceinline__ uint32_t xoshiro_out_hi_nc(uint64_t s0, uint64_t s3) {
  const uint64_t a = s0 + s3;
  return __builtin_amdgcn_alignbit(hi32(a), lo32(a), 9) + hi32(s0);  // hi32(rotl(a, 23)) + hi32(s0)
}
__device__ __forceinline__ uint64_t sat_sub(uint64_t a, uint64_t b) { return a > b ? a - b : 0; }
__device__ __forceinline__ uint64_t mul_sat(uint64_t a, uint64_t b, uint64_t cap) {
  uint64_t hi = __umul64hi(a, b);
  uint64_t lo = a * b;
  return (hi != 0 || lo > cap) ? cap : lo;
}
// EmulatedTime::saturating_add (emulated_time.rs:106-111)
__device__ __forceinline__ uint64_t emu_sat_add(uint64_t t, uint64_t d) {
  uint64_t x = t + d;
  return (x < t || x > EMU_MAX) ? EMU_MAX : x;
}

__device__ __forceinline__ bool ev_less(const EvRec& a, const EvRec& b) {
  if (a.time != b.time) return a.time < b.time;
  if (a.src != b.src) return a.src < b.src;
  return a.eid < b.eid;
}

// ---- cross-workgroup data inside one launch (persistent rounds; MI355X L2s are per XCD and
// not coherent): data another workgroup reads in a later round is stored write-through with
// device-scope atomic stores, and control words are read with device-scope atomic loads.
template <typename T>
__device__ __forceinline__ T ld_dev(SGN_GLB T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_dev(SGN_GLB T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ EvRec ld_dev_rec(SGN_GLB const EvRec* p) {
  SGN_GLB uint64_t* q = (SGN_GLB uint64_t*)p;
  EvRec r;
  r.time = ld_dev(q);
  r.eid = ld_dev(q + 1);
  const uint64_t sd = ld_dev(q + 2), pt = ld_dev(q + 3);
  r.src = (uint32_t)sd;
  r.dst = (uint32_t)(sd >> 32);
  r.pc = (uint32_t)pt;
  r.tag = (uint32_t)(pt >> 32);
  return r;
}
// A 16-byte write-through store (global_store_dwordx4 sc1: the agent-scope form of a store,
// MI355X_MICROARCH.md's store table): a 32-byte record as two of them is two 32-B fabric
// writes, where four 8-byte sc1 stores were four (tools/pmc_calib.sh: an 8-B sc1 store costs
// a 32-B write). hipcc does not count an asm store in its waits: the round's arrival waits for
// every store with its own s_waitcnt vmcnt(0); the s_nop keeps the data registers from being
// overwritten under the store.
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_wt16(SGN_GLB void* p, uint64_t lo, uint64_t hi) {
  u64x2 v;
  v.x = lo;
  v.y = hi;
  // (no "memory" clobber: nothing in this wave reads the stored bytes before the round's
  // arrival, whose own volatile asm s_waitcnt stays after this one; the clobber made hipcc
  // keep a local aggregate in scratch)
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"((uint64_t)p), "v"(v));
}
__device__ __forceinline__ void st_dev_rec(SGN_GLB EvRec* p, const EvRec& r) {
  SGN_GLB char* q = (SGN_GLB char*)p;
  st_wt16(q, r.time, r.eid);
  st_wt16(q + 16, (uint64_t)r.src | ((uint64_t)r.dst << 32), (uint64_t)r.pc | ((uint64_t)r.tag << 32));
}

// Multi-shard exchange data (a peer shard's inbox: another GPU's memory over xGMI, or the
// RCCL transport's send block): written through to memory at system scope (sc0 sc1), so the
// record is in the receiver's memory when the writing wave's s_waitcnt vmcnt(0) completes — the
// sender publishes its round-edge message only after every such store has completed.
__device__ __forceinline__ void st_sys16(SGN_GLB void* p, uint64_t lo, uint64_t hi) {
  u64x2 v;
  v.x = lo;
  v.y = hi;
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"((uint64_t)p), "v"(v));
}
__device__ __forceinline__ void st_sys_rec(SGN_GLB EvRec* p, const EvRec& r) {
  SGN_GLB char* q = (SGN_GLB char*)p;
  st_sys16(q, r.time, r.eid);
  st_sys16(q + 16, (uint64_t)r.src | ((uint64_t)r.dst << 32), (uint64_t)r.pc | ((uint64_t)r.tag << 32));
}
__device__ __forceinline__ void st_sys(SGN_GLB uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys(SGN_GLB uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ EvRec ld_sys_rec(SGN_GLB const EvRec* p) {
  SGN_GLB uint64_t* q = (SGN_GLB uint64_t*)p;
  EvRec r;
  r.time = ld_sys(q);
  r.eid = ld_sys(q + 1);
  const uint64_t sd = ld_sys(q + 2), pt = ld_sys(q + 3);
  r.src = (uint32_t)sd;
  r.dst = (uint32_t)(sd >> 32);
  r.pc = (uint32_t)pt;
  r.tag = (uint32_t)(pt >> 32);
  return r;
}

// CoDel pool entries: a page serves other hosts (other workgroups, other XCDs) after it is
// freed, so its entries are written through and read from memory like other cross-workgroup
// data (a dirty L2 line of the previous owner must never overwrite the new owner's runs)
__device__ __forceinline__ CodelEnt ld_dev_cq(SGN_GLB const CodelEnt* p) {
#ifdef SGN_EXP_PLAINCQ  // cost experiment only (build_exp.sh): what device scope costs config C
  return *p;
#endif
  SGN_GLB uint64_t* q = (SGN_GLB uint64_t*)p;
  CodelEnt e;
  e.enqueue_ts = ld_dev(q);
  e.eid = ld_dev(q + 1);
  const uint64_t a = ld_dev(q + 2), b = ld_dev(q + 3);
  e.src = (uint32_t)a;
  e.payload = (uint32_t)(a >> 32);
  e.tag = (uint32_t)b;
  e.count = (uint32_t)(b >> 32);
  return e;
}
__device__ __forceinline__ void st_dev_cq(SGN_GLB CodelEnt* p, const CodelEnt& e) {
#ifdef SGN_EXP_PLAINCQ
  *p = e;
  return;
#endif
  SGN_GLB char* q = (SGN_GLB char*)p;
  st_wt16(q, e.enqueue_ts, e.eid);
  st_wt16(q + 16, (uint64_t)e.src | ((uint64_t)e.payload << 32), (uint64_t)e.tag | ((uint64_t)e.count << 32));
}

// device-scope atomic min whose result is not used: the wave does not wait for it here (a
// returning one costs a round trip per call); the arrival's s_waitcnt vmcnt(0) completes it
// before the round edge reads the minima
__device__ __forceinline__ void min_nr(SGN_GLB uint64_t* p, uint64_t v) {
  (void)__hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a rare per-host counter in the host record: a no-return atomic add, so the lane does not
// wait for a load of the old value
__device__ __forceinline__ void cnt_add(SGN_GLB uint64_t* p, uint64_t v) {
  (void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a / b for a divisor below 2^32: u32 division when the dividend fits too
__device__ __forceinline__ uint64_t div_small(uint64_t a, uint64_t b) {
  if (((a | b) >> 32) == 0) return (uint32_t)a / (uint32_t)b;
  return a / b;
}

__device__ __forceinline__ uint32_t bucket_of(const DevSim& S, uint64_t t) {
  return (uint32_t)S.bw_div.div(t - SIM_START) & (S.NB - 1);
}

// CoDel control law (router/codel_queue.rs:285-298)
__device__ __forceinline__ uint64_t codel_law(uint64_t time, uint64_t count) {
  double sq = count == 0 ? 1.0 : sqrt((double)count);
  double div = 100000000.0 / sq;
  uint64_t inc = (uint64_t)round(div);
  uint64_t orig = time - SIM_START;
  uint64_t adj = orig + inc;
  if (adj < orig || adj > SIMTIME_MAX) adj = SIMTIME_MAX;
  return SIM_START + adj;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, off, 64);
    uint32_t hi = __shfl_xor((uint32_t)(v >> 32), off, 64);
    uint64_t o = ((uint64_t)hi << 32) | lo;
    v = o < v ? o : v;
  }
  return v;
}

// wave-uniform values (the same in every lane) into scalar registers: vector registers are the
// round kernels' scarce resource
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni32((uint32_t)(v >> 32)) << 32) | uni32((uint32_t)v);
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, off, 64);
    uint32_t hi = __shfl_xor((uint32_t)(v >> 32), off, 64);
    uint64_t o = ((uint64_t)hi << 32) | lo;
    v = o > v ? o : v;
  }
  return v;
}

// ---- a big slab's order key: Shadow's (time, src host, src event id) (core/work/event.rs:84-155)
// as one 160-bit string (time - tmin, src, eid) in three words, for a radix select over it ----
struct BigKey {
  uint64_t hi, mid, lo;  // time - tmin | src << 32 | eid >> 32 | eid << 32 (low 32 bits zero)
};
__device__ __forceinline__ BigKey big_key(const EvRec& r, uint64_t tmin) {
  return {r.time - tmin, ((uint64_t)r.src << 32) | (r.eid >> 32), r.eid << 32};
}
__device__ __forceinline__ bool bk_less(const BigKey& a, const BigKey& b) {
  return a.hi != b.hi ? a.hi < b.hi : a.mid != b.mid ? a.mid < b.mid : a.lo < b.lo;
}
// the 8-bit digit at bit p from the top (p a multiple of 8, < 192)
__device__ __forceinline__ uint32_t bk_digit(const BigKey& k, uint32_t p) {
  const uint64_t w = p < 64 ? k.hi : p < 128 ? k.mid : k.lo;
  return (uint32_t)(w >> (56 - (p & 63))) & 0xFFu;
}
__device__ __forceinline__ BigKey bk_set_digit(BigKey k, uint32_t p, uint32_t d) {
  const uint64_t v = (uint64_t)d << (56 - (p & 63));
  if (p < 64) k.hi |= v; else if (p < 128) k.mid |= v; else k.lo |= v;
  return k;
}
// k with every bit below the top p set (the largest key with k's top p bits)
__device__ __forceinline__ uint64_t bk_fill_w(uint64_t w, int keep) {
  return keep >= 64 ? w : keep <= 0 ? ~0ULL : (w | (~0ULL >> keep));
}
__device__ __forceinline__ BigKey bk_fill(const BigKey& k, uint32_t p) {
  return {bk_fill_w(k.hi, (int)p), bk_fill_w(k.mid, (int)p - 64), bk_fill_w(k.lo, (int)p - 128)};
}
// the masks of a key's top p bits (wave-uniform: scalar registers)
__device__ __forceinline__ BigKey bk_mask(uint32_t p) {
  auto m = [](int keep) -> uint64_t { return keep >= 64 ? ~0ULL : keep <= 0 ? 0ULL : ~(~0ULL >> keep); };
  return {m((int)p), m((int)p - 64), m((int)p - 128)};
}
__device__ __forceinline__ bool bk_prefix_eq(const BigKey& a, const BigKey& b, const BigKey& m) {
  return (((a.hi ^ b.hi) & m.hi) | ((a.mid ^ b.mid) & m.mid) | ((a.lo ^ b.lo) & m.lo)) == 0;
}
// the key fields of a record written by another workgroup (device-scope loads)
__device__ __forceinline__ void ld_dev_key(SGN_GLB const EvRec* p, uint64_t& t, uint64_t& e, uint32_t& src) {
  SGN_GLB uint64_t* q = (SGN_GLB uint64_t*)p;
  t = ld_dev(q);
  e = ld_dev(q + 1);
  src = (uint32_t)ld_dev(q + 2);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int off) {
  const uint32_t lo = __shfl_xor((uint32_t)v, off, 64);
  const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), off, 64);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// block-wide (256 threads) minimum, result valid in every thread
__device__ __forceinline__ uint64_t block_min_u64(uint64_t v, uint64_t* sh) {
  v = wave_min_u64(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  uint64_t r = sh[0];
  const int nw = blockDim.x >> 6;
  for (int i = 1; i < nw; i++) r = sh[i] < r ? sh[i] : r;
  __syncthreads();
  return r;
}

struct Pkt {
  uint32_t src;
  uint32_t dst_ip;
  uint32_t payload;
  uint32_t tag;
  uint64_t eid;
};

// ------------------------------------------------------------------------------------
// Per-host executor: the host's whole state lives in registers for the round.
// ------------------------------------------------------------------------------------
// A lane's LDS slot: the pending digest runs and the digests themselves (touched once per
// run), and the CoDel queue's cached head and open tail runs.
constexpr uint32_t GATHER_SPEC = 16;  // slab slots a gather loads before the fill is known
// The round kernels' dynamic LDS before the optional bucket-minimum table: CAP event runs and
// two u16 index arrays (padded to 8 bytes), at least 1 KB — a big slab's radix select keeps its
// 256-bin histogram there (exec_group), and test hooks may set CAP below 32
__host__ __device__ __forceinline__ size_t exec_lds_runs_bytes(uint32_t cap) {
  const size_t b = (size_t)cap * sizeof(EvRec) + 2 * (size_t)((cap + 3) & ~3u) * 2;
  return b > 1024 ? b : 1024;
}

// The wave's outbox: event records for this shard's calendar, placed after the event loop
// by all 64 lanes at once (one round trip for all the slab reservations of the wave instead
// of one per send in the sending lane's serial path). A full outbox falls back to placing
// the record at once.
// Its size is per kernel: 40 records for TGEN (config C: ~100 of 1563 server groups send more
// than 24 records a round, up to ~90; same-box A/B 24 -> 40: -0.5 % per launch, and 40 still
// leaves C at 7 workgroups per CU), 24 for the others (config D's PERIODIC kernel must keep 8
// workgroups per CU WITH its bucket-minimum table of 256 buckets: at 48 records the table no
// longer fit and D ran 3.4x slower; 32 measured the same as 24, round 4).
// a forwarding step of more packets than this waits for the wave's other lanes (HostExec::run)
#ifndef SGN_TRAIN_WAIT
#define SGN_TRAIN_WAIT 8
#endif
constexpr uint32_t kTrainWait = SGN_TRAIN_WAIT;
// PERIODIC forwarding waits only in waves with at least this many lanes in their event loops
#ifndef SGN_FWD_WAIT_LANES
#define SGN_FWD_WAIT_LANES 24
#endif
constexpr uint32_t kFwdWaitLanes = SGN_FWD_WAIT_LANES;
template <uint32_t kApp>
#ifndef SGN_OBOX_PERIODIC
#define SGN_OBOX_PERIODIC 24
#endif
constexpr uint32_t kObox = kApp == SGN_TRAFFIC_TGEN ? 40 : kApp == SGN_TRAFFIC_PERIODIC ? SGN_OBOX_PERIODIC : 24;
struct OutboxHdr {
  uint32_t n;          // records appended (may exceed the outbox: those were placed directly)
  uint64_t xmin;       // earliest run exported to another shard this round (multi-shard)
  uint64_t hz;         // calendar horizon: a run at or after it would alias a live bucket
  SGN_GLB uint64_t* keepmin;  // minimum of this round's new runs for the window's last bucket
  uint32_t* bmin;             // LDS minima per bucket (+ [NB]: the spare slab) or null (below),
  uint64_t bbase;             // ... as offsets from this time (the round's window start)
  uint64_t pg_avail;          // CoDel page pool: free-ring entries allocations may use this round
  SGN_GLB uint64_t* pg_freed; // ... and the round's freed-page counter
  SGN_GLB uint64_t* pg_allocd;// ... and allocated-page counter (the round edge's guard)
  SGN_GLB uint64_t* spilled;  // runs this round put in the calendar's spill area
  SGN_GLB uint32_t* xn;       // multi-shard: this round's per-peer run counters
  uint32_t* xc;               // k_rounds_x: this workgroup's runs per peer this round (LDS; null:
                              // no inbox bins, every remote run goes to its peer's slot)
  uint32_t xbuf;              // ... and the peer blocks they go to (XPeer::runs[xbuf])
};
template <uint32_t N>
struct OutboxN : OutboxHdr {
  EvRec rec[N];
  uint32_t idx[N];  // (slab set, group) slab index
};
template <uint32_t kApp>
using Outbox = OutboxN<kObox<kApp>>;
#ifdef SGN_EXP_NOPAIR  // cost experiment (build_exp.sh): one lane per outbox record
constexpr bool kPairOff = true;
#else
constexpr bool kPairOff = false;
#endif

// A run whose calendar slab is full goes to the spill area with its slab index (lossless; the
// round edge holds and the host re-lays the calendar out before the run can be due). Only a
// full spill area is an overflow.
__device__ __forceinline__ void spill_run(const DevSim& S, OutboxHdr* ob, uint32_t idx, const EvRec& r) {
  SGN_GLB Ctrl* C = S.ctrl;
  const uint64_t i = __hip_atomic_fetch_add(&C->spill_n, 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (ob) cnt_add(ob->spilled, 1);
  if (i < S.spill_cap) {
    st_dev_rec(S.spill + i, r);
    st_dev(&S.spill_idx[i], idx);
  } else if ((atomicOr(&C->overflow, OVF_BUCKET) & OVF_BUCKET) == 0) {
    C->overflow_info = r.dst;
  }
}

// A run at position pos >= CAP of slab idx: the slab's extension when it has room, else the
// spill area (lossless either way).
__device__ __forceinline__ void place_overflow(const DevSim& S, OutboxHdr* ob, uint32_t idx, uint32_t pos,
                                               const EvRec& r) {
  if (S.ext) {
    const uint64_t x = S.ext[idx];
    const uint32_t k = pos - S.CAP;
    if (k < (uint32_t)(x >> 40)) {
      st_dev_rec(S.ext_pool + (x & EXT_OFF_MASK) + k, r);
      return;
    }
  }
  spill_run(S, ob, idx, r);
}

// LDS copies of queue entries need only 8-byte alignment (a 16-byte-aligned member would
// pad every lane's slot to a multiple of 16 B and cost a workgroup per CU)
// (copies between them and the 16-byte-aligned global entries are compiled as 8-byte LDS
// pairs, ds_write2_b64 / ds_read2_b64; clang's align-mismatch note on them is expected)
#pragma clang diagnostic ignored "-Walign-mismatch"
typedef CodelEnt CodelEnt8 __attribute__((aligned(8)));
typedef FifoEnt FifoEnt8 __attribute__((aligned(8)));
// Per-lane state in the lane's LDS slot or, for the PERIODIC kernels (configs B and D, whose
// occupancy LDS limits: config D's 15,625 groups on the resident grid), elsewhere (every
// field keeps its full width: no limit beyond the reference's):
// * CoDel drop state (interval end, drop next, current / previous count): the PERIODIC
//   kernels keep it in the host record only (HostRec::cq_*, touched only when the queue
//   stands);
// * route cache, token-bucket increments, app counter, send-queue head index: the PERIODIC
//   kernels keep them in registers (they have ~40 VGPRs to spare below the 256 of two waves
//   per SIMD; the TGEN kernel, whose occupancy is fine, keeps its registers).
// Config D's per-workgroup LDS went 26.1 -> 23.1 -> 20.0 KB: 6 -> 7 -> 8 workgroups per CU.
struct LaneCq {
  uint64_t cq[4];
};
struct LaneNoCq {};
struct LaneRc {
  uint64_t rc_lat;   // route cache: latency and loss threshold (send_batch) ...
  uint64_t rc_T;
  uint64_t tbc[2];   // token buckets' refill increments (capacity = increment + MTU)
  uint64_t app_k;    // synthetic app counter
  uint32_t rc_dst;   // ... to this peer (NO_HOST: none)
  uint32_t rc_sid;   // ... whose slot id is this
  uint32_t fh_idx;   // the send queue head copy's ring index (NO_HOST: none)
};
struct LaneNoRc {};
template <uint32_t kApp>
constexpr bool kRcReg = kApp == SGN_TRAFFIC_PERIODIC;
// the hot host line in per-64-host tiles, field-major (DevSim::htile, hot_idx): every chunk load
// or store of a wave is one contiguous access instead of one line per lane. PERIODIC only:
// same-box A/B, D 4.45 -> 4.61 G, B +0.3 %; the TGEN kernel of config C
// measured 1.1 % slower (its cold lines are read with the hot one anyway)
template <uint32_t kApp>
constexpr bool kSoa = kApp == SGN_TRAFFIC_PERIODIC;  // (TGEN with them in registers: C unchanged)
// the kernels whose sends fold their bucket minima in an LDS table (S.agg_bmin, flush_bmin):
// PERIODIC (configs B and D: ~1 M sends a round on a few bucket words at D). TGEN has the LDS
// since round 3's slimmer lane slots, but measured 2 % slower with the table on C.
template <uint32_t kApp>
constexpr bool kAggBmin = kApp == SGN_TRAFFIC_PERIODIC;
// a pending digest run (sgn_drun of sgn_workload.h) with its count kept apart (LaneLDS::rn):
// sgn_drun's 4-byte count pads it to 32 bytes, three of them 12 bytes of every lane's slot
struct DRunL {
  uint64_t a, b, c;
};
template <uint32_t kApp>
struct LaneLDS : std::conditional_t<kApp == SGN_TRAFFIC_PERIODIC, LaneNoCq, LaneCq>,
                 std::conditional_t<kRcReg<kApp>, LaneNoRc, LaneRc> {
  DRunL run[3];      // tx, rx, app pending runs (sgn_workload.h) ...
  uint64_t dig[3];   // tx, rx, app digests
  CodelEnt8 hd, tl;  // head run being consumed / tail run being extended
  FifoEnt8 fh;       // copy of the send queue's head entry (ring index: LaneRc::fh_idx)
  uint32_t cq_tp;    // CoDel chain's tail page
  uint32_t rn[3];    // ... and their counts
};

// A slab with more due runs than the LDS holds (a hot spot: thousands of sources sending to one
// host group within a bucket width) is ordered and executed in pieces of at most CAP runs in
// Shadow's key order: piece k holds the runs with keys in (bound k-1, bound k]. The piece state
// lives in LDS across the pieces' event loops (registers are the round kernel's scarce resource:
// nothing of it is live in registers across HostExec::run, which reads the piece's tail time
// and flush flag from here — INVALID and 1 outside the big-slab path).
struct BigLDS {
  uint64_t tmin, range;  // earliest due run's time, latest - earliest
  uint64_t kp[3];        // the last piece's upper bound (BigKey)
  uint64_t ib;           // the slab
  uint64_t tail;         // run(): a host's next packet time after its runs of this piece
  uint64_t spill_imp;    // spill-area entries that may hold imported runs (multi-shard): set by
                         // the round kernels (k_import's count, or k_rounds_x's after its imports)
  uint32_t ndue, done, have_prev, nraw, flush, pad;
};

// kTrace: the per-packet trace can be on (k_execute). The persistent k_rounds is built
// without it (its registers are fully used; a traced run executes round by round).
// kApp: the traffic kind (SGN_TRAFFIC_*), fixed per instantiation so that each kernel
// carries only its application's code (fewer registers, no dead branches).
template <bool kTrace, uint32_t kApp>
struct HostExec {
  const DevSim& S;
  SGN_GLB Ctrl* C;
  uint32_t h, gid, my_ip, my_unode;
  uint64_t now, we;
  uint32_t b1, keep_slab;  // the window's last bucket (its new events go to the spare slab)
  // RNG (host/host.rs:234) and counters (host.rs:259-263)
  uint64_t r0, r1, r2, r3;
  uint64_t eid;
  uint64_t st0, st1, st2, se0, se1, se2;  // local event slots: relay out, relay in, app
  uint32_t fl;
  uint32_t ro_dst, ro_pay, ro_tag;
  uint32_t ri_src, ri_pay, ri_tag;
  uint64_t ri_eid;
  uint64_t tbb0, tbl0, tbb1, tbl1;  // balances / last refills (capacity, increment: memory)
  uint32_t cq_head, cq_nr, cq_len;  // head run's pool index (page * CQ_PAGE + offset), runs, packets queued
  uint64_t cq_bytes;  // (CoDel drop state: the lane's LDS slot)
  uint32_t fq_head, fq_len;
  // per-round counter increments (a host cannot see 2^32 events in one window)
  uint32_t c_sent, c_loss, c_popped, c_deliv, c_localev, c_maxcodel;
  uint32_t c_runs;  // event runs this host appended to this shard's calendar (occupancy)
  uint64_t c_bytes;
  // CoDel run cache: the head run being consumed and the tail run being extended live in
  // registers; their ring slots are stale until store() (or until the tail is closed).
  bool hd_valid, tl_open;
  // state touched O(1) times per run lives in this lane's LDS slot (registers are the
  // scarce resource: they set how many waves are resident)
  LaneLDS<kApp>* L;
  std::conditional_t<kRcReg<kApp>, LaneRc, LaneNoRc> rr;  // (see LaneLDS)
  __device__ __forceinline__ LaneRc& lr() {
    if constexpr (kRcReg<kApp>) return rr;
    else return *L;
  }
  __device__ __forceinline__ const LaneRc& lr() const {
    if constexpr (kRcReg<kApp>) return rr;
    else return *L;
  }
  SGN_GLB HostRec* R;     // this host's record (set by load())
  const uint16_t* bslab;  // LDS copy of the bucket -> slab table (when NB <= LDS_BSLAB)
  Outbox<kApp>* ob;       // the wave's outbox (LDS)
  const BigLDS* bg;       // the big-slab piece state (LDS)
#ifdef SGN_DIAG
  uint32_t dgt[DGT_N];
  uint32_t wk[5];
#endif

  __device__ HostExec(const DevSim& s, uint32_t hh, uint64_t w, uint32_t bucket1, uint32_t ks,
                      LaneLDS<kApp>* l, const uint16_t* bs, Outbox<kApp>* o, const BigLDS* b)
      : S(s), C(s.ctrl), h(hh), now(0), we(w), b1(bucket1), keep_slab(ks), L(l), bslab(bs), ob(o), bg(b) {}

  // the host's state into registers (once per round, only for hosts with something due);
  // fresh = false: a reload after park() (the pending digest runs in LDS continue)
  __device__ __forceinline__ void load(bool fresh = true) {
    R = S.hrec + h;
    const HostRec& r = *R;
    if constexpr (kApp == SGN_TRAFFIC_PERIODIC) {
      const HostConst& k = S.hconst[h];
      gid = k.gid;
      my_ip = k.ip;
      my_unode = k.unode;
      lr().tbc[0] = k.tb_inc[0];
      lr().tbc[1] = k.tb_inc[1];
    } else {  // (in the cold lines these kinds read anyway)
      gid = r.k_gid;
      my_ip = r.k_ip;
      my_unode = r.k_unode;
      lr().tbc[0] = r.k_tbinc[0];
      lr().tbc[1] = r.k_tbinc[1];
    }
    // the hot line
    if constexpr (kSoa<kApp>) {
      const SGN_GLB u64x2* T = (const SGN_GLB u64x2*)S.htile + hot_idx(h, 0);
      // (chunk 7 first: the flags decide the cold loads below; then the rest in order of use)
      const u64x2 c7 = T[448];
      fl = (uint32_t)c7.y;
      cq_head = (uint32_t)(c7.y >> 32);
      lr().app_k = c7.x;
      const u64x2 c0 = T[0], c1 = T[64], c2 = T[128], c3 = T[192], c4 = T[256], c5 = T[320], c6 = T[384];
      r0 = c0.x;
      r1 = c0.y;
      r2 = c1.x;
      r3 = c1.y;
      eid = c2.x;
      st2 = c2.y;
      se2 = c3.x;
      tbb0 = c3.y;
      tbb1 = c4.x;
      tbl0 = c4.y;
      tbl1 = c5.x;
      L->dig[0] = c5.y;
      L->dig[1] = c6.x;
      L->dig[2] = c6.y;
    } else {
    r0 = r.rng[0];
    r1 = r.rng[1];
    r2 = r.rng[2];
    r3 = r.rng[3];
    eid = r.eid;
    st2 = r.st2;
    se2 = r.se2;
    fl = r.flags;
    tbb0 = r.tb_bal[0];
    tbl0 = r.tb_last[0];
    tbb1 = r.tb_bal[1];
    tbl1 = r.tb_last[1];
    cq_head = r.cq_head;
    lr().app_k = r.app_k;
    L->dig[0] = r.dig[0];
    L->dig[1] = r.dig[1];
    L->dig[2] = r.dig[2];
    }
    // the cold lines (PERIODIC: only when the host ended its last round with state there)
    if (kApp != SGN_TRAFFIC_PERIODIC || (fl & F_COLD)) {
      st0 = r.st0;
      st1 = r.st1;
      se0 = r.se0;
      se1 = r.se1;
      ro_dst = r.ro_dst;
      ro_pay = r.ro_pay;
      ro_tag = r.ro_tag;
      ri_src = r.ri_src;
      ri_pay = r.ri_pay;
      ri_tag = r.ri_tag;
      ri_eid = r.ri_eid;
      L->cq_tp = r.cq_tp;
      cq_nr = r.cq_nr;
      cq_len = r.cq_len;
      cq_bytes = r.cq_bytes;
      fq_head = r.fq_head;
      fq_len = r.fq_len;
      lr().rc_dst = r.rc_dst;
      lr().rc_sid = r.rc_sid;
      lr().rc_lat = r.rc_lat;
      lr().rc_T = r.rc_T;
      if constexpr (kApp != SGN_TRAFFIC_PERIODIC) {
        L->cq[0] = r.cq_ie;
        L->cq[1] = r.cq_dn;
        L->cq[2] = r.cq_cur;
        L->cq[3] = r.cq_prev;
      }
    } else {  // an idle host: both relays idle, no cached packets, both queues empty
      st0 = st1 = INVALID;
      se0 = se1 = 0;
      ro_dst = ro_pay = ro_tag = ri_src = ri_pay = ri_tag = 0;
      ri_eid = 0;
      L->cq_tp = cq_head / CQ_PAGE;  // (an empty queue keeps its page: head and tail)
      cq_nr = cq_len = 0;
      cq_bytes = 0;
      fq_head = fq_len = 0;
      lr().rc_dst = NO_HOST;
      lr().rc_sid = 0;
      lr().rc_lat = lr().rc_T = 0;
    }
    c_sent = c_loss = c_popped = c_deliv = c_localev = c_bytes = 0;
    c_runs = 0;
    c_maxcodel = kApp == SGN_TRAFFIC_PERIODIC ? 0u : r.max_codel;
    hd_valid = tl_open = false;
    if (cq_nr > 0) {
      L->hd = ld_dev_cq(cq_head_slot());
      hd_valid = true;
    }
    lr().fh_idx = NO_HOST;
    if (fq_len > 0) {
      L->fh = *fq_slot(0);
      lr().fh_idx = fq_head;
    }
    if (fresh) L->rn[0] = L->rn[1] = L->rn[2] = 0;
#ifdef SGN_DIAG
    for (int i = 0; i < DGT_N; i++) dgt[i] = 0;
    for (int i = 0; i < 5; i++) wk[i] = 0;
#endif
  }

  // PERIODIC traffic: the app's next datagram goes to a peer that is a hash of the app counter
  // (sgn_periodic_dst), so its route can be in the route cache before the event loop needs it.
  // store() leaves that peer in S.npeer; the next round's prefetch_peer(np) issues the peer's
  // load beside the host record's (one round trip for both, not one after the other);
  // prefetch_route() (after the gather's sort, so the load's latency hides behind it) fetches
  // the route entry. A cache fill only: the entry is a pure function of (this host's node, the
  // peer), so a hint that is not the next peer costs a miss, never a different result.
  uint32_t pf_peer;
  uint64_t pf_pi;
  // a peer's slot id | used-node index << 32: from the 4-byte table when sim_init built one
  // (half the bytes of the 8-byte one: config D's 1 M-host table is 4 MB, about an XCD's L2)
  __device__ __forceinline__ uint64_t peer_info(uint32_t dst) const {
    if (S.peer32) {
      const uint32_t v = S.peer32[dst];
      return (v & ((1u << S.peer_sb) - 1u)) | ((uint64_t)(v >> S.peer_sb) << 32);
    }
    return S.peer[dst];
  }
  __device__ __forceinline__ void prefetch_peer(uint32_t np) {
    pf_peer = np;
    pf_pi = np != NO_HOST ? peer_info(np) : 0;
  }
  __device__ __forceinline__ uint32_t next_peer() const {
    uint32_t peer = NO_HOST, uip = 0;
    if (!periodic_dst(lr().app_k, &peer, &uip)) peer = NO_HOST;
    return peer;
  }
  // sgn_periodic_dst / sgn_tgen_fetch (sgn_workload.h) with the remainders by multiply-high
  // (u64 % is a long software routine on the GPU; the results are the same integers)
  __device__ __forceinline__ uint64_t mod_by(const UDiv64& d, uint64_t x, uint64_t n) const { return x - d.div(x) * n; }
  __device__ __forceinline__ bool periodic_dst(uint64_t k, uint32_t* peer, uint32_t* uip) const {
    const uint64_t r = sgn_flow_hash(S.flow_seed, gid, k);
    if ((uint32_t)mod_by(S.div_1000, r, 1000u) < S.unknown_permille) {
      *uip = SGN_UNKNOWN_IP_BASE + (uint32_t)((r >> 32) & 0xFFFFu);
      return false;
    }
    *peer = (uint32_t)mod_by(S.div_n, r >> 16, S.n_all);
    return true;
  }
  __device__ __forceinline__ void prefetch_route() {
    if (pf_peer == NO_HOST) return;
    const RouteEnt re = S.route[(size_t)my_unode * S.U + (uint32_t)(pf_pi >> 32)];
    lr().rc_dst = pf_peer;
    lr().rc_sid = (uint32_t)pf_pi;
    lr().rc_lat = re.lat;
    lr().rc_T = re.T;
  }

  // old_next / old_peer: this host's S.nextloc / S.npeer as the round read them (a value that did
  // not change is not stored again: a host-round that only took deliveries writes neither,
  // and at config B's 16-host waves each was a partial-line write of its own)
  __device__ __forceinline__ void store(uint64_t old_next, uint32_t old_peer) {
    HostRec& r = *R;
    if constexpr (!kSoa<kApp>) {
    r.rng[0] = r0;
    r.rng[1] = r1;
    r.rng[2] = r2;
    r.rng[3] = r3;
    r.eid = eid;
    r.st2 = st2;
    r.se2 = se2;
    r.tb_bal[0] = tbb0;
    r.tb_bal[1] = tbb1;
    r.tb_last[0] = tbl0;
    r.tb_last[1] = tbl1;
    r.dig[0] = L->dig[0];
    r.dig[1] = L->dig[1];
    r.dig[2] = L->dig[2];
    r.app_k = lr().app_k;
    r.cq_head = cq_head;
    }
    if (fl & F_FH_DIRTY) *fq_slot(0) = L->fh;  // a queued head that lived in LDS
    // the cold lines: PERIODIC writes them only when the host leaves state there (load() gives
    // an idle host its defaults: this must list every field that differs from them)
    const bool cold = kApp != SGN_TRAFFIC_PERIODIC || st0 != INVALID || st1 != INVALID ||
                      (fl & (F_RO_STATE | (3u << F_RI_STATE_SHIFT) | F_RO_NEXT | F_RI_NEXT | F_CODEL_IE |
                             F_CODEL_DN | F_CODEL_DROP)) ||
                      cq_nr || cq_len || cq_bytes || fq_len || fq_head;
    if constexpr (kSoa<kApp>) {
      SGN_GLB u64x2* T = (SGN_GLB u64x2*)S.htile + hot_idx(h, 0);
      const uint32_t f = (fl & ~(F_FH_DIRTY | F_COLD)) | (cold ? F_COLD : 0u);
      T[0] = u64x2{r0, r1};
      T[64] = u64x2{r2, r3};
      T[128] = u64x2{eid, st2};
      T[192] = u64x2{se2, tbb0};
      T[256] = u64x2{tbb1, tbl0};
      T[320] = u64x2{tbl1, L->dig[0]};
      T[384] = u64x2{L->dig[1], L->dig[2]};
      T[448] = u64x2{lr().app_k, (uint64_t)f | ((uint64_t)cq_head << 32)};
    } else {
      r.flags = (fl & ~(F_FH_DIRTY | F_COLD)) | (cold ? F_COLD : 0u);
    }
    if (cold) {
      r.st0 = st0;
      r.st1 = st1;
      r.se0 = se0;
      r.se1 = se1;
      r.ri_eid = ri_eid;
      r.cq_bytes = cq_bytes;
      r.rc_lat = lr().rc_lat;
      r.rc_T = lr().rc_T;
      r.ro_dst = ro_dst;
      r.ro_pay = ro_pay;
      r.ro_tag = ro_tag;
      r.ri_src = ri_src;
      r.ri_pay = ri_pay;
      r.ri_tag = ri_tag;
      r.cq_tp = L->cq_tp;
      r.cq_nr = cq_nr;
      r.cq_len = cq_len;
      r.fq_head = fq_head;
      r.fq_len = fq_len;
      r.rc_dst = lr().rc_dst;
      r.rc_sid = lr().rc_sid;
      if constexpr (kApp != SGN_TRAFFIC_PERIODIC) {
        r.cq_ie = L->cq[0];
        r.cq_dn = L->cq[1];
        r.cq_cur = L->cq[2];
        r.cq_prev = L->cq[3];
      }
    }
    // the per-host totals: PERIODIC no-return adds into dense arrays (no load of the old
    // value, no cold line); the other kinds in their cold lines
    if constexpr (kApp == SGN_TRAFFIC_PERIODIC) {
#ifndef SGN_EXP_NOCNT  // (cost experiments only, build_exp.sh: the traffic of each per-host stream)
      const size_t nH = S.nH;
      if (c_sent) cnt_add(&S.n_cnt[N_SENT * nH + h], c_sent);
      if (c_popped) cnt_add(&S.n_cnt[N_POPPED * nH + h], c_popped);
      if (c_deliv) cnt_add(&S.n_cnt[N_DELIVERED * nH + h], c_deliv);
      if (c_maxcodel)
        (void)__hip_atomic_fetch_max(&S.maxq[h], c_maxcodel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
    } else {
      r.max_codel = c_maxcodel;
      r.n_sent += c_sent;
      r.n_popped += c_popped;
      r.n_delivered += c_deliv;
    }
#ifndef SGN_EXP_NONEXT
    const uint64_t nl = next_local_time();
    if (nl != old_next) S.nextloc[h] = nl;
    if (kApp == SGN_TRAFFIC_PERIODIC) {
      const uint32_t p = next_peer();
      if (p != old_peer) S.npeer[h] = p;
    }
#endif
    if (hd_valid) st_dev_cq(cq_head_slot(), L->hd);
    if (tl_open) st_dev_cq(cq_tail_slot(), L->tl);
  }

  // The register state is dead from here (a big slab's passes run with the whole register file;
  // park: the state went to memory with store(), and loaded lanes reload it): constants in every
  // field that load() defines, on every path, so no earlier value stays live across the passes.
  __device__ __forceinline__ void kill() {
    gid = my_ip = my_unode = 0;
    r0 = r1 = r2 = r3 = eid = 0;
    st0 = st1 = st2 = se0 = se1 = se2 = 0;
    fl = ro_dst = ro_pay = ro_tag = ri_src = ri_pay = ri_tag = 0;
    ri_eid = tbb0 = tbl0 = tbb1 = tbl1 = 0;
    cq_head = cq_nr = cq_len = fq_head = fq_len = 0;
    cq_bytes = 0;
    c_sent = c_loss = c_popped = c_deliv = c_localev = c_maxcodel = c_runs = 0;
    c_bytes = 0;
    hd_valid = tl_open = false;
    if constexpr (kRcReg<kApp>) rr = LaneRc{};
    pf_peer = 0;
    pf_pi = 0;
    R = nullptr;
  }



  __device__ __forceinline__ uint64_t next_local_time() const {
    uint64_t m = st0;
    m = st1 < m ? st1 : m;
    m = st2 < m ? st2 : m;
    return m;
  }

  // ---- Xoshiro256++ (rand_xoshiro 0.7.0) + rand 0.9.2 StandardUniform f64 ----
  __device__ __forceinline__ uint64_t rng_next() {
    const uint64_t result = xoshiro_out(r0, r3);
    xoshiro_step(r0, r1, r2, r3);
    return result;
  }
  __device__ __forceinline__ void rng_skip() { xoshiro_step(r0, r1, r2, r3); }  // rng_next without its output
  // rng_next's high word without the carry out of its low word (the true high word is this
  // or this + 1): three VALU ops where the whole output takes six
  __device__ __forceinline__ uint32_t rng_next_hi_nc() {
    const uint32_t h = xoshiro_out_hi_nc(r0, r3);
    xoshiro_step(r0, r1, r2, r3);
    return h;
  }
  __device__ __forceinline__ double rng_f64() {
    return (double)(rng_next() >> 11) * 0x1.0p-53;
  }

  __device__ __forceinline__ bool tr() const { return kTrace && S.trace_on; }
  __device__ __forceinline__ void trace(uint32_t kind, uint32_t peer, uint32_t flags, uint64_t a, uint64_t b,
                        uint64_t c) {
    if (!tr()) return;
    const uint64_t seq = R->tseq++;
    uint64_t pos = atomicAdd((unsigned long long*)&C->trace_n, 1ULL);
    if (pos >= S.trace_cap) {
      atomicOr(&C->overflow, OVF_TRACE);
      return;
    }
    sgn_trace_rec r;
    r.kind = kind;
    r.host = gid;
    r.peer = peer;
    r.flags = flags;
    r.a = a;
    r.b = b;
    r.c = c;
    r.seq = seq;
    r.rng_pos = R->rng_pos;
    S.trace[pos] = r;
  }

  __device__ __forceinline__ void overflow(uint32_t bit) {
    if ((atomicOr(&C->overflow, bit) & bit) == 0) C->overflow_info = gid;
  }

  // EXTERNAL traffic: a datagram's fate for the CPU-side applications (sgn_drain)
  __device__ __forceinline__ void drain_rec(uint32_t status, uint32_t src, uint32_t dst, uint64_t seid,
                            uint32_t payload, uint32_t tag) {
    const uint64_t pos = atomicAdd((unsigned long long*)&C->drain_n, 1ULL);
    if (pos >= S.drain_cap) {
      overflow(OVF_DRAIN);
      return;
    }
    sgn_drain_rec r;
    r.time = now;
    r.src_eid = seid;
    r.handle = 0;
    r.host = gid;
    r.src_host = src;
    r.dst_host = dst;
    r.status = status;
    r.payload_len = payload;
    r.tag = tag;
    S.drain[pos] = r;
  }
  __device__ __forceinline__ bool external() const { return kApp == SGN_TRAFFIC_EXTERNAL; }

  // ---- local event slots: Host::schedule_task_* / push_local_event (host.rs:703-722);
  //      Event::new_local consumes an event id even if the event is then dropped ----
  template <int SL>
  __device__ __forceinline__ void schedule(uint64_t t) {
    uint64_t e = eid++;
    if (t >= S.end_time) return;
    if (SL == SLOT_RO) { st0 = t; se0 = e; }
    if (SL == SLOT_RI) { st1 = t; se1 = e; }
    if (SL == SLOT_APP) { st2 = t; se2 = e; }
  }

  template <int W>
  __device__ __forceinline__ uint32_t relay_state() const {
    return W == 0 ? (fl & 3u) : ((fl >> F_RI_STATE_SHIFT) & 3u);
  }
  template <int W>
  __device__ __forceinline__ void set_relay_state(uint32_t v) {
    if (W == 0)
      fl = (fl & ~3u) | v;
    else
      fl = (fl & ~(3u << F_RI_STATE_SHIFT)) | (v << F_RI_STATE_SHIFT);
  }

  // Relay::notify (relay/mod.rs:111-136) and forward_later (:145-163)
  template <int W>
  __device__ __forceinline__ void forward_later(uint64_t delay) {
    set_relay_state<W>(RELAY_PENDING);
    schedule<W == 0 ? SLOT_RO : SLOT_RI>(now + delay);
  }
  template <int W>
  __device__ __forceinline__ void relay_notify() {
    if (relay_state<W>() == RELAY_IDLE) forward_later<W>(0);
  }

  // ---- TokenBucket::comforming_remove (network/relay/token_bucket.rs:65-154) ----
  template <int W>
  __device__ __forceinline__ bool tb_remove(uint64_t dec, uint64_t* dur) {
    DGT_BEGIN(tt);
    const bool ok = tb_remove_<W>(dec, dur);
    DGT_END(DGT_TBRM, tt);
    return ok;
  }
  template <int W>
  __device__ __forceinline__ bool tb_remove_(uint64_t dec, uint64_t* dur) {
    uint64_t& bal = W == 0 ? tbb0 : tbb1;
    uint64_t& last = W == 0 ? tbl0 : tbl1;
    const uint64_t interval = 1000000ULL;  // relay/mod.rs:279
    // lazy_refill. The refill increment and capacity stay in memory (they are only read
    // when a refill is due or a removal fails, not on the per-packet fast path).
    uint64_t span = now - last;
    if (span >= interval) {
      const uint64_t inc = lr().tbc[W];
      uint64_t nref = span / interval;
      uint64_t ntok = mul_sat(inc, nref, ~0ULL);
      uint64_t b = bal + ntok;
      if (b < bal) b = ~0ULL;
      const uint64_t cap = inc + SGN_CONFIG_MTU;  // every relay's bucket: sim_init
      bal = b > cap ? cap : b;
      uint64_t adv = mul_sat(interval, nref, SIMTIME_MAX);
      last = emu_sat_add(last, adv);
      span = now - last;
    }
    uint64_t next_refill_span = interval - span;
    if (dec > bal) {
      // compute_conforming_duration (:91-117)
      const uint64_t inc = lr().tbc[W];
      uint64_t req = dec - bal;
      uint64_t n;
      if (((req | inc) >> 32) == 0) {  // u32 division: the u64 routine is long
        const uint32_t r32 = (uint32_t)req, i32 = (uint32_t)inc;
        const uint32_t q = r32 / i32;
        n = q + (r32 - q * i32 ? 1 : 0);
      } else {
        n = req / inc + ((req % inc) ? 1 : 0);
      }
      if (n == 0)
        *dur = 0;
      else if (n == 1)
        *dur = next_refill_span;
      else {
        uint64_t m = mul_sat(interval, n - 1, SIMTIME_MAX);
        uint64_t s = next_refill_span + m;
        if (s < next_refill_span || s > SIMTIME_MAX) s = SIMTIME_MAX;
        *dur = s;
      }
      return false;
    }
    bal -= dec;
    return true;
  }

  // sgn_drun_{flush,add}_{seq,same} (sgn_workload.h) over LaneLDS::run / rn
  template <int K>
  __device__ __forceinline__ void dr_flush_seq() {
#ifndef SGN_EXP_NODIGEST
    const uint32_t n = L->rn[K];
    if (n) L->dig[K] = sgn_digest3(L->dig[K], L->run[K].a, L->run[K].b | ((uint64_t)n << 32), L->run[K].c - n);
    L->rn[K] = 0;
#endif
  }
  template <int K>
  __device__ __forceinline__ void dr_flush_same() {
#ifndef SGN_EXP_NODIGEST
    const uint32_t n = L->rn[K];
    if (n) L->dig[K] = sgn_digest3(L->dig[K], L->run[K].a, L->run[K].b | ((uint64_t)n << 34), L->run[K].c);
    L->rn[K] = 0;
#endif
  }
  template <int K>
  __device__ __forceinline__ void dr_add_seq(uint64_t a, uint64_t b, uint64_t c0, uint32_t n) {
#ifndef SGN_EXP_NODIGEST
    DRunL& r = L->run[K];
    if (L->rn[K] && r.a == a && r.b == b && r.c == c0) {
      L->rn[K] += n;
      r.c += n;
      return;
    }
    dr_flush_seq<K>();
    r.a = a;
    r.b = b;
    r.c = c0 + n;
    L->rn[K] = n;
#endif
  }
  template <int K>
  __device__ __forceinline__ void dr_add_same(uint64_t a, uint64_t b, uint64_t c, uint32_t n) {
#ifndef SGN_EXP_NODIGEST
    DRunL& r = L->run[K];
    if (L->rn[K] && r.a == a && r.b == b && r.c == c) {
      L->rn[K] += n;
      return;
    }
    dr_flush_same<K>();
    r.a = a;
    r.b = b;
    r.c = c;
    L->rn[K] = n;
#endif
  }

  // the CoDel drop state (LaneCq / HostRec::cq_*, see LaneLDS)
  template <int I>
  __device__ __forceinline__ uint64_t cqg() const {
    if constexpr (kApp == SGN_TRAFFIC_PERIODIC)
      return I == 0 ? R->cq_ie : I == 1 ? R->cq_dn : I == 2 ? R->cq_cur : R->cq_prev;
    else
      return L->cq[I];
  }
  template <int I>
  __device__ __forceinline__ void cqs(uint64_t v) {
    if constexpr (kApp == SGN_TRAFFIC_PERIODIC) {
      if (I == 0) R->cq_ie = v;
      if (I == 1) R->cq_dn = v;
      if (I == 2) R->cq_cur = v;
      if (I == 3) R->cq_prev = v;
    } else {
      L->cq[I] = v;
    }
  }

  // ---- CoDel (router/codel_queue.rs) on a chain of pool pages ----
  // The queue's runs in order fill the head page from cq_head's offset, whole pages, and the
  // tail page (L->cq_tp) up to run cq_nr - 1; only the head and tail runs are ever touched.
  __device__ __forceinline__ SGN_GLB CodelEnt* cq_head_slot() { return S.codel + cq_head; }
  __device__ __forceinline__ SGN_GLB CodelEnt* cq_tail_slot() {
    return S.codel + ((size_t)L->cq_tp * CQ_PAGE + ((cq_head + cq_nr - 1) & (CQ_PAGE - 1)));
  }
  // a page from the pool: the free ring's next entry, if it was freed before this round
  // (the entries of the current round are still being written by other waves)
  __device__ __forceinline__ uint32_t cq_alloc_page() {
    DGT_BEGIN(ta);
    const uint64_t i = __hip_atomic_fetch_add(&C->pg_alloc, 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    cnt_add(ob->pg_allocd, 1);
    if (i >= ob->pg_avail) return NO_HOST;
    const uint32_t pg = ld_dev(&S.cq_free[i % S.cq_pages]);
#ifdef SGN_DIAG
    DGT_WAIT();
    DGT_END(DGT_CQALLOC, ta);
#endif
    return pg;
  }
  __device__ __forceinline__ void cq_free_page(uint32_t pg) {
    DGT_BEGIN(tf);
    const uint64_t j = __hip_atomic_fetch_add(&C->pg_tail, 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    st_dev(&S.cq_free[j % S.cq_pages], pg);
    cnt_add(ob->pg_freed, 1);
    DGT_END(DGT_CQFREE, tf);
  }
  // the head run left the queue: next run, next page (the old one back to the pool), or an
  // empty queue that keeps its page from the start
  __device__ __forceinline__ void cq_pop_head() {
    cq_nr--;
    if (cq_nr == 0) {
      cq_head &= ~(CQ_PAGE - 1);
      L->cq_tp = cq_head / CQ_PAGE;
    } else if (((cq_head + 1) & (CQ_PAGE - 1)) != 0) {
      cq_head++;
    } else {
      const uint32_t pg = cq_head / CQ_PAGE;
      const uint32_t nx = ld_dev(&S.cq_next[pg]);  // (neighbouring links belong to other hosts)
      cq_free_page(pg);
      cq_head = nx * CQ_PAGE;
    }
  }
  // Router::route_incoming_packet (router/mod.rs:55-57) -> CoDelQueue::push (:303-317) for a
  // run of n packets arriving at `now`: extends the open tail run when it continues it.
  __device__ __forceinline__ void codel_push_run(uint32_t src, uint64_t eid0, uint32_t payload, uint32_t tag,
                                 uint32_t n) {
    const auto continues = [&](const CodelEnt& r) {
      return r.enqueue_ts == now && r.src == src && r.eid + r.count == eid0 &&
             r.payload == payload && r.tag == tag;
    };
    if (tl_open && continues(L->tl)) {
      L->tl.count += n;
    } else if (!tl_open && hd_valid && cq_nr == 1 && continues(L->hd)) {
      L->hd.count += n;
    } else {
      if (tl_open) {
        st_dev_cq(cq_tail_slot(), L->tl);
        tl_open = false;
      }
      if (cq_nr > 0 && ((cq_head + cq_nr) & (CQ_PAGE - 1)) == 0) {
        // the tail page is full: link a page from the pool
        const uint32_t np = cq_alloc_page();
        if (np == NO_HOST) {
          overflow(OVF_CODEL);
          return;
        }
        st_dev(&S.cq_next[L->cq_tp], np);
        L->cq_tp = np;
      }
      L->tl.enqueue_ts = now;
      L->tl.eid = eid0;
      L->tl.src = src;
      L->tl.payload = payload;
      L->tl.tag = tag;
      L->tl.count = n;
      tl_open = true;
      cq_nr++;
    }
    cq_len += n;
    cq_bytes += (uint64_t)n * ((uint64_t)payload + sgn_header_bytes(tag));
    if (cq_len > c_maxcodel) c_maxcodel = cq_len;
  }
  // process_standing_delay (:231-262)
  __device__ __forceinline__ bool codel_standing(uint64_t sd) {
    if (sd < CODEL_TARGET || cq_bytes <= SGN_CONFIG_MTU) {
      fl &= ~F_CODEL_IE;
      return false;
    }
    if (fl & F_CODEL_IE) return now >= cqg<0>();
    fl |= F_CODEL_IE;
    cqs<0>(emu_sat_add(now, CODEL_INTERVAL));
    return false;
  }
  // the head run into registers (queue not empty)
  __device__ __forceinline__ void load_head() {
    if (hd_valid) return;
    if (tl_open && cq_nr == 1) {  // the only run is the open tail: take it over
      L->hd = L->tl;
      tl_open = false;
    } else {
      DG(DG_HDLOAD);
      DGT_BEGIN(th);
      L->hd = ld_dev_cq(cq_head_slot());
      DGT_WAIT();
      DGT_END(DGT_HDLD, th);
    }
    hd_valid = true;
  }
  // codel_pop (:204-227)
  __device__ __forceinline__ bool codel_pop_raw(Pkt* p, bool* ok_to_drop) {
    if (cq_len == 0) {
      fl &= ~F_CODEL_IE;
      return false;
    }
    load_head();
    const CodelEnt e = L->hd;
    L->hd.eid++;
    if (--L->hd.count == 0) {
      hd_valid = false;
      cq_pop_head();
    }
    cq_len--;
    cq_bytes = sat_sub(cq_bytes, (uint64_t)e.payload + sgn_header_bytes(e.tag));
    *ok_to_drop = codel_standing(sat_sub(now, e.enqueue_ts));
    p->src = e.src;
    p->dst_ip = my_ip;
    p->payload = e.payload;
    p->tag = e.tag;
    p->eid = e.eid;
    return true;
  }
  __device__ __forceinline__ void codel_drop(const Pkt& p) {  // drop_packet (:319-321)
    cnt_add(&R->n_codel, 1);
    if (external()) drain_rec(SGN_DRAIN_CODEL, p.src, gid, p.eid, p.payload, p.tag);
    dr_add_seq<2>(now, (uint64_t)p.src | (1ULL << 63), p.eid, 1);
    trace(SGN_TRACE_CODEL_DROP, p.src, 0, now, 0, p.eid);
  }
  __device__ __forceinline__ bool codel_was_dropping_recently() const {  // :273-281
    if (!(fl & F_CODEL_DN)) return false;
    return sat_sub(now, cqg<1>()) < CODEL_INTERVAL * 16;
  }
  // CoDelQueue::pop (:125-201)
  __device__ __forceinline__ bool codel_pop(Pkt* out) {
    Pkt p;
    bool okd;
    if (!codel_pop_raw(&p, &okd)) {
      fl &= ~F_CODEL_DROP;
      return false;
    }
    if (!okd) {
      fl &= ~F_CODEL_DROP;
      *out = p;
      return true;
    }
    if (!(fl & F_CODEL_DROP)) {
      // drop_from_store_mode (:150-170)
      codel_drop(p);
      Pkt n;
      bool nok;
      bool has_n = codel_pop_raw(&n, &nok);
      fl |= F_CODEL_DROP;
      uint64_t delta = sat_sub(cqg<2>(), cqg<3>());
      const uint64_t cur = (codel_was_dropping_recently() && delta > 1) ? delta : 1;
      cqs<2>(cur);
      fl |= F_CODEL_DN;
      cqs<1>(codel_law(now, cur));
      cqs<3>(cur);
      if (has_n) *out = n;
      return has_n;
    }
    // drop_from_drop_mode (:172-201)
    bool has_item = true;
    Pkt item = p;
    while (has_item && (fl & F_CODEL_DROP) && (fl & F_CODEL_DN) && now >= cqg<1>()) {
      codel_drop(item);
      cqs<2>(cqg<2>() + 1);
      bool iok = false;
      has_item = codel_pop_raw(&item, &iok);
      if (has_item && iok)
        cqs<1>(codel_law(cqg<1>(), cqg<2>()));
      else
        fl &= ~F_CODEL_DROP;
    }
    if (has_item) *out = item;
    return has_item;
  }

  // ---- synthetic socket send queue (interface qdisc source for relay_inet_out) ----
  __device__ __forceinline__ FifoEnt* fq_slot(uint32_t i) {
    uint32_t idx = fq_head + i;
    if (idx >= S.fifo_cap) idx -= S.fifo_cap;
    return S.fifo + (size_t)h * S.fifo_cap + idx;
  }
  // dst NO_HOST: a datagram to `addr`, an address outside the simulation (the trace keeps
  // it in a side array, S.fifo_addr, for the capture record)
  __device__ __forceinline__ bool fifo_push(uint32_t dst, uint32_t payload, uint32_t last, uint32_t count,
                            uint32_t tag, uint32_t addr = 0) {
    if (fq_len >= S.fifo_cap) return false;
    if (tr() && dst == NO_HOST) S.fifo_addr[fq_slot(fq_len) - S.fifo] = addr;
    FifoEnt e;
    e.dst = dst;
    e.pay = (payload & 0xFFFFu) | (last << 16);
    e.count = count;
    e.tag = tag;
    if (fq_len == 0) {
      // the new head lives in LDS only: most are sent within the round, and a global store
      // here would hold up the wave's next dependent load (stores and loads share vmcnt);
      // store() writes it back if it is still queued
      L->fh = e;
      lr().fh_idx = fq_head;
      fl |= F_FH_DIRTY;
    } else {
      *fq_slot(fq_len) = e;
    }
    fq_len++;
    return true;
  }
  // the head entry (from the LDS copy when it is current)
  __device__ __forceinline__ FifoEnt fifo_head() {
    if (lr().fh_idx == fq_head) return L->fh;
    DGT_BEGIN(tf);
    const FifoEnt e = *fq_slot(0);
    DGT_WAIT();
    DGT_END(DGT_FHLD, tf);
    L->fh = e;
    lr().fh_idx = fq_head;
    return e;
  }

  // ---- Dns::addr_to_host_id (network/dns.rs:174) ----
  __device__ __forceinline__ bool dns_lookup(uint32_t ip, uint32_t* host) const {
    uint32_t i = (ip * 0x9E3779B1u) & S.dns_mask;
    while (true) {
      uint32_t k = S.dns_key[i];
      if (k == ip) {
        *host = S.dns_val[i];
        return true;
      }
      if (k == 0) return false;
      i = (i + 1) & S.dns_mask;
    }
  }

  // interface delivery to the synthetic app (NetworkInterface::push -> socket) of m packets
  // from src with consecutive event ids e0.. at `now` (one run-encoded app digest step)
  __device__ __forceinline__ void deliver_run(uint32_t src, uint64_t e0, uint32_t m, uint32_t payload,
                              uint32_t tag) {
    c_deliv += m;
    c_bytes += (uint64_t)m * payload;
    dr_add_seq<2>(now, src, e0, m);
    if (tr())
      for (uint32_t k = 0; k < m; k++)
        trace(SGN_TRACE_DELIVER, src, 0, now, (uint64_t)payload | ((uint64_t)tag << 32), e0 + k);
    if (external())
      for (uint32_t k = 0; k < m; k++) drain_rec(SGN_DRAIN_DELIVERED, src, gid, e0 + k, payload, tag);
    if (kApp == SGN_TRAFFIC_TGEN && (fl & F_SERVER) && (tag & SGN_TAG_REQ)) {
      const uint32_t c = tag & 3u;  // the class picks one of three (scalar) sizes
      const uint64_t size = c == 0 ? S.file_bytes[0] : (c == 1 ? S.file_bytes[1] : S.file_bytes[2]);
      const uint64_t n = (size + SGN_TGEN_MSS - 1) / SGN_TGEN_MSS;
      if (n == 0) return;
      const uint32_t last = (uint32_t)(size - (n - 1) * SGN_TGEN_MSS);
      for (uint32_t k = 0; k < m; k++) {
        if (fifo_push(src, SGN_TGEN_MSS, last, (uint32_t)n, SGN_TAG_RESP))
          relay_notify<0>();
        else
          cnt_add(&R->n_blocked, 1);
      }
    }
  }
  __device__ __forceinline__ void deliver_local(const Pkt& p) {  // loopback: a digest run of its own
    cnt_add(&R->n_local_deliv, 1);
    if (tr()) trace(SGN_TRACE_LOCAL, gid, 0, now, (uint64_t)p.payload | ((uint64_t)p.tag << 32), 0);
    if (external()) drain_rec(SGN_DRAIN_LOCAL, gid, gid, 0, p.payload, p.tag);
    dr_flush_seq<2>();
    L->dig[2] = sgn_digest3(L->dig[2], now, (uint64_t)p.src | (1ULL << 62) | (1ULL << 32), p.payload);
  }

  // ---- Relay::forward_until_blocked (network/relay/mod.rs:201-273) for relay_inet_in:
  //      the router's CoDel queue -> the interface (relay_inet_out uses forward_out) ----
  __device__ __forceinline__ bool forward_in(uint64_t* dur) {
    const bool boot = now < S.boot_end;
    set_relay_state<1>(RELAY_FORWARDING);
    while (true) {
      Pkt p;
      if (fl & F_RI_NEXT) {
        fl &= ~F_RI_NEXT;
        p.src = ri_src;
        p.dst_ip = my_ip;
        p.payload = ri_pay;
        p.tag = ri_tag;
        p.eid = ri_eid;
      } else {
        if (cq_len > 0) {
          load_head();
          // Fast path over the head run: every packet of it has the same standing delay and
          // wire size, and all removals happen at the same `now`. CoDelQueue::pop returns
          // each of them (codel_queue.rs:125-262) unless the delay is standing (>= TARGET)
          // past an interval end that is already due: below TARGET it clears interval_end
          // and drop mode; at or above it clears drop mode and only moves interval_end (set
          // to now + INTERVAL by the first pop that leaves more than an MTU queued, cleared
          // by the first that leaves less; the queued bytes only fall here, so the last pop
          // decides). After the first comforming_remove (which applies the lazy refill)
          // balance / wire more packets conform; the first that does not is cached.
          // In drop mode before drop_next, pop returns every packet without a drop too
          // (drop_from_drop_mode's loop does not run, :172-201) and changes nothing until a
          // pop leaves <= MTU queued (then interval_end and drop mode end).
          const bool standing = sat_sub(now, L->hd.enqueue_ts) >= CODEL_TARGET;
          const bool ie_due = (fl & F_CODEL_IE) && now >= cqg<0>();
          const bool drop_quiet = (fl & F_CODEL_DROP) && (fl & F_CODEL_DN) && now < cqg<1>();
          if (!standing || !ie_due || drop_quiet) {
            const uint32_t n = L->hd.count;
            const uint64_t wire = (uint64_t)L->hd.payload + sgn_header_bytes(L->hd.tag);
            uint32_t m = n;
            bool blocked = false;
            if (!boot) {
              if (!tb_remove<1>(wire, dur)) {
                m = 0;
                blocked = true;
              } else if (n > 1) {
                const uint64_t more = div_small(tbb1, wire);
                if (more >= n - 1) {
                  tbb1 -= (uint64_t)(n - 1) * wire;
                } else {
                  tbb1 -= more * wire;
                  m = 1 + (uint32_t)more;
                  blocked = true;
                  tb_remove<1>(wire, dur);  // fails: same `now`, gives the conforming duration
                }
              }
            }
            const uint32_t used = m + (blocked ? 1u : 0u);
            const CodelEnt r = L->hd;
            L->hd.eid += used;
            L->hd.count -= used;
            cq_len -= used;
            cq_bytes = sat_sub(cq_bytes, (uint64_t)used * wire);
            if (!standing || cq_bytes <= SGN_CONFIG_MTU) {
              fl &= ~(F_CODEL_IE | F_CODEL_DROP);
            } else if (!ie_due) {
              fl &= ~F_CODEL_DROP;
              if (!(fl & F_CODEL_IE)) {
                fl |= F_CODEL_IE;
                cqs<0>(emu_sat_add(now, CODEL_INTERVAL));
              }
            }  // else drop mode before drop_next: unchanged
            if (L->hd.count == 0) {
              hd_valid = false;
              cq_pop_head();
            }
            if (m) deliver_run(r.src, r.eid, m, r.payload, r.tag);
            if (blocked) {
              fl |= F_RI_NEXT;
              ri_src = r.src;
              ri_pay = r.payload;
              ri_tag = r.tag;
              ri_eid = r.eid + m;
              set_relay_state<1>(RELAY_IDLE);
              return true;
            }
            continue;
          }
        }
        const bool gotp = codel_pop(&p);
        if (!gotp) {
          set_relay_state<1>(RELAY_IDLE);
          return false;
        }
        DG(DG_FQLOAD);
      }
      // the source address is the router's (0.0.0.0), never this host's: no local bypass
      if (!boot && !tb_remove<1>((uint64_t)p.payload + sgn_header_bytes(p.tag), dur)) {
        fl |= F_RI_NEXT;
        ri_src = p.src;
        ri_pay = p.payload;
        ri_tag = p.tag;
        ri_eid = p.eid;
        set_relay_state<1>(RELAY_IDLE);
        return true;
      }
      deliver_run(p.src, p.eid, 1, p.payload, p.tag);
    }
  }

  // A run of n identical datagrams pushed to the router at the same `now`: n consecutive
  // Worker::send_packet calls (core/worker.rs:330-403). The DNS lookup, route entry,
  // reliability and delivery time are the same for all of them, so they are computed
  // once; the per-packet loss draws stay sequential (same RNG stream, same order) and the
  // digest takes runs of equal outcomes. Sent packets take consecutive source event ids and
  // share one delivery time, so their events are reserved with one atomic and written as
  // one contiguous run.
  // pop: (trace) each packet was just popped from the interface (an IF_POP record precedes its
  // SEND record, as NetworkInterface::pop precedes send_packet)
  __device__ __forceinline__ void send_batch(uint32_t dst, uint32_t payload, uint32_t tag, uint32_t n,
                                             bool pop = false) {
    DGT_BEGIN(t0);
    send_batch_(dst, payload, tag, n, pop);
    DGT_END(DGT_SEND, t0);
  }
  // one loss-draw outcome of send_batch_'s record-free path (tx digest runs only)
  __device__ __forceinline__ void loss_step(bool lost, uint32_t& run, uint32_t& sent, uint32_t dst,
                                            uint64_t deliver) {
    if (lost) {
      c_loss++;
      if (run) dr_add_same<0>(now, (uint64_t)dst, deliver, run);
      run = 0;
      dr_add_same<0>(now, (uint64_t)dst | (1ULL << 32), 0, 1);
    } else {
      run++;
      sent++;
    }
  }
  // dst: the HostId the address resolves to (FifoEnt), NO_HOST: not in the simulation
  // IF_POP of the send queue's head entry (an unknown address from the trace's side array)
  __device__ __forceinline__ void trace_pop(uint32_t dst, uint32_t payload, uint32_t tag) {
    trace(SGN_TRACE_IF_POP, dst, 0, now, (uint64_t)payload | ((uint64_t)tag << 32),
          dst == NO_HOST ? S.fifo_addr[fq_slot(0) - S.fifo] : 0);
  }
  __device__ __forceinline__ void send_batch_(uint32_t dst, uint32_t payload, uint32_t tag, uint32_t n, bool pop) {
    if (n == 0 || now >= S.end_time) return;
    DG(DG_BATCH);
    const bool boot = now < S.boot_end;
    if (dst == NO_HOST) {  // resolve_ip_to_host_id failed: InetDropped (worker.rs:347-357)
      cnt_add(&R->n_unknown, n);
      dr_add_same<0>(now, 0xFFFFFFFFULL | (2ULL << 32), 0, n);
      if (tr())
        for (uint32_t j = 0; j < n; j++) {
          if (pop) trace_pop(NO_HOST, payload, tag);
          trace(SGN_TRACE_SEND, 0xFFFFFFFFu, 2, now, 0, 0);
        }
      if (external())
        for (uint32_t j = 0; j < n; j++) drain_rec(SGN_DRAIN_UNKNOWN, gid, NO_HOST, 0, payload, tag);
      return;
    }
    // the route (WorkerShared::latency / reliability, worker.rs:523-537): a train goes to
    // one peer for many rounds, so the host keeps its last (peer, latency, threshold)
    uint64_t delay, T;
    uint32_t dsid;  // the destination's slot id (where its events are filed)
    if (lr().rc_dst == dst) {
      delay = lr().rc_lat;
      T = lr().rc_T;
      dsid = lr().rc_sid;
    } else {
      DG(DG_RMISS);
      DGT_BEGIN(trt);
      // the peer's slot and used node (one load), then its route entry (one 16-byte load):
      // drop iff chance >= reliability (worker.rs:366-371) with chance = (x >> 11) * 2^-53;
      // reliability = (f64)(1.0f - loss) is 0 or >= 2^-24, so reliability * 2^53 is an exact
      // integer T (precomputed per route, sim_init) and the test is (x >> 11) >= T, bit for
      // bit the same decision
      const uint64_t pi = peer_info(dst);
      dsid = (uint32_t)pi;
      const RouteEnt re = S.route[(size_t)my_unode * S.U + (uint32_t)(pi >> 32)];
      delay = re.lat;
      T = re.T;
      DGT_WAIT();
      DGT_END(DGT_RTLD, trt);
      lr().rc_dst = dst;
      lr().rc_sid = dsid;
      lr().rc_lat = delay;
      lr().rc_T = T;
    }
    uint64_t deliver = now + delay;
    if (deliver < we) deliver = we;
    const uint64_t eid0 = eid;
    const bool can_drop = !boot && payload > 0;
    uint32_t run = 0;  // consecutive sent packets not yet folded into the digest
    DGT_BEGIN(tr0);
#ifdef SGN_DIAG
    dgt[DGT_DRAWS] += n;
    if ((uint32_t)(__ffsll((long long)__ballot(1)) - 1) == (threadIdx.x & 63)) dgt[DGT_RENTRY] += 1;
    {
      const uint64_t lb = __ballot(n > kTrainWait);
      if (n > kTrainWait) dgt[DGT_LLANE] += 1;
      if (lb && (uint32_t)(__ffsll((long long)lb) - 1) == (threadIdx.x & 63)) dgt[DGT_LENTRY] += 1;
    }
#endif
#ifdef SGN_EXP_NORNG
    if (true) {
      run = n;
      eid += n;
    } else
#endif
    if (tr() || external()) {  // per-packet records
      for (uint32_t j = 0; j < n; j++) {
        if (tr() && pop) trace_pop(dst, payload, tag);
        const uint64_t x = rng_next() >> 11;
        if (tr()) R->rng_pos++;
        if (can_drop && x >= T) {
          c_loss++;
          if (run) dr_add_same<0>(now, (uint64_t)dst, deliver, run);
          run = 0;
          dr_add_same<0>(now, (uint64_t)dst | (1ULL << 32), 0, 1);
          if (tr()) trace(SGN_TRACE_SEND, dst, 1, now, 0, 0);
          if (external()) drain_rec(SGN_DRAIN_LOSS, gid, dst, 0, payload, tag);
        } else {
          const uint64_t e = eid++;
          run++;
          if (tr()) trace(SGN_TRACE_SEND, dst, 0, now, deliver, e);
        }
      }
    } else if (!can_drop || T >= (1ULL << 53)) {
      // nothing can drop (bootstrapping, empty payload, or a lossless path: chance < 1.0 =
      // reliability always); the draws still advance the stream (worker.rs:366 draws first)
#pragma unroll 8
      for (uint32_t j = 0; j < n; j++) rng_skip();
      run = n;
      eid += n;
    } else {
      // x >> 11 >= T  <=>  x >= T << 11 (T < 2^53); eight, then four draws per test
      const uint64_t Tx = T << 11;
      uint32_t sent = 0, j = 0;
      // eight draws per test (same-box A/B on config C: +1.3 % over four, sixteen was slower;
      // the loop's scalar control and test sit on the slowest waves' chain). The test is a
      // screen: a draw drops only if its high word is >= Tx's, and the high word is at most
      // the carry-less one + 1, so when the eight carry-less high words' maximum + 1 is below
      // Tx's high word none drops; otherwise the eight draws are redone exactly from the saved
      // state (probability ~ 8 x the path's loss). The stream advances the same either way.
      // Paths losing more than 1/32 of their packets would redo most batches (~1.7x the
      // exact test's cost), so they keep the exact test below. Same-box A/B: C -2.2 % per
      // launch (3486 -> 3411 us); micro-benchmark 126 -> 87 cycles per draw for a lone lane.
      // (TGEN kernel only: its servers send trains; a PERIODIC host sends single datagrams,
      // and the screen's registers took that kernel from 231 to 256 VGPRs)
      const uint32_t Th = (uint32_t)(Tx >> 32);
      if (kApp == SGN_TRAFFIC_TGEN && Th >= 0xF8000000u) for (; j + 8 <= n; j += 8) {
        const uint64_t a0 = r0, a1 = r1, a2 = r2, a3 = r3;
        const uint32_t h0 = rng_next_hi_nc(), h1 = rng_next_hi_nc(), h2 = rng_next_hi_nc(), h3 = rng_next_hi_nc();
        const uint32_t h4 = rng_next_hi_nc(), h5 = rng_next_hi_nc(), h6 = rng_next_hi_nc(), h7 = rng_next_hi_nc();
        const uint32_t hm = max(max(max(h0, h1), max(h2, h3)), max(max(h4, h5), max(h6, h7)));
        if (hm >= Th - 1 || Th == 0) {  // (hm + 1 >= Th without the wrap)
          r0 = a0;
          r1 = a1;
          r2 = a2;
          r3 = a3;
          const uint64_t x0 = rng_next(), x1 = rng_next(), x2 = rng_next(), x3 = rng_next();
          const uint64_t x4 = rng_next(), x5 = rng_next(), x6 = rng_next(), x7 = rng_next();
          loss_step(x0 >= Tx, run, sent, dst, deliver);
          loss_step(x1 >= Tx, run, sent, dst, deliver);
          loss_step(x2 >= Tx, run, sent, dst, deliver);
          loss_step(x3 >= Tx, run, sent, dst, deliver);
          loss_step(x4 >= Tx, run, sent, dst, deliver);
          loss_step(x5 >= Tx, run, sent, dst, deliver);
          loss_step(x6 >= Tx, run, sent, dst, deliver);
          loss_step(x7 >= Tx, run, sent, dst, deliver);
        } else {
          run += 8;
          sent += 8;
        }
      }
      for (; j + 8 <= n; j += 8) {
        const uint64_t x0 = rng_next(), x1 = rng_next(), x2 = rng_next(), x3 = rng_next();
        const uint64_t x4 = rng_next(), x5 = rng_next(), x6 = rng_next(), x7 = rng_next();
        if ((x0 >= Tx) | (x1 >= Tx) | (x2 >= Tx) | (x3 >= Tx) | (x4 >= Tx) | (x5 >= Tx) | (x6 >= Tx) |
            (x7 >= Tx)) {
          loss_step(x0 >= Tx, run, sent, dst, deliver);
          loss_step(x1 >= Tx, run, sent, dst, deliver);
          loss_step(x2 >= Tx, run, sent, dst, deliver);
          loss_step(x3 >= Tx, run, sent, dst, deliver);
          loss_step(x4 >= Tx, run, sent, dst, deliver);
          loss_step(x5 >= Tx, run, sent, dst, deliver);
          loss_step(x6 >= Tx, run, sent, dst, deliver);
          loss_step(x7 >= Tx, run, sent, dst, deliver);
        } else {
          run += 8;
          sent += 8;
        }
      }
      for (; j + 4 <= n; j += 4) {
        const uint64_t x0 = rng_next(), x1 = rng_next(), x2 = rng_next(), x3 = rng_next();
        if ((x0 >= Tx) | (x1 >= Tx) | (x2 >= Tx) | (x3 >= Tx)) {
          loss_step(x0 >= Tx, run, sent, dst, deliver);
          loss_step(x1 >= Tx, run, sent, dst, deliver);
          loss_step(x2 >= Tx, run, sent, dst, deliver);
          loss_step(x3 >= Tx, run, sent, dst, deliver);
        } else {
          run += 4;
          sent += 4;
        }
      }
      for (; j < n; j++) loss_step(rng_next() >= Tx, run, sent, dst, deliver);
      eid += sent;
    }
    DGT_END(DGT_APP, tr0);
    if (run) dr_add_same<0>(now, (uint64_t)dst, deliver, run);
    const uint32_t nsent = (uint32_t)(eid - eid0);
    if (nsent == 0) return;
    c_sent += nsent;
    // sent packets have consecutive ids (drops take none): one event run record each
    // RUN_MAX packets
    const uint32_t nrec = (nsent + RUN_MAX - 1) / RUN_MAX;
    if (S.dynamic) {  // Worker::update_lowest_used_latency (no return value: fire and forget)
      min_nr(&C->min_used, delay);
    }
    SGN_GLB EvRec* dstp;
    uint32_t cap;
    uint32_t pos;
    uint32_t sidx = 0;  // owned: the slab index (its spill tag)
    const bool owned = dst - S.lo < S.nH;
    if (owned) {
      if (deliver >= ob->hz) {  // past the calendar's horizon (sim_init sizes NB so it cannot be)
        overflow(OVF_HORIZON);
        return;
      }
      c_runs += nrec;
      const uint32_t b = bucket_of(S, deliver);
      const uint32_t slab = b == b1 ? keep_slab : (S.NB <= LDS_BSLAB ? bslab[b] : ld_dev(&S.bucket_slab[b]));
      const size_t idx = (size_t)slab * S.G + ((dsid - S.lo) >> S.gsh);
      // the bucket's pending minimum: folded in the workgroup's LDS table when it has one
      // (flush_bmin publishes it before the round's arrival), else one device atomic per run
      // (compiled for PERIODIC traffic only — configs B and D, where every host sends every
      // round; the TGEN kernel of config C keeps its per-run atomic, uncontended there)
      if (kAggBmin<kApp> && S.agg_bmin)
        atomicMin(&ob->bmin[b == b1 ? S.NB : b], (uint32_t)(deliver - ob->bbase));
      else
        min_nr(b == b1 ? ob->keepmin : &S.bucket_min[b], deliver);
      if (nrec == 1) {
        const uint32_t k = atomicAdd(&ob->n, 1u);  // LDS
        if (k < kObox<kApp>) {
          EvRec& r = ob->rec[k];
          r.time = deliver;
          r.eid = eid0;
          r.src = gid;
          r.dst = dsid;
          r.pc = payload | (nsent << 16);
          r.tag = tag;
          ob->idx[k] = (uint32_t)idx;
          return;
        }
      }
      DGT_BEGIN(tsl);
      pos = atomicAdd(&S.slab_n[idx], nrec);
      DGT_WAIT();
      DGT_END(DGT_SLAB, tsl);
      dstp = S.pool + idx * S.CAP;
      cap = S.CAP;
      sidx = (uint32_t)idx;
    } else {
      uint32_t lo = 0, hi = S.n_ranks, lov = 0;  // (rank_lo[0] = 0)
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint32_t v = S.rank_lo[mid];
        if (v <= dst) {
          lo = mid;
          lov = v;
        } else {
          hi = mid;
        }
      }
      atomicMin((unsigned long long*)&ob->xmin, (unsigned long long)deliver);  // LDS
      sidx = SPILL_PEER | lo;  // (runs beyond the peer's slot: the slot grows at a held round)
      bool binned = false;
      if (ob->xc) {
        // persistent rounds: the receiving host group's bin in the peer's inbox (its gather
        // reads it next round); a full bin sends the run to the peer's slot instead
        atomicAdd(&ob->xc[lo], nrec);  // LDS
        const uint32_t gr = (dsid - lov) >> S.gsh;
        pos = atomicAdd(&S.xbin_n[((size_t)ob->xbuf * S.n_ranks + lo) * S.xgx + gr], nrec);
        if (pos + nrec <= S.xbk) {
          binned = true;
          dstp = S.xp[lo].bins[ob->xbuf] + (size_t)gr * S.xbk;
          cap = S.xbk;
        }
      }
      if (!binned) {
        pos = atomicAdd(&ob->xn[lo], nrec);
        // the peer's block: the RCCL transport's send block (after its message records), or the
        // peer's inbox slot for this shard and round parity (persistent rounds: peer-mapped memory)
        dstp = S.xp[lo].runs[ob->xbuf];
        cap = ob->xbuf == 2 ? S.xslot : S.xislot;
      }
    }
    for (uint32_t m = 0; m < nrec; m++) {
      const uint32_t k = min(RUN_MAX, nsent - m * RUN_MAX);
      EvRec r;
      r.time = deliver;
      r.eid = eid0 + (uint64_t)m * RUN_MAX;
      r.src = gid;
      r.dst = dsid;
      r.pc = payload | (k << 16);
      r.tag = tag;
      if (pos + m < cap) {
        if (owned || !S.xsys)
          st_dev_rec(dstp + pos + m, r);
        else  // (another GPU's inbox)
          st_sys_rec(dstp + pos + m, r);
      } else if (owned)  // the slab is full: its extension, or the spill area
        place_overflow(S, ob, sidx, pos + m, r);
      else  // the peer's exchange slot is full
        spill_run(S, ob, sidx, r);
    }
  }

  // Relay::forward_until_blocked for relay_inet_out (network/relay/mod.rs:201-273), taking
  // the send queue a run at a time: a run is the leading datagrams of the head train that
  // share a payload size. All of them see the same `now`, so after the first
  // comforming_remove (which applies the lazy refill) no further refill happens and the
  // number that conform is balance / wire_len; the first that does not is cached exactly
  // like Relay::next_packet.
  // One step = the cached packet or one send-queue entry. The task runs step by step, one
  // step per iteration of the wave's event loop (F_RO_CONT: the host stays inside the task,
  // `now` does not move and none of its other events run until the queue is empty or the
  // bucket blocks), so lanes forwarding long trains send them side by side instead of one
  // after another (a train's per-packet loss draws are the serial part of a round).
  __device__ __forceinline__ void forward_out_step() {
    DGT_BEGIN(tf0);
    const bool boot = now < S.boot_end;
    uint64_t dur = 0;
    bool blocked = false;
    if (fl & F_RO_NEXT) {
      fl &= ~F_RO_NEXT;
      const bool is_local = ro_dst == gid;
      if (!boot && !is_local && !tb_remove<0>((uint64_t)ro_pay + sgn_header_bytes(ro_tag), &dur)) {
        fl |= F_RO_NEXT;
        blocked = true;
      } else {
        Pkt p;
        p.src = gid;
        p.dst_ip = my_ip;
        p.payload = ro_pay;
        p.tag = ro_tag;
        p.eid = 0;
        if (is_local)
          deliver_local(p);
        else
          send_batch(ro_dst, ro_pay, ro_tag, 1);
      }
    } else if (fq_len > 0) {
      const FifoEnt e = fifo_head();
      // round-robin qdisc with other sockets waiting: one packet, then this socket goes to
      // the back (NetworkInterface::pop, interface.rs:216-256); otherwise the leading
      // datagrams of the train that share a payload size
      const bool rr = S.qdisc_rr && fq_len > 1;
      const uint32_t run = (e.count == 1 || rr) ? 1u : e.count - 1;
      const uint32_t payload = e.count == 1 ? (e.pay >> 16) : (e.pay & 0xFFFFu);
      const uint64_t wire = (uint64_t)payload + sgn_header_bytes(e.tag);
      const bool is_local = e.dst == gid;
      uint32_t n_ok = run;
      if (!boot && !is_local) {
        if (!tb_remove<0>(wire, &dur)) {
          n_ok = 0;
          blocked = true;
        } else if (run > 1) {
          const uint64_t more = div_small(tbb0, wire);
          if (more >= run - 1) {
            tbb0 -= (uint64_t)(run - 1) * wire;
          } else {
            tbb0 -= more * wire;
            n_ok = 1 + (uint32_t)more;
            blocked = true;
            tb_remove<0>(wire, &dur);  // fails: same `now`, gives the conforming duration
          }
        }
      }
      if (is_local) {
        Pkt p;
        p.src = gid;
        p.dst_ip = my_ip;
        p.payload = payload;
        p.tag = e.tag;
        p.eid = 0;
        for (uint32_t j = 0; j < n_ok; j++) {
          if (tr()) trace_pop(gid, payload, e.tag);
          deliver_local(p);
        }
      } else {
        send_batch(e.dst, payload, e.tag, n_ok, true);
      }
      // the packet the bucket refused was popped too: it waits in Relay::next_packet
      if (tr() && blocked) trace_pop(e.dst, payload, e.tag);
      const uint32_t consumed = n_ok + (blocked ? 1u : 0u);
      if (consumed == e.count) {
        fq_head = fq_head + 1 == S.fifo_cap ? 0 : fq_head + 1;
        fq_len--;
        if (fq_len == 0) fq_head = 0;  // (an empty queue's head is 0: an idle host's default)
        fl &= ~F_FH_DIRTY;
      } else if (rr) {
        // the socket still has data: re-queued behind the others (same length)
        FifoEnt m = e;
        m.count = e.count - consumed;
        fq_head = fq_head + 1 == S.fifo_cap ? 0 : fq_head + 1;
        *fq_slot(fq_len - 1) = m;
        lr().fh_idx = NO_HOST;  // the cached head is stale
        fl &= ~F_FH_DIRTY;
      } else {
        if (!(fl & F_FH_DIRTY)) fq_slot(0)->count = e.count - consumed;
        L->fh.count = e.count - consumed;
      }
      if (blocked) {
        fl |= F_RO_NEXT;
        ro_dst = e.dst;
        ro_pay = payload;
        ro_tag = e.tag;
      }
    }
    if (blocked || (fq_len == 0 && !(fl & F_RO_NEXT))) {  // the task returns
      fl &= ~F_RO_CONT;
      set_relay_state<0>(RELAY_IDLE);
      if (blocked) forward_later<0>(dur);
    }
    DGT_END(DGT_FWDOUT, tf0);
  }

  // run_forward_task + forward_now (relay/mod.rs:166-187)
  template <int W>
  __device__ __forceinline__ void run_forward_task() {
    set_relay_state<W>(RELAY_IDLE);
    uint64_t dur;
    DGT_BEGIN(t0);
    const bool blocked = forward_in(&dur);
    DGT_END(DGT_FWDIN, t0);
    if (blocked) forward_later<W>(dur);
  }

  __device__ __forceinline__ void app_task() {
    const uint64_t k = lr().app_k++;
    uint32_t dst, payload, tag, uip = 0;
    uint64_t next_delay;
    if (kApp == SGN_TRAFFIC_PERIODIC) {
      uint32_t peer = 0;
      // an address outside the simulation (10.255.0.0/16, never registered) is NO_HOST
      dst = periodic_dst(k, &peer, &uip) ? peer : NO_HOST;
      payload = S.payload_len;
      tag = SGN_TAG_DATA;
      next_delay = S.period;
    } else {
      uint32_t si = 0, cls = 0;
      {  // sgn_tgen_fetch
        const uint64_t r = sgn_flow_hash(S.flow_seed, gid, k);
        si = (uint32_t)mod_by(S.div_ns, r >> 8, S.n_servers);
        cls = (uint32_t)((r >> 40) % 3u);
      }
      DGT_BEGIN(tsv);
      dst = S.servers[si];
      DGT_WAIT();
      DGT_END(DGT_SVLD, tsv);
      payload = S.req_payload;
      tag = SGN_TAG_REQ | cls;
      next_delay = sgn_tgen_think(S.flow_seed, gid, k, S.period, S.period_jitter);
    }
    if (fifo_push(dst, payload, payload, 1, tag, uip))
      relay_notify<0>();  // Host::notify_socket_has_packets (host.rs:969-983)
    else
      cnt_add(&R->n_blocked, 1);
    schedule<SLOT_APP>(now + next_delay);
  }

  // EXTERNAL traffic: the application's socket write (sgn_submit) enters the socket send
  // queue and notifies relay_inet_out (Host::notify_socket_has_packets, host.rs:969-983),
  // as app_task does for the synthetic apps. The record carries the destination address in
  // the low half of its event id (the high half is the submission order).
  __device__ __forceinline__ void app_submit(const EvRec& e) {
    uint32_t dst;
    if (!dns_lookup((uint32_t)e.eid, &dst)) dst = NO_HOST;
    const uint32_t payload = ev_payload(e);
    if (fifo_push(dst, payload, payload, 1, e.tag, (uint32_t)e.eid)) {
      relay_notify<0>();
    } else {
      cnt_add(&R->n_blocked, 1);
      drain_rec(SGN_DRAIN_BLOCKED, gid, NO_HOST, 0, payload, e.tag);
    }
  }

  // Is local slot W (0: relay_inet_out, 1: relay_inet_in) due at `now` and the host's next
  // event? No packet run at `now` (pt: the next due run's time) and every other local event
  // later by (time, event id).
  template <int W>
  __device__ __forceinline__ bool next_local_now(uint64_t pt) const {
    const uint64_t t = W == 0 ? st0 : st1, e = W == 0 ? se0 : se1;
    const uint64_t ta = W == 0 ? st1 : st0, ea = W == 0 ? se1 : se0;
    return t == now && pt > now && (ta > now || (ta == now && ea > e)) && (st2 > now || (st2 == now && se2 > e));
  }

  // ---- Host::execute (host.rs:762-830) over the host's due event runs + local slots ----
  // ev[ord[s0 .. s1)] are the host's runs due before `until` in Shadow's order, (time, src
  // host, src event id) (core/work/event.rs:84-155), in LDS; local events run while their
  // time < until. A window is executed as consecutive sub-windows (one per calendar
  // bucket): nothing created inside a window is due in it (packet deliveries are >= the
  // window end, worker.rs:386-390), so this is the same sequence of events.
  // bg->tail: the time of the host's next packet run after ev[ord[s1 - 1]] (INVALID: none) — a
  // slab ordered in pieces (exec_group's big-slab path) runs a host's runs over several calls,
  // each up to the next piece's bound; bg->flush: close the digests' pending runs (the last
  // piece of the sub-window only, so the digest steps are those of one call over all runs)
  __device__ __forceinline__ void run(const EvRec* ev, const uint16_t* ord, uint32_t s0, uint32_t s1,
                      uint64_t until) {
    uint32_t pi = s0;
    // (bg null: kernels without the big-slab path — no later piece, digests close here; the
    // tail is re-read from LDS where it is needed: a register across the loop spilled the
    // PERIODIC big-slab kernel)
    uint64_t pt = pi < s1 ? ev[ord[pi]].time : bg ? bg->tail : INVALID;  // next due packet run's time
#ifdef SGN_DIAG
#endif
    while (true) {
      const uint64_t act = __ballot(1);  // (the wave's lanes still in their event loops)
      // earliest local event by (time, event id)
      uint64_t lt = st0, le = se0;
      int ls = 0;
      if (st1 < lt || (st1 == lt && se1 < le)) { lt = st1; le = se1; ls = 1; }
      if (st2 < lt || (st2 == lt && se2 < le)) { lt = st2; le = se2; ls = 2; }
#ifdef SGN_DIAG
      {  // wave-level: iterations, and iterations in which some lane runs each handler;
         // the previous iteration's cycles are added to its handler combination's slot
        const bool ispop = pi < s1 && ev[ord[pi]].time <= lt;
        const int kind = (fl & F_RO_CONT) ? 1 : ispop ? 0 : (lt >= until ? 4 : 1 + ls);
        const uint64_t act = __ballot(1);
        const uint64_t b0 = __ballot(kind == 0), b1 = __ballot(kind == 1),
                       b2 = __ballot(kind == 2), b3 = __ballot(kind == 3);
        const uint64_t tnow = __builtin_amdgcn_s_memtime();
        if ((uint32_t)(__ffsll((long long)act) - 1) == (threadIdx.x & 63)) {
          wk[0]++;
          wk[1] += b0 != 0;
          wk[2] += b1 != 0;
          wk[3] += b2 != 0;
          wk[4] += b3 != 0;
          // (per-combination cycles: off — a global read-modify-write per iteration would
          // add a dependent round trip to every iteration of the diag build)
        }
        (void)tnow;
      }
#endif
      // inside relay_inet_out's forwarding task: its next step (the one call site of
      // forward_out_step below), no other event of the host
      if (!(fl & F_RO_CONT)) {
        int run_ls;
        if (pi < s1 && pt <= lt) {  // Packet < Local at equal times (event.rs:102-110)
          const EvRec& e = ev[ord[pi]];
          pi++;
          pt = pi < s1 ? ev[ord[pi]].time : bg ? bg->tail : INVALID;  // the next run's time, ahead of need
          now = e.time;
          if (external() && e.src == gid) {  // a CPU application's datagram (sgn_submit)
            app_submit(e);
            continue;
          }
          DG(DG_POPRUN);
          DGT_BEGIN(t0);
          // the run's packets pop back to back (nothing sorts between them); each is
          // routed into CoDel and notifies relay_inet_in, which schedules its task on
          // the first notification only (Relay::notify, relay/mod.rs:111-136)
          const uint32_t n = ev_count(e);
          const uint32_t src = e.src;
          const uint64_t eid0 = e.eid;
          c_popped += n;
          dr_add_seq<1>(now, src, eid0, n);
          if (tr())
            for (uint32_t k = 0; k < n; k++) trace(SGN_TRACE_POP, src, 0, now, 0, eid0 + k);
          // Router::route_incoming_packet (router/mod.rs:55-57)
          codel_push_run(src, eid0, ev_payload(e), e.tag, n);
          relay_notify<1>();  // Host::notify_router_has_packets (host.rs:958-960)
          DGT_END(DGT_POP, t0);
          // the relay_inet_in task at `now` is the host's next event when no packet is due at
          // `now` (Packet < Local at equal times) and no other local event precedes it by
          // (time, event id): it runs in this iteration (the same sequence of events; the wave
          // saves a trip round the loop)
          if (!next_local_now<1>(pt)) continue;
          run_ls = 1;
        } else {
          if (lt >= until) break;
          now = lt;
          run_ls = ls;
        }
        c_localev++;
        if (run_ls != 0) {
          if (run_ls == 1) {
            st1 = INVALID;
            run_forward_task<1>();
          } else {
            st2 = INVALID;
            DGT_BEGIN(t0);
            app_task();
            DGT_END(DGT_LOAD, t0);
          }
          // a send queued at `now` makes relay_inet_out's task the next event: start it here
          if (!next_local_now<0>(pt)) continue;
          c_localev++;
        }
        // run_forward_task for relay_inet_out (relay/mod.rs:166-187): Idle, then Forwarding
        st0 = INVALID;
        set_relay_state<0>(RELAY_FORWARDING);
        fl |= F_RO_CONT;
      }
      // Trains side by side (TGEN: the servers' responses): a lane whose step is a long train
      // waits while other lanes of the wave are still on other events — they may reach a train
      // of their own, and then the trains' per-packet loss draws run in one pass instead of one
      // pass per lane (config C's slowest waves ran their servers' draw loops 3 to 7 times
      // over, diag build). Waiting changes nothing of the host's own sequence: `now` is fixed
      // inside the forwarding task, and other lanes are other hosts.
      if constexpr (kApp == SGN_TRAFFIC_TGEN) {
        const bool lng = !(fl & F_RO_NEXT) && fq_len > 0 && fifo_head().count > kTrainWait;
        if (lng && __ballot(1) != act) continue;
      }
      // Forwarding side by side (PERIODIC, waves with many lanes in their loops — config D, where
      // every host sends every round): a lane about to forward waits until every lane still in
      // its event loop is about to forward too, so the wave runs the forwarding step once for
      // all of them instead of once per iteration in which some lane reaches it. Same argument as
      // the trains: `now` is fixed inside the forwarding task. Few lanes (config B's waves of 16
      // hosts, 2-6 busy) lose more in extra loop trips than they share (same-box A/B: D +6.4 %,
      // B -1.0 % when every wave waits).
      if constexpr (kApp == SGN_TRAFFIC_PERIODIC) {
        if (__popcll(act) >= kFwdWaitLanes && __ballot(1) != act) continue;
      }
      forward_out_step();
    }
    // the sub-window is done: close the digests' pending runs (sgn_workload.h)
    if (!bg || bg->flush) flush_digests();
  }
  __device__ __forceinline__ void flush_digests() {
    dr_flush_same<0>();
    dr_flush_seq<1>();
    dr_flush_seq<2>();
  }
};

// ------------------------------------------------------------------------------------
// Round kernels
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = __shfl((uint32_t)v, src, 64);
  const uint32_t hi = __shfl((uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}

// exclusive position of this lane among the lanes where m has a bit set
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  const uint32_t lane = threadIdx.x & 63;
  return (uint32_t)__popcll(lane ? (m & ((~0ULL) >> (64 - lane))) : 0ULL);
}

// The CoDel pages a round over [ws, we) may take. A page is taken only when a CoDel push
// opens a new run on a full tail page (codel_push_run), and every push is one due event run:
// a host receiving k runs takes at most ceil(k / 16) pages, so the round takes at most
// (D + 15 min(D, hosts)) / 16 for D due runs — at most the calendar's runs (occupancy) and at
// most the slabs of the buckets the window overlaps. A round edge whose free pages fall below
// this holds before the round (Ctrl::hold) and the host grows the pool: a CoDel queue never
// refuses a packet (codel_queue.rs:33,303-317 has no limit).
__host__ __device__ __forceinline__ uint64_t codel_pages_bound(uint64_t due, uint64_t hosts) {
  return (due + 15 * (due < hosts ? due : hosts) + 15) / 16;
}
__device__ __forceinline__ uint64_t codel_round_bound(const DevSim& S, uint64_t occ, uint64_t ws, uint64_t we) {
  const uint32_t nbk = ((bucket_of(S, we - 1) - bucket_of(S, ws)) & (S.NB - 1)) + 1;
  const uint64_t capb = (uint64_t)nbk * S.G * S.CAP + S.ext_total;
  return codel_pages_bound(occ < capb ? occ : capb, S.nH);
}
__device__ __forceinline__ uint64_t pages_free(uint64_t avail, uint64_t alloc) {
  return avail > alloc ? avail - alloc : 0;
}

// finalize_round for the fused single-shard path, run by the last wave of k_execute: the
// waves' minima come from the chunk slots; every value another wave changed during this
// launch is read with a device-scope atomic (plain loads could hit a stale L2 line).
// local != 0 (multi-shard): instead of moving the window, the shard's {min next event, min
// used latency} and its per-peer run counts go into the round-edge messages (comm.cpp sends
// them with the runs; k_import's last block reduces them on every shard).
__device__ void finalize_fused(const DevSim& S, uint32_t lane, uint32_t nch, uint64_t ws,
                               uint64_t we, uint32_t ks, uint32_t slab_b1, int local = 0) {
  SGN_GLB Ctrl* C = S.ctrl;
  const uint32_t b0 = bucket_of(S, ws), b1 = bucket_of(S, we - 1);
  // one round trip: every value to read (chunk minima, spare-slab minimum, bucket minima,
  // lowest used latency) is fetched at once; the buckets [b0, b1) are consumed and b1 is
  // replaced, so neither is read
  uint64_t kk = INVALID, wn = INVALID, m = INVALID, od = 0;
  for (uint32_t i = lane; i < nch; i += 64) {
    const uint64_t a = __hip_atomic_exchange(&S.fin_keep[i], (unsigned long long)INVALID,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t b = __hip_atomic_exchange(&S.fin_next[i], (unsigned long long)INVALID,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    od += __hip_atomic_exchange(&S.fin_occ[i], 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    kk = a < kk ? a : kk;
    wn = b < wn ? b : wn;
  }
  for (uint32_t b = lane; b < S.NB; b += 64) {
    const bool consumed = ((b - b0) & (S.NB - 1)) < ((b1 - b0) & (S.NB - 1)) || b == b1;
    if (!consumed) {
      const uint64_t bm = ld_dev(&S.bucket_min[b]);
      m = bm < m ? bm : m;
    }
  }
  uint64_t km = INVALID, mu = INVALID;
  if (lane == 0) {
    km = __hip_atomic_exchange(&C->keep_min, (unsigned long long)INVALID, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    mu = ld_dev(&C->min_used);
  }
  kk = wave_min_u64(kk);
  wn = wave_min_u64(wn);
  m = wave_min_u64(m);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) od += shfl_xor64(od, off);
  // then the writes (the caller drains them before publishing the round edge)
  for (uint32_t i = lane; i <= nch; i += 64) st_dev(&S.fin_cnt[i], 0u);
  if (lane == 0) {
    for (uint32_t b = b0; b != b1; b = (b + 1) & (S.NB - 1))
      st_dev(&S.bucket_min[b], (uint64_t)INVALID);  // consumed
    // the spare slab set (survivors + this round's new runs for b1) becomes bucket b1
    st_dev(&S.bucket_slab[b1], ks);
    st_dev(&C->keep_slab, slab_b1);
    const uint64_t nb1 = km < kk ? km : kk;
    st_dev(&S.bucket_min[b1], nb1);
    // CoDel page pool: the pages freed this round become allocatable in the next
    const uint64_t fr = __hip_atomic_exchange(&C->pg_freed, 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t avail = ld_dev(&C->pg_avail) + fr;
    if (fr) st_dev(&C->pg_avail, avail);
    const uint64_t occ = ld_dev(&C->cal_occ) + od;  // (wraps back from a negative sum)
    st_dev(&C->cal_occ, occ);
    const uint64_t pfree = pages_free(avail, ld_dev(&C->pg_alloc));
    const bool spilled = ld_dev(&C->spill_n) != 0;
    m = nb1 < m ? nb1 : m;
    m = wn < m ? wn : m;
    if (local) {
      // word 3: this shard's largest per-peer run count this round (every shard compares the
      // maxima of all shards with the exchange size: the same decision everywhere), with the
      // spill flag in its high half; words 4-7 let every shard evaluate every shard's CoDel
      // guard for the next window alike (k_import): free pages, calendar occupancy, runs
      // exported this round (a bound on what any shard receives), slab runs per bucket
      uint64_t xmax = 0, xsum = 0;
      for (uint32_t p = 0; p < S.n_ranks; p++) {
        const uint64_t cnt = p == S.rank ? 0 : ld_dev(&S.xout_n[p]);
        xmax = cnt > xmax ? cnt : xmax;
        xsum += cnt;
      }
      for (uint32_t p = 0; p < S.n_ranks; p++) {
        const uint64_t cnt = p == S.rank ? 0 : ld_dev(&S.xout_n[p]);
        // the message records of the peer's outgoing block (travel with the runs); this
        // shard's own in its incoming block, where k_import reads every shard's message
        SGN_GLB uint64_t* o = (SGN_GLB uint64_t*)((p == S.rank ? S.xin : S.xout) + (size_t)p * (S.xslot + XHDR));
        st_dev(o, cnt);
        st_dev(o + 1, m);
        st_dev(o + 2, mu);
        st_dev(o + 3, (uint64_t)(xmax | ((spilled ? 1ULL : 0ULL) << 32)));
        st_dev(o + 4, pfree);
        st_dev(o + 5, occ);
        st_dev(o + 6, xsum);
        st_dev(o + 7, (uint64_t)S.G * S.CAP + S.ext_total);
      }
      return;
    }
    const uint64_t min_next = m == INVALID ? EMU_MAX : m;  // unwrap_or(MAX)
    st_dev(&C->last_min_next, min_next);
    // Runahead::get (runahead.rs:44-57)
    uint64_t ra = (S.dynamic && mu != INVALID) ? mu : S.min_possible;
    ra = ra > S.runahead_cfg ? ra : S.runahead_cfg;
    // Controller::manager_finished_current_round (controller.rs:88-112)
    uint64_t ne = min_next + ra;
    if (ne < min_next || ne > EMU_MAX) ne = EMU_MAX;
    ne = ne < S.end_time ? ne : S.end_time;
    st_dev(&C->active, min_next < ne ? 1u : 0u);
    if (min_next < ne) {  // the next round's guards (hold before it runs)
      const uint64_t need = codel_round_bound(S, occ, min_next, ne);
      const uint32_t hold = (pfree < need ? HOLD_CODEL : 0u) | (spilled ? HOLD_SPILL : 0u);
      if (hold) {
        st_dev(&C->hold, hold);
        st_dev(&C->hold_need, need);
      }
    }
    st_dev(&C->prev_we, we);
    st_dev(&C->ws, min_next);
    st_dev(&C->we, ne);
    st_dev(&C->round_min, (uint64_t)INVALID);
    __hip_atomic_fetch_add(&C->rounds, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One wave per host group (GROUP consecutive hosts), lane = host. A round is:
//  1. gather: the group's slabs of the window's buckets are read; runs due in the window go
//     to LDS, the last bucket's later runs move to the spare slab (Ctrl::keep_slab);
//  2. order: counting sort of the due runs by destination lane (LDS atomics + wave scan),
//     then a rank sort inside each destination's segment by (time, src host, src event
//     id) — Shadow's EventQueue order (core/work/event.rs:84-155; keys are unique);
//  3. execute: every lane runs Host::execute (host.rs:762-830) for its host over its
//     segment and local slots, emitting new runs into the calendar / exchange slots;
//  4. the wave's minimum next local event time goes to Ctrl::round_min.
// LDS of the round kernels (one wave per workgroup)
// no-return LDS atomics on a workgroup's statistics (ds_add_u64 / ds_max_u64: the wave does not
// wait for them)
__device__ __forceinline__ void wacc_add(uint64_t* p, uint64_t v) {
  (void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void wacc_max(uint64_t* p, uint64_t v) {
  (void)__hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
struct ExecLDS {
  EvRec* lev;         // due runs of one bucket (dynamic LDS, CAP entries)
  uint16_t* lb;       // grouped by destination lane (unordered)
  uint16_t* lc;       // ... ordered inside each destination segment
  uint32_t* lcnt;
  uint32_t* lcur;     // placement cursors (after placement: segment ends, start = end - count)
  void* lslot;        // the lanes' LDS slots (LaneLDS<kApp>[64])
  uint16_t* lbs;      // bucket -> slab table for this round (when NB <= LDS_BSLAB; ids <= NB)
  OutboxHdr* ob;      // the wave's outbox (an Outbox<kApp>)
  uint32_t* bmin;     // per-bucket minima of the workgroup's sends this round (S.agg_bmin) or null
  struct BigLDS* big; // a big slab's piece state (exec_group)
  uint64_t* wacc;     // k_rounds: the workgroup's w_cnt sums (max for W_MAXFILL) over its whole
                      // launch, flushed once at its end; null: exec_group adds to w_cnt itself
};


// One group (2^gsh consecutive hosts, one per lane) through the window [ws, we):
//  1. gather: the group's slabs of the window's buckets are read; runs due in the window go
//     to LDS, the last bucket's later runs move to the spare slab set ks;
//  2. order: counting sort of the due runs by destination lane (LDS atomics + wave scan),
//     then a rank sort inside each destination's segment by (time, src host, src event
//     id) — Shadow's EventQueue order (core/work/event.rs:84-155; keys are unique);
//  3. execute: every lane runs Host::execute (host.rs:762-830) for its host over its
//     segment and local slots, emitting new runs into the calendar / exchange slots;
//  4. the group's minimum kept-event time and next local event time are returned.
// at_end(kmin, next) runs once the group's cross-workgroup data (calendar records, slab
// fills, minima) is issued and before the host records are written back: the round's
// arrival goes there, so its wait covers only what other workgroups read.
// kXb (k_rounds_x): the group's inbox bins (the runs other shards sent it last round) are read in
// the round trip of its first gather and taken into the calendar (see take_bins).
template <bool kTrace, uint32_t kApp, bool kBig, bool kXb = false, typename AtEnd>
__device__ __forceinline__ void exec_group(const DevSim& S, uint32_t g, uint64_t ws, uint64_t we, uint32_t ks,
                           const ExecLDS& X, uint64_t* kmin_out, uint64_t* next_out,
                           AtEnd&& at_end) {
  SGN_GLB Ctrl* C = S.ctrl;
  EvRec* lev = X.lev;
  uint16_t* lb = X.lb;
  uint16_t* lc = X.lc;
  uint32_t* lcnt = X.lcnt;
  uint32_t* lcur = X.lcur;
  LaneLDS<kApp>* lslot = (LaneLDS<kApp>*)X.lslot;
  uint16_t* lbs = X.lbs;
  const uint32_t lane = threadIdx.x;
  const uint32_t gsz = 1u << S.gsh;
  const uint32_t h = (g << S.gsh) + lane;  // local host index
  const bool valid = lane < gsz && h < S.nH;
  const uint32_t bs = bucket_of(S, ws), be = bucket_of(S, we - 1);
  const uint32_t nbk = ((be + S.NB - bs) & (S.NB - 1)) + 1;  // buckets overlapping the window
  const uint32_t gbase = S.lo + (g << S.gsh);  // HostId of lane 0
  const uint64_t clk0 = S.stamps ? __builtin_amdgcn_s_memtime() : 0;
#ifdef SGN_DIAG
  if (S.stamps && lane < 32) S.stamps[SGN_STAMP_WORDS * (size_t)g + 48 + lane] = 0;
  __syncthreads();
#endif
  const uint64_t rt0 = S.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
  const size_t ik = (size_t)ks * S.G + g;
  SGN_GLB EvRec* pk = S.pool + ik * S.CAP;

  uint64_t lmin = INVALID;
  uint32_t np = NO_HOST;  // PERIODIC: the next datagram's peer (store() of the host's last round)
  if (valid) {
    lmin = S.nextloc[h];
    if (kApp == SGN_TRAFFIC_PERIODIC) np = S.npeer[h];
  }
  Outbox<kApp>* ob = static_cast<Outbox<kApp>*>(X.ob);
  if (lane == 0) {
    ob->n = 0;
    ob->xmin = INVALID;
    ob->hz = SIM_START + (S.bw_div.div(ws - SIM_START) + S.NB) * S.BW;
  }
  __syncthreads();
  HostExec<kTrace, kApp> ex(S, h, we, be, ks, lslot + lane, lbs, ob, kBig ? X.big : nullptr);
  bool loaded = false;
  uint32_t N_all = 0, sorted = 0;
  uint64_t kmin = INVALID;

  uint64_t t_gather = 0, t_exec = 0;
#ifdef SGN_DIAG
  uint64_t w_load = 0, w_run = 0;
#endif
  // a big slab's passes run with the lanes' host state parked in memory: store() (its round
  // counters here), then the registers are dead until the lanes that had state reload it
  uint32_t pk_runs = 0, pk_loss = 0, pk_lev = 0, n_pieces = 0;
  uint64_t pk_bytes = 0;
  auto park = [&]() {
    if (loaded) {
      ex.store(lmin, np);
      lmin = ex.next_local_time();  // (what memory holds now)
      if (kApp == SGN_TRAFFIC_PERIODIC) np = ex.next_peer();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (its write-through stores are asm)
      pk_runs += ex.c_runs;
      pk_loss += ex.c_loss;
      pk_lev += ex.c_localev;
      pk_bytes += ex.c_bytes;
    }
    ex.kill();
  };
  // the last bucket's later runs (keep: this lane's r) move to the spare slab set: through the
  // outbox (placed with the sends after the event loop), or at once when it is full
  auto keep_runs = [&](const EvRec& r, bool keep) {
    const uint64_t km = __ballot(keep);
    if (km) {
      uint32_t k = 0;
      if (lane == 0) k = atomicAdd(&ob->n, (uint32_t)__popcll(km));
      k = __shfl(k, 0, 64) + lanes_below(km);
      if (keep) {
        kmin = r.time < kmin ? r.time : kmin;
        if (k < kObox<kApp>) {
          ob->rec[k] = r;
          ob->idx[k] = (uint32_t)ik;
        } else {
          const uint32_t base = atomicAdd(&S.slab_n[ik], 1u);
          if (base < S.CAP)
            st_dev_rec(pk + base, r);
          else
            place_overflow(S, ob, (uint32_t)ik, base, r);
        }
      }
    }
  };
  // Append the runs of one slab (fill n, its first GATHER_SPEC records already in r0) that
  // are due to lev[N..]; in the window's last bucket the runs at >= we move to the spare slab.
  auto gather_slab = [&](SGN_GLB const EvRec* pb, const EvRec& r0, uint32_t n, bool last, uint32_t& N) {
    for (uint32_t j0 = 0; j0 < n; j0 += 64) {
      const uint32_t j = j0 + lane;
      EvRec r = r0;
      if ((j0 > 0 || lane >= S.gspec) && j < n) r = ld_dev_rec(pb + j);
      const bool due = j < n && (!last || r.time < we);
      const bool keep = j < n && !due;
      const uint64_t dm = __ballot(due);
      if (due) lev[N + lanes_below(dm)] = r;
      N += (uint32_t)__popcll(dm);
      keep_runs(r, keep);
    }
  };
  // ---- a big slab (more runs than CAP: its extension, and multi-shard runs k_import spilled) ----
  // every pass reads the slab's runs from memory: the pool part, the extension, and (only when
  // the fill exceeds both) the spill area's entries tagged with this slab (f: per 64-run batch,
  // every lane; ok = the lane holds one of the slab's runs, si = its spill-area index or ~0)
  auto big_scan = [&](size_t ib, SGN_GLB const EvRec* pb, uint32_t nraw, auto&& f) {
    const uint32_t np = min(nraw, S.CAP);
    for (uint32_t j0 = 0; j0 < np; j0 += 64) {
      const uint32_t j = j0 + lane;
      EvRec r{};
      if (j < np) r = ld_dev_rec(pb + j);
      f(r, j < np, ~0ULL);
    }
    const uint64_t x = S.ext ? S.ext[ib] : 0ULL;
    const uint32_t ecap = (uint32_t)(x >> 40), ne = min(nraw - np, ecap);
    SGN_GLB const EvRec* pe = S.ext_pool + (x & EXT_OFF_MASK);
    for (uint32_t j0 = 0; j0 < ne; j0 += 64) {
      const uint32_t j = j0 + lane;
      EvRec r{};
      if (j < ne) r = ld_dev_rec(pe + j);
      f(r, j < ne, ~0ULL);
    }
    if (nraw - np > ecap) {
      const uint64_t ns = min(X.big->spill_imp, S.spill_cap);
      for (uint64_t i0 = 0; i0 < ns; i0 += 64) {
        const uint64_t i = i0 + lane;
        const bool mine = i < ns && ld_dev(&S.spill_idx[i]) == (uint32_t)ib;
        EvRec r{};
        if (mine) r = ld_dev_rec(S.spill + i);
        f(r, mine, i);
      }
    }
  };
  // big_scan over the key fields only (the radix select's passes)
  auto big_scan_keys = [&](size_t ib, SGN_GLB const EvRec* pb, uint32_t nraw, auto&& f) {
    const uint32_t np = min(nraw, S.CAP);
    for (uint32_t j0 = 0; j0 < np; j0 += 64) {
      const uint32_t j = j0 + lane;
      uint64_t t = 0, e = 0;
      uint32_t src = 0;
      if (j < np) ld_dev_key(pb + j, t, e, src);
      f(t, e, src, j < np);
    }
    const uint64_t x = S.ext ? S.ext[ib] : 0ULL;
    const uint32_t ecap = (uint32_t)(x >> 40), ne = min(nraw - np, ecap);
    SGN_GLB const EvRec* pe = S.ext_pool + (x & EXT_OFF_MASK);
    for (uint32_t j0 = 0; j0 < ne; j0 += 64) {
      const uint32_t j = j0 + lane;
      uint64_t t = 0, e = 0;
      uint32_t src = 0;
      if (j < ne) ld_dev_key(pe + j, t, e, src);
      f(t, e, src, j < ne);
    }
    if (nraw - np > ecap) {
      const uint64_t ns = min(X.big->spill_imp, S.spill_cap);
      for (uint64_t i0 = 0; i0 < ns; i0 += 64) {
        const uint64_t i = i0 + lane;
        const bool mine = i < ns && ld_dev(&S.spill_idx[i]) == (uint32_t)ib;
        uint64_t t = 0, e = 0;
        uint32_t src = 0;
        if (mine) ld_dev_key(S.spill + i, t, e, src);
        f(t, e, src, mine);
      }
    }
  };
  // first pass: the later runs of the window's last bucket move to the spare slab set; the due
  // runs' count and time range go to the piece state
  auto big_prepare = [&](size_t ib, uint32_t nraw, bool last) {
    SGN_GLB const EvRec* pb = S.pool + ib * S.CAP;
    uint64_t tmin = INVALID, tmax = 0;
    uint32_t nd = 0;
    big_scan(ib, pb, nraw, [&](const EvRec& r, bool ok, uint64_t) {
      const bool due = ok && (!last || r.time < we);
      if (due) {
        tmin = r.time < tmin ? r.time : tmin;
        tmax = r.time > tmax ? r.time : tmax;
      }
      nd += (uint32_t)__popcll(__ballot(due));
      keep_runs(r, ok && !due);
    });
    tmin = wave_min_u64(tmin);
    tmax = wave_max_u64(tmax);
    if (lane == 0) {
      X.big->tmin = tmin;
      X.big->range = nd ? tmax - tmin : 0;
      X.big->ndue = nd;
      X.big->done = 0;
      X.big->have_prev = 0;
      X.big->ib = ib;
      X.big->nraw = nraw;
      X.big->pad = last ? 1u : 0u;  // (the window's last bucket)
    }
    __syncthreads();
  };
  // The next piece into lev[0, N): the due runs with keys above the last piece's bound, up to CAP
  // of them in key order. Its bound is found by a radix select over the 160-bit key (8-bit
  // digits from the top, one pass and an LDS histogram per digit): the largest prefix range
  // holding at most CAP of the remaining keys, taken at the first digit where it holds at least
  // half of what is still wanted. Returns true for the last piece; else *bound_t = the bound's
  // time part: the piece's runs are at or before it, every later run at or after it.
  auto big_piece = [&](uint32_t& N) -> bool {
    BigLDS& B = *X.big;
    const size_t ib = uni64(B.ib);
    const uint32_t nraw = uni32(B.nraw);
    const bool last = uni32(B.pad) != 0;
    SGN_GLB const EvRec* pb = S.pool + ib * S.CAP;
    const uint64_t tmin = uni64(B.tmin);
    const bool have = uni32(B.have_prev) != 0;
    const BigKey kp = {uni64(B.kp[0]), uni64(B.kp[1]), uni64(B.kp[2])};
    const bool fin = uni32(B.ndue - B.done) <= S.CAP;
    auto in_s = [&](const EvRec& r, bool ok, BigKey& k) {
      k = big_key(r, tmin);
      return ok && (!last || r.time < we) && (!have || bk_less(kp, k));
    };
    BigKey kt = {~0ULL, ~0ULL, ~0ULL};
    if (!fin) {
      uint32_t* hist = (uint32_t*)lev;  // (lev is free until the piece is loaded)
      const uint64_t range = uni64(B.range);
      uint32_t p = range ? ((uint32_t)__builtin_clzll(range) & ~7u) : 64u;  // first digit that varies
      BigKey P = {0, 0, 0};
      uint32_t acc = 0;
      while (true) {
        for (uint32_t i = lane; i < 256; i += 64) hist[i] = 0;
        __syncthreads();
        const BigKey pm = bk_mask(p);
        big_scan_keys(ib, pb, nraw, [&](uint64_t t, uint64_t e, uint32_t src, bool ok) {
          const BigKey k = {t - tmin, ((uint64_t)src << 32) | (e >> 32), e << 32};
          if (ok && (!last || t < we) && (!have || bk_less(kp, k)) && bk_prefix_eq(k, P, pm))
            atomicAdd(&hist[bk_digit(k, p)], 1u);
        });
        __syncthreads();
        const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
        const uint32_t ls = h0 + h1 + h2 + h3;
        uint32_t incl = ls;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const uint32_t y = __shfl_up(incl, off, 64);
          if ((int)lane >= off) incl += y;
        }
        const uint32_t want = S.CAP - acc;
        const uint32_t c0 = incl - ls + h0, c1 = c0 + h1, c2 = c1 + h2, c3 = c2 + h3;
        // this lane's largest bin whose cumulative count is <= want (-1: none)
        int dl = -1;
        uint32_t cl = 0;
        if (c0 <= want) { dl = 4 * (int)lane; cl = c0; }
        if (c1 <= want) { dl = 4 * (int)lane + 1; cl = c1; }
        if (c2 <= want) { dl = 4 * (int)lane + 2; cl = c2; }
        if (c3 <= want) { dl = 4 * (int)lane + 3; cl = c3; }
        int df = dl;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          const int o = __shfl_xor(df, off, 64);
          df = o > df ? o : df;
        }
        df = (int)uni32((uint32_t)df);
        const uint32_t cf = uni32(df >= 0 ? __shfl(cl, df >> 2, 64) : 0u);
        __syncthreads();  // every lane has read the histogram
        if (df >= 0 && (2 * cf >= want || p + 8 >= 160 || df == 255)) {
          kt = bk_fill(bk_set_digit(P, p, (uint32_t)df), p + 8);
          break;
        }
        // descend into the bin that crosses: every key of the bins before it is in the piece
        acc += cf;
        P = bk_set_digit(P, p, (uint32_t)(df + 1));
        p += 8;
      }
    }
    N = 0;
    big_scan(ib, pb, nraw, [&](const EvRec& r, bool ok, uint64_t) {
      BigKey k;
      const bool sel = in_s(r, ok, k) && !bk_less(kt, k);
      const uint64_t m = __ballot(sel);
      if (sel && N + lanes_below(m) < S.CAP) lev[N + lanes_below(m)] = r;
      N += (uint32_t)__popcll(m);
    });
    bool bad = false;
    if (N > S.CAP || (!fin && N == 0)) {  // (cannot happen: the select bounds every piece by
      // CAP and takes at least one run) never silent, and the pieces end
      if (lane == 0 && (atomicOr(&C->overflow, OVF_SEG) & OVF_SEG) == 0) C->overflow_info = gbase;
      N = min(N, S.CAP);
      bad = true;
    }
    if (fin || bad) {
      // runs taken from the spill area are tagged done (the re-layout must not file them again)
      big_scan(ib, pb, nraw, [&](const EvRec&, bool ok, uint64_t si) {
        if (ok && si != ~0ULL) st_dev(&S.spill_idx[si], SPILL_DEAD);
      });
    }
    __syncthreads();
    if (lane == 0) {
      B.done = bad ? B.ndue : B.done + N;
      B.have_prev = 1;
      B.kp[0] = kt.hi;
      B.kp[1] = kt.mid;
      B.kp[2] = kt.lo;
      // the host's runs of this piece end at the bound's time T: every later run is at or after it
      B.tail = fin || bad ? INVALID : (kt.hi > EMU_MAX - tmin ? EMU_MAX : tmin + kt.hi);
      B.flush = fin || bad ? 1u : 0u;
    }
    __syncthreads();
    return fin || bad;
  };
  auto slab_done = [&](size_t ib, uint32_t n) {
    if (lane == 0) {
      st_dev(&S.slab_n[ib], 0u);  // consumed (or moved); nobody appends to it this round
      if (n && X.wacc)
        wacc_max(&X.wacc[W_MAXFILL], n);
      else if (n)
        __hip_atomic_fetch_max(&S.w_cnt[W_MAXFILL * S.G + g], (uint64_t)n, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);  // high-water mark, this wave's slot
    }
  };
  // ---- k_rounds_x: the runs other shards sent this group last round (its inbox bins) ----
  // A run for a bucket of this window goes into its slab before the gathers read it (returns
  // true: the first gather's loads are redone); a later one goes through the outbox into its
  // bucket's slab like a send, with the bucket's minimum (its first bucket is not read while
  // it is the window's: k_import's rule). bp, r: this lane's entry of the first pass (r loaded);
  // a sender whose last entry of a pass was full is read on. Taken entries are zeroed (pc 0 is
  // an empty entry) for the bin's next use two rounds later; the runs were counted in this
  // shard's occupancy at the round edge (XH_TOT).
  auto take_bins = [&](SGN_GLB EvRec* bp, EvRec r, uint32_t q, uint32_t e, bool on) -> bool {
    const uint32_t E = 1u << (S.n_ranks <= 2 ? 5u : S.n_ranks <= 4 ? 4u : 3u);
    bool slow = false;
    bool more = on;
    for (uint32_t e0 = 0;;) {
      const bool ok = more && r.pc != 0;
      if (ok) {
        SGN_GLB uint64_t* pw = (SGN_GLB uint64_t*)(bp + e0) + 3;
        if (S.xsys) st_sys(pw, 0ull); else st_dev(pw, (uint64_t)0);
        if (r.time >= ob->hz) {
          if ((atomicOr(&C->overflow, OVF_HORIZON) & OVF_HORIZON) == 0) C->overflow_info = r.dst;
        } else {
          const uint32_t b = bucket_of(S, r.time);
          const size_t idx = (size_t)lbs[b] * S.G + g;
          bool direct = ((b - bs) & (S.NB - 1)) < nbk;
          slow |= direct;
          if (!direct) {
            // (the workgroup's LDS table of bucket minima where the kernel has one, as for sends:
            // config D's ~100 k imports a round per shard would queue on a few bucket words)
            if (kAggBmin<kApp> && S.agg_bmin)
              atomicMin(&ob->bmin[b], (uint32_t)(r.time - ob->bbase));
            else
              min_nr(&S.bucket_min[b], r.time);
            const uint32_t k = atomicAdd(&ob->n, 1u);  // LDS
            if (k < kObox<kApp>) {
              ob->rec[k] = r;
              ob->idx[k] = (uint32_t)idx;
            } else {
              direct = true;
            }
          }
          if (direct) {
            const uint32_t pos = atomicAdd(&S.slab_n[idx], 1u);
            if (pos < S.CAP)
              st_dev_rec(S.pool + idx * S.CAP + pos, r);
            else
              place_overflow(S, ob, (uint32_t)idx, pos, r);
          }
        }
      }
      const uint64_t m = __ballot(ok && e == E - 1);
      e0 += E;
      if (!m || e0 >= S.xbk) break;
      more = on && ((m >> (q * E + E - 1)) & 1ull) && e0 + e < S.xbk;
      r = EvRec{};
      if (more) r = S.xsys ? ld_sys_rec(bp + e0) : ld_dev_rec(bp + e0);
    }
    return __ballot(slow) != 0;
  };
  for (uint32_t bi = 0; bi < nbk; bi++) {
    const uint64_t c0 = S.stamps ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t b = (bs + bi) & (S.NB - 1);
    bool last = bi == nbk - 1;
    uint64_t sub_end = last ? we : SIM_START + (S.bw_div.div(ws - SIM_START) + bi + 1) * S.BW;
    // ---- 1. gather the group's runs of bucket b that are due (all but the last bucket's
    //      runs at >= we, which join this round's new runs for it in the spare slab) ----
    const size_t ib = (size_t)uni32(S.NB <= LDS_BSLAB ? lbs[b] : ld_dev(&S.bucket_slab[b])) * S.G + g;
    // the slab's fill and its first GATHER_SPEC records in ONE round trip: the records are
    // loaded before the fill is known (S.gspec <= CAP; slots past the fill are ignored) — nothing
    // appends to a bucket's slab while its window runs (new runs for the window's last
    // bucket go to the spare slab set). Only GATHER_SPEC lanes load speculatively: a slab
    // holds ~4 runs on average, and loading all 64 slots pulled 2 KB of cold HBM lines per
    // slab (PMC fetch 58 -> 342 MB per launch); fuller slabs load the rest below.
    // A window that straddles one bucket boundary (the common case) loads both slabs in
    // that round trip and, when both fit one 64-run pass, runs as one sub-window: one sort,
    // one event-loop pass (the runs of the second bucket are all later than the first's).
    // (compiled into the PERIODIC kernel only: same-box A/B, config B +25 %, while C's TGEN
    // kernel — whose rounds are set by its servers' trains — measured 0.7 % slower with it)
    const bool pair = kApp == SGN_TRAFFIC_PERIODIC && bi == 0 && nbk == 2;
    SGN_GLB const EvRec* pb = S.pool + ib * S.CAP;
    EvRec r0{}, r1{};
    size_t ib1 = 0;
    SGN_GLB const EvRec* pb1 = nullptr;
    if (pair) {
      ib1 = (size_t)(S.NB <= LDS_BSLAB ? lbs[(b + 1) & (S.NB - 1)] : ld_dev(&S.bucket_slab[(b + 1) & (S.NB - 1)])) * S.G + g;
      pb1 = S.pool + ib1 * S.CAP;
    }
    // k_rounds_x: the first pass over the group's inbox bins, in the same round trip (lane =
    // sender x E + entry, E entries per sender and pass)
    const bool bins = kXb && bi == 0 && S.xin_bins != nullptr;
    const uint32_t bsh = S.n_ranks <= 2 ? 5u : S.n_ranks <= 4 ? 4u : 3u;
    const uint32_t bq = lane >> bsh, be_ = lane & ((1u << bsh) - 1);
    const bool bon = bins && bq < S.n_ranks && bq != S.rank && be_ < S.xbk;
    SGN_GLB EvRec* bp = bon ? S.xin_bins + (((size_t)(ob->xbuf ^ 1u) * S.n_ranks + bq) * S.G + g) * S.xbk + be_ : nullptr;
    EvRec br{};
    if (bon) br = S.xsys ? ld_sys_rec(bp) : ld_dev_rec(bp);
    if (lane < S.gspec) {
      r0 = ld_dev_rec(pb + lane);
      if (pair) r1 = ld_dev_rec(pb1 + lane);
    }
    uint32_t nraw_v = ld_dev(&S.slab_n[ib]);
    uint32_t n1raw_v = pair ? ld_dev(&S.slab_n[ib1]) : 0u;
    // PERIODIC traffic (configs B and D: most executed hosts have their app timer due): the
    // host record of a lane whose local event is due in the window loads in the same round trip
    // as the gather, and the app's next route is prefetched behind the sort
    const bool early = kApp == SGN_TRAFFIC_PERIODIC && bi == 0 && valid && lmin < we;
    if (early) {
      ex.load();
      ex.prefetch_peer(np);
      loaded = true;
    }
    if (bins && take_bins(bp, br, bq, be_, bon)) {
      // runs due in this window's buckets went into their slabs ahead of the gathers: the
      // first bucket's (and its pair's) loads again (spill-area entries included, big path)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (kBig && lane == 0) X.big->spill_imp = ld_dev(&C->spill_n);
      if (lane < S.gspec) {
        r0 = ld_dev_rec(pb + lane);
        if (pair) r1 = ld_dev_rec(pb1 + lane);
      }
      nraw_v = ld_dev(&S.slab_n[ib]);
      n1raw_v = pair ? ld_dev(&S.slab_n[ib1]) : 0u;
    }
    // (scalar copies after the host record's loads are issued: a readfirstlane waits for its load)
    const uint32_t nraw = uni32(nraw_v), n1raw = uni32(n1raw_v);
    // more runs than the LDS holds: the big-slab path (ordered and executed in pieces). The
    // kernels without it (kBig false: no slab extension exists, so a run past CAP went to the
    // spill area and the round edge held for the re-layout before the slab could be due) never
    // see one; if one did, it is an overflow, not a silent truncation.
    const bool big = kBig && nraw > S.CAP;
    if (!kBig && nraw > S.CAP && lane == 0) atomicOr((unsigned int*)&C->overflow, OVF_BUCKET);
    const uint32_t n = min(nraw, S.CAP);
    uint32_t N = 0;
    if (!big) {
      lcnt[lane] = 0;
      gather_slab(pb, r0, n, last, N);
      slab_done(ib, n);
      // (merged only while the pair fits one 64-run pass: config D's slabs hold ~64 runs each,
      // and merging them made its longer per-lane rank sorts cost more than the pass saved)
      if (pair && n + n1raw <= min(S.CAP, 64u)) {
        gather_slab(pb1, r1, n1raw, true, N);
        slab_done(ib1, n1raw);
        bi = 1;  // the second bucket is done: this is the window's last sub-window
        last = true;
        sub_end = we;
      }
      if (kBig && lane == 0) {  // one pass: no later packet run, digests close with it
        X.big->tail = INVALID;
        X.big->flush = 1;
      }
    } else {
      park();
      big_prepare(ib, nraw, last);
      slab_done(ib, nraw);
    }
    for (bool first = true;; first = false) {  // pieces (one unless big)
      uint64_t until = sub_end;
      bool fin = true;
      if (big) {
        if (!first) park();
        lcnt[lane] = 0;
        fin = big_piece(N);
        if (!fin) until = uni64(X.big->tail);
        n_pieces++;
        if (loaded) ex.load(false);
      }
    N_all += N;
    __syncthreads();
    // ---- 2. order: counting sort by destination lane, then rank sort by Shadow's key ----
    for (uint32_t j = lane; j < N; j += 64) atomicAdd(&lcnt[lev[j].dst - gbase], 1u);
    __syncthreads();
    const uint32_t cnt = lcnt[lane];
    uint32_t incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(incl, off, 64);
      if ((int)lane >= off) incl += y;
    }
    const uint32_t start = incl - cnt;
    lcur[lane] = start;
    __syncthreads();
    for (uint32_t j = lane; j < N; j += 64) {
      const uint32_t pos = atomicAdd(&lcur[lev[j].dst - gbase], 1u);
      lb[pos] = (uint16_t)j;
    }
    __syncthreads();
    for (uint32_t q = lane; q < N; q += 64) {
      const uint32_t idx = lb[q];
      const EvRec& r = lev[idx];
      const uint32_t d = r.dst - gbase;
      const uint32_t k = lcnt[d], a = lcur[d] - k;  // (placement left lcur at the segment's end)
      uint32_t rank = 0;
      for (uint32_t t = a; k > 1 && t < a + k; t++) {
        const EvRec& o = lev[lb[t]];
        rank += (o.time < r.time ||
                 (o.time == r.time && (o.src < r.src || (o.src == r.src && o.eid < r.eid))))
                    ? 1u : 0u;
      }
      lc[a + rank] = (uint16_t)idx;
    }
    sorted += cnt > 1 ? 1u : 0u;
    if (early && !big) ex.prefetch_route();
    __syncthreads();
    // ---- 3. execute the sub-window [.., sub_end) (a big slab's piece: up to its bound) ----
    const uint64_t c1 = S.stamps ? __builtin_amdgcn_s_memtime() : 0;
#ifdef SGN_DIAG
    // wave-level phase times (the loads are drained inside the load phase here)
    const bool go = valid && (cnt > 0 || (loaded ? ex.next_local_time() : lmin) < until);
    const uint64_t ta = __builtin_amdgcn_s_memtime();
    if (go && !loaded) {
      ex.load();
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      loaded = true;
    }
    const uint64_t tb = __builtin_amdgcn_s_memtime();
    if (go) ex.run(lev, lc, start, start + cnt, until);
    const uint64_t tc = __builtin_amdgcn_s_memtime();
    w_load += tb - ta;
    w_run += tc - tb;
#else
    const bool go = valid && (cnt > 0 || (loaded ? ex.next_local_time() : lmin) < until);
    if (go) {
      if (!loaded) {
        ex.load();
        loaded = true;
      }
      ex.run(lev, lc, start, start + cnt, until);
    }
#endif
    // a big slab's host that ran in an earlier piece closes its digest runs with the last one
    if (big && fin && !go && loaded) ex.flush_digests();
    __syncthreads();  // LDS is reused by the next piece or bucket
    if (S.stamps) {
      const uint64_t c2 = __builtin_amdgcn_s_memtime();
      t_gather += c1 - c0;
      t_exec += c2 - c1;
    }
      if (fin) break;
    }
  }

  // the outbox's records into their slabs, all lanes at once (the arrival's vmcnt(0)
  // completes them before the round edge)
  {
    const uint32_t no = min(ob->n, kObox<kApp>);
    if constexpr (kApp == SGN_TRAFFIC_PERIODIC && !kBig && !kPairOff) {  // (not with the big-slab path: registers)
      // two lanes per record, each storing one 16-byte half: the record is one 32-byte write
      // (a lane's two 16-byte write-through stores of one record are two; config D writes a
      // record per host-round, MI355X_MICROARCH.md: write-through stores and their granules)
      for (uint32_t i0 = 0; i0 < no; i0 += 32) {
        const uint32_t i = i0 + (lane >> 1), half = lane & 1;
        const bool has = i < no;
        uint32_t idx = 0, pos = 0;
        if (has) idx = ob->idx[i];
        if (has && !half) pos = atomicAdd(&S.slab_n[idx], 1u);
        pos = __shfl(pos, (int)(lane & ~1u), 64);
        if (has) {
          const EvRec& r = ob->rec[i];
          if (pos < S.CAP) {
            SGN_GLB char* q = (SGN_GLB char*)(S.pool + (size_t)idx * S.CAP + pos) + 16 * half;
            if (half)
              st_wt16(q, (uint64_t)r.src | ((uint64_t)r.dst << 32), (uint64_t)r.pc | ((uint64_t)r.tag << 32));
            else
              st_wt16(q, r.time, r.eid);
          } else if (!half) {
            place_overflow(S, ob, idx, pos, r);
          }
        }
      }
    } else {
      for (uint32_t i = lane; i < no; i += 64) {
        const uint32_t idx = ob->idx[i];
        const uint32_t pos = atomicAdd(&S.slab_n[idx], 1u);
        if (pos < S.CAP)
          st_dev_rec(S.pool + (size_t)idx * S.CAP + pos, ob->rec[i]);
        else
          place_overflow(S, ob, idx, pos, ob->rec[i]);
      }
    }
  }
  uint64_t my_min = lmin;  // a host with nothing due sleeps through the window
  if (loaded) my_min = ex.next_local_time();
  kmin = wave_min_u64(kmin);
  uint64_t m = wave_min_u64(my_min);
  m = ob->xmin < m ? ob->xmin : m;  // runs exported to other shards are pending events too
  *kmin_out = kmin;
  *next_out = m;
  // the calendar's occupancy change: runs this group appended minus the due runs it took out
  // (the last bucket's later runs moved to the spare slab set count out and in)
  const uint64_t occd = (uint64_t)wave_sum_u32((loaded ? ex.c_runs : 0u) + pk_runs) - (uint64_t)N_all;
  at_end(kmin, m, occd);
  uint32_t n_ev = 0;
#ifdef SGN_DIAG
  const uint64_t td = __builtin_amdgcn_s_memtime();
#endif
  if (loaded) {
    ex.store(lmin, np);
    n_ev = ex.c_popped + ex.c_sent + ex.c_loss + ex.c_deliv + ex.c_localev;
  }
#ifdef SGN_DIAG
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  const uint64_t w_store = __builtin_amdgcn_s_memtime() - td;
#endif
  if (S.stamps) {
    // per-wave diagnostics: shader cycles, total and max events over the wave's lanes
    const uint64_t clk1 = __builtin_amdgcn_s_memtime();
    uint32_t sum = n_ev, mx = n_ev;
    for (int off = 32; off > 0; off >>= 1) {
      sum += __shfl_xor(sum, off, 64);
      const uint32_t o = __shfl_xor(mx, off, 64);
      mx = o > mx ? o : mx;
    }
    const uint32_t busy = __popcll(__ballot(n_ev > 0));
    SGN_GLB uint64_t* st = S.stamps + SGN_STAMP_WORDS * (size_t)g;
    if (lane == 0) {
      st[0] = clk1 - clk0;
      st[1] = sum;
      st[2] = mx;
      st[3] = busy;
      st[4] = N_all;
      st[5] = t_gather;
      st[6] = t_exec;
      st[7] = rt0;  // 100 MHz constant clock: wave start / end across the chip
      st[8] = ob->n;  // records sent to this shard's calendar (past the outbox: placed at once)
      st[30] = __builtin_amdgcn_s_memrealtime();
    }
#ifdef SGN_DIAG
    for (int i = 0; i < DGT_N; i++) {
      const uint32_t v = loaded ? ex.dgt[i] : 0u;
      const uint32_t vs = wave_sum_u32(v);  // the wave's time in section i
      if (lane == 0) st[i < 16 ? 80 + i : 10 + (i - 16)] = vs;  // (sections past 15: words 10..)
    }
    if (lane == 0) {
      st[32] = w_load;
      st[33] = w_run;
      st[34] = w_store;
    }
    for (int i = 0; i < 5; i++) {
      const uint32_t v = wave_sum_u32(loaded ? ex.wk[i] : 0u);
      if (lane == 0) st[35 + i] = v;
    }
#endif
  }
  // ---- 4. hosts that ran (roofline accounting): per-wave counters, no-return adds ----
  const uint64_t ex_mask = __ballot(loaded);
  const uint32_t n_sorted = wave_sum_u32(sorted);
  const uint32_t w_loss = wave_sum_u32((loaded ? ex.c_loss : 0u) + pk_loss);
  const uint32_t w_lev = wave_sum_u32((loaded ? ex.c_localev : 0u) + pk_lev);
  uint64_t w_bytes = (loaded ? ex.c_bytes : 0) + pk_bytes;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) w_bytes += shfl_xor64(w_bytes, off);
  if (lane == 0 && X.wacc) {  // (persistent launches: per-round statistics stay in LDS; at config
    // B these ~8 small atomics per group and round were ~70 % of the round kernel's PMC writes;
    // no-return LDS atomics: this runs after the round's arrival, on the next round's path)
    wacc_add(&X.wacc[W_EXEC], (uint64_t)__popcll(ex_mask));
    wacc_add(&X.wacc[W_RUNS], N_all);
    wacc_add(&X.wacc[W_SORTED], n_sorted);
    wacc_add(&X.wacc[W_LOSS], w_loss);
    wacc_add(&X.wacc[W_LOCAL_EV], w_lev);
    wacc_add(&X.wacc[W_BYTES], w_bytes);
    if (n_pieces) wacc_add(&X.wacc[W_BIG], n_pieces);
  } else if (lane == 0) {
    const size_t G = S.G;
    if (ex_mask) cnt_add(&S.w_cnt[W_EXEC * G + g], (uint64_t)__popcll(ex_mask));
    if (N_all) cnt_add(&S.w_cnt[W_RUNS * G + g], N_all);
    if (n_sorted) cnt_add(&S.w_cnt[W_SORTED * G + g], n_sorted);
    if (w_loss) cnt_add(&S.w_cnt[W_LOSS * G + g], w_loss);
    if (w_lev) cnt_add(&S.w_cnt[W_LOCAL_EV * G + g], w_lev);
    if (w_bytes) cnt_add(&S.w_cnt[W_BYTES * G + g], w_bytes);
    if (n_pieces) cnt_add(&S.w_cnt[W_BIG * G + g], n_pieces);
  }
}

#define SGN_EXEC_LDS(X)                                                              \
  extern __shared__ __attribute__((aligned(16))) char lds_dyn[];                     \
  __shared__ uint32_t lcnt_[64], lcur_[64];                                         \
  __shared__ LaneLDS<kApp> lslot_[64];                                               \
  __shared__ uint16_t lbs_[LDS_BSLAB];                                               \
  __shared__ Outbox<kApp> ob_;                                                       \
  __shared__ BigLDS big_;                                                            \
  ExecLDS X;                                                                         \
  X.lev = (EvRec*)lds_dyn;                                                           \
  X.lb = (uint16_t*)(X.lev + S.CAP);                                                 \
  X.lc = X.lb + ((S.CAP + 3) & ~3u);                                                 \
  X.bmin = S.agg_bmin ? (uint32_t*)(lds_dyn + exec_lds_runs_bytes(S.CAP)) : nullptr;  \
  X.lcnt = lcnt_;                                                                    \
  X.lcur = lcur_;                                                                    \
  X.lslot = lslot_;                                                                  \
  X.lbs = lbs_;                                                                      \
  X.ob = &ob_;                                                                       \
  X.big = &big_;                                                                     \
  X.wacc = nullptr;                                                                  \
  if (threadIdx.x == 0) {                                                            \
    ob_.bmin = X.bmin;                                                               \
    ob_.xc = nullptr;                                                                \
    big_.spill_imp = ld_dev(&S.ctrl->spill_imp);                                     \
  }

// The workgroup's LDS table of bucket minima (S.agg_bmin): its sends of the round fold their
// delivery times there with LDS atomics; before the round's arrival every lane publishes a
// share of the table with one device atomic per touched bucket and resets it. Config D (every
// host sends to a random peer every round) otherwise puts ~1 M device atomics per round on
// the ~50 bucket words of the next 50 ms — a few cache lines — and serialises on them.
// Entries are u32 offsets from the round's window start (a delivery is below the calendar's
// horizon, at most (NB + 1) bucket widths ahead; sim_init enables the table only when that
// fits 32 bits).
template <uint32_t kApp>
__device__ __forceinline__ void init_bmin(const DevSim& S, const ExecLDS& X) {
  if (kAggBmin<kApp> && X.bmin)
    for (uint32_t i = threadIdx.x; i <= S.NB; i += blockDim.x) X.bmin[i] = 0xFFFFFFFFu;
}
template <uint32_t kApp>
__device__ __forceinline__ void flush_bmin(const DevSim& S, const ExecLDS& X) {
  if (!kAggBmin<kApp> || !X.bmin) return;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i <= S.NB; i += blockDim.x) {
    const uint32_t v = X.bmin[i];
    if (v != 0xFFFFFFFFu) {
      min_nr(i == S.NB ? X.ob->keepmin : &S.bucket_min[i], X.ob->bbase + v);
      X.bmin[i] = 0xFFFFFFFFu;
    }
  }
}

// Arrival of one workgroup at the end of a round: its minima go into its chunk's slots with
// returning device-scope atomics, then it counts itself in (64 workgroups per chunk counter,
// then chunks). Only atomics cross between workgroups (no fences: an agent-scope release
// writes the whole L2 back on gfx950). Returns true (all lanes) for the last arrival.
__device__ bool arrive(const DevSim& S, uint32_t w, uint32_t nw, uint64_t kmin, uint64_t m, uint64_t occd) {
  uint32_t last = 0;
  if (threadIdx.x == 0) {
    const uint32_t ch = w >> 6;
    const uint32_t csz = min(64u, nw - (ch << 6));
    const uint32_t nch = (nw + 63) >> 6;
    if (occd) cnt_add(&S.fin_occ[ch], occd);
    if (kmin != INVALID)
      __hip_atomic_fetch_min(&S.fin_keep[ch], (unsigned long long)kmin, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    if (m != INVALID)
      __hip_atomic_fetch_min(&S.fin_next[ch], (unsigned long long)m, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store/atomic of the round done
    const uint32_t c = __hip_atomic_fetch_add(&S.fin_cnt[ch], 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (c == csz - 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t t = __hip_atomic_fetch_add(&S.fin_cnt[nch], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      last = t == nch - 1 ? 1u : 0u;
    }
  }
  return __shfl(last, 0, 64) != 0;
}

// One round per launch: one workgroup (one wave) per group; single shard: the last arrival
// runs the round edge (finalize_fused), multi-shard: comm.cpp's exchange follows.
// kTrace: the per-packet trace compiled in (traced runs); untraced per-round launches — the
// multi-shard rounds, sgn_round, the persistent kernel's fallback — use the lean twin.
template <bool kTrace, uint32_t kApp>
__global__ __launch_bounds__(64, 2) void k_execute(const DevSim* __restrict__ Sg) {
  // the simulation constants are read from device memory where they are used (a by-value
  // kernel argument would pin ~90 scalar registers for the whole kernel)
  const DevSim& S = *Sg;
  SGN_GLB Ctrl* C = S.ctrl;
  if (!C->active || C->xspill || C->hold) return;  // a held round waits for the host
  SGN_EXEC_LDS(X)
  const uint64_t ws = C->ws, we = C->we;
  const uint32_t ks = C->keep_slab;
  if (S.NB <= LDS_BSLAB)
    for (uint32_t i = threadIdx.x; i < S.NB; i += 64) X.lbs[i] = (uint16_t)S.bucket_slab[i];
  if (threadIdx.x == 0) {
    X.ob->keepmin = &C->keep_min;
    X.ob->bbase = C->ws;
    X.ob->pg_avail = C->pg_avail;
    X.ob->pg_freed = &C->pg_freed;
    X.ob->pg_allocd = &C->rnd_alloc;
    X.ob->spilled = &C->rnd_spill;
    X.ob->xn = S.xout_n;
    X.ob->xbuf = 2;  // (the RCCL send blocks)
  }
  init_bmin<kApp>(S, X);
  __syncthreads();
  uint64_t kmin, m;
  bool last = false;
  exec_group<kTrace, kApp, true>(S, blockIdx.x, ws, we, ks, X, &kmin, &m, [&](uint64_t k, uint64_t n, uint64_t od) {
    flush_bmin<kApp>(S, X);
    last = arrive(S, blockIdx.x, gridDim.x, k, n, od);
  });
  if (!last) return;
  const uint32_t b1 = bucket_of(S, we - 1);
  // single shard: the round edge; multi-shard: the local part of it (comm.cpp finishes it)
  finalize_fused(S, threadIdx.x, (gridDim.x + 63) >> 6, ws, we, ks,
                 S.NB <= LDS_BSLAB ? X.lbs[b1] : ld_dev(&S.bucket_slab[b1]), S.fuse_finalize ? 0 : 1);
}

// ---- persistent rounds: a decentralized round edge ----
// Per round r every workgroup folds its minima (runs kept in the spare slab, next local
// events) into its chunk's slots of buffer p = r % 3, counts itself in (64 workgroups per
// chunk, then chunks), waits for the whole grid, and then computes the next window ITSELF
// from the same values (Controller::manager_finished_current_round, controller.rs:88-112):
// no workgroup publishes the edge, so the barrier costs one arrival and one observation
// instead of arrival + finalize + publish + wake-up. Shared bookkeeping is done by workgroup
// 0 during the FOLLOWING round (bucket minima of consumed buckets, the swapped bucket's new
// minimum, the global bucket -> slab table) and before the launch ends; buffer (r + 1) % 3 is
// reset by workgroup 0 during round r (its last readers passed barrier r - 1). sim_init sizes
// the calendar so no send of round r + 1 can reach a bucket consumed in round r.
constexpr uint32_t RB_CH = 64;  // chunk slots per buffer (persistent grids up to 4096 workgroups)
// Strides between chunks (u32 counters, u64 minimum pairs, u64 occupancy sums). TGEN rounds
// (config C: 1563 workgroups in 25 chunks) give every chunk its own 128-B line for each, so
// the ~4.7 k arrival atomics of a round do not queue on a few shared lines: same-box A/B on
// C 3549 -> 3513 us per 100-round launch; with config B at 16 hosts per wave (625 workgroups)
// and D at 8 workgroups per CU (2048), padding plus a poll sleep of 8 is -0.6 % on B and
// -0.3 % on D. Buffers are allocated for the padded layout.
template <uint32_t kApp> struct RbLayout {
  static constexpr bool pad = kApp != SGN_TRAFFIC_EXTERNAL;
  static constexpr uint32_t CS = pad ? 32 : 1, MS = pad ? 16 : 2, OS = pad ? 16 : 1;
  static constexpr uint32_t CB = (RB_CH + 1) * CS;  // u32 per buffer of counters (chunks, then the top)
};
constexpr uint32_t RB_CS_MAX = 32, RB_MS_MAX = 16, RB_OS_MAX = 16, RB_CB_MAX = (RB_CH + 1) * RB_CS_MAX;

template <uint32_t kApp>
__device__ __forceinline__ void rb_arrive(const DevSim& S, uint32_t p, uint32_t w, uint32_t nw, uint64_t kmin,
                                          uint64_t m, uint64_t occd) {
  if (threadIdx.x != 0) return;
  const uint32_t ch = w >> 6;
  const uint32_t csz = min(64u, nw - (ch << 6));
  using Y = RbLayout<kApp>;
  SGN_GLB uint64_t* mn = S.rb_min + ((size_t)p * RB_CH + ch) * Y::MS;
  if (kmin != INVALID) min_nr(mn, kmin);
  if (m != INVALID) min_nr(mn + 1, m);
  if (occd) cnt_add(&S.rb_occ[((size_t)p * RB_CH + ch) * Y::OS], occd);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this round's stores and atomics done
  SGN_GLB uint32_t* cnt = S.rb_cnt + (size_t)p * Y::CB;
  const uint32_t c = __hip_atomic_fetch_add(&cnt[ch * Y::CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (c == csz - 1) (void)__hip_atomic_fetch_add(&cnt[RB_CH * Y::CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The next window from buffer p after the barrier (every workgroup, identical results).
struct RbEdge {
  uint64_t ws, we, min_next, nb1;
  uint64_t occd, nalloc, nfree, nspill;  // the round's calendar occupancy change, CoDel pages
                                         // allocated / freed, runs spilled (buffer p: stable)
  uint32_t active;
};
template <uint32_t kApp>
__device__ __forceinline__ RbEdge rb_edge(const DevSim& S, uint32_t p, uint32_t nch, uint64_t ws, uint64_t we) {
  using Y = RbLayout<kApp>;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t b0 = bucket_of(S, ws), b1 = bucket_of(S, we - 1);
  // Every load of the edge is issued before any is used: one round trip. (The loop form of the
  // bucket scan — one load per 64 buckets, each waited for before the next — and the counters
  // loaded after it made the edge ~5 dependent round trips; C scans ~151 buckets.) Lanes past
  // a range load a valid word of it and ignore it; the single words are loaded by every lane
  // (one request), so no broadcast follows.
  const uint32_t nc = nch ? nch : 1u;
  SGN_GLB uint64_t* mn = S.rb_min + ((size_t)p * RB_CH + min(lane, nc - 1)) * Y::MS;
  uint64_t kk = ld_dev(mn), wn = ld_dev(mn + 1);
  uint64_t od = ld_dev(&S.rb_occ[((size_t)p * RB_CH + min(lane, nc - 1)) * Y::OS]);
  const uint64_t km = ld_dev(&S.rb_keep[p]), mu = ld_dev(&S.ctrl->min_used);
  const uint64_t na = ld_dev(&S.rb_occ[3 * RB_CH * RB_OS_MAX + p]), ns = ld_dev(&S.rb_occ[3 * RB_CH * RB_OS_MAX + 3 + p]);
  const uint64_t nf = ld_dev(&S.rb_free[p]);
  // the buckets to scan: synthetic traffic — every pending event is a delivery, so it lies in
  // [we, we + max_lat) (sends happen inside a window and arrive at most max_lat later,
  // worker.rs:386-390): only the buckets after b1 up to bucket_of(we + max_lat - 1) can hold
  // one (b1: nb1 below; C scans ~151 of its 256 buckets, B and D ~51). CPU-submitted datagrams
  // may be filed further ahead: every bucket the window has not consumed. (The persistent
  // kernels run with NB <= LDS_BSLAB = 256: at most four buckets per lane.)
  const bool ext = S.tkind == SGN_TRAFFIC_EXTERNAL;
  const uint32_t span = (b1 - b0) & (S.NB - 1);
  const uint32_t nscan = ext ? S.NB - 1 - span
                             : (uint32_t)min<uint64_t>(S.NB - 1 - span, S.bw_div.div(S.max_lat + S.BW - 1) + 1);
  uint64_t m = INVALID;
  if (nscan) {
    uint64_t bm[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; q++)
      bm[q] = ld_dev(&S.bucket_min[(b1 + 1 + min(lane + 64 * q, nscan - 1)) & (S.NB - 1)]);
#pragma unroll
    for (uint32_t q = 0; q < 4; q++)
      if (lane + 64 * q < nscan) m = bm[q] < m ? bm[q] : m;
    for (uint32_t k = lane + 256; k < nscan; k += 64) {  // (NB > 256: not on the persistent path)
      const uint64_t v = ld_dev(&S.bucket_min[(b1 + 1 + k) & (S.NB - 1)]);
      m = v < m ? v : m;
    }
  }
  if (lane >= nch) {
    kk = INVALID;
    wn = INVALID;
    od = 0;
  }
  kk = wave_min_u64(kk);
  wn = wave_min_u64(wn);
  m = wave_min_u64(m);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) od += shfl_xor64(od, off);
  RbEdge e;
  e.occd = od;
  e.nalloc = na;
  e.nfree = nf;
  e.nspill = ns;
  e.nb1 = km < kk ? km : kk;  // the spare slab set becomes bucket b1
  m = e.nb1 < m ? e.nb1 : m;
  m = wn < m ? wn : m;
  e.min_next = m == INVALID ? EMU_MAX : m;  // unwrap_or(MAX)
  // Runahead::get (runahead.rs:44-57)
  uint64_t ra = (S.dynamic && mu != INVALID) ? mu : S.min_possible;
  ra = ra > S.runahead_cfg ? ra : S.runahead_cfg;
  uint64_t ne = e.min_next + ra;
  if (ne < e.min_next || ne > EMU_MAX) ne = EMU_MAX;
  ne = ne < S.end_time ? ne : S.end_time;
  e.active = e.min_next < ne ? 1u : 0u;
  e.ws = e.min_next;
  e.we = ne;
  return e;
}

// Workgroup 0's bookkeeping of a finished round [ws, we) (lane-parallel plain stores).
__device__ __forceinline__ void rb_bookkeep(const DevSim& S, uint64_t ws, uint64_t we, uint64_t nb1,
                                            uint32_t new_keep) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t b0 = bucket_of(S, ws), b1 = bucket_of(S, we - 1);
  const uint32_t nc = (b1 - b0) & (S.NB - 1);
  for (uint32_t i = lane; i < nc; i += 64) st_dev(&S.bucket_min[(b0 + i) & (S.NB - 1)], (uint64_t)INVALID);
  if (lane == 0) {
    st_dev(&S.bucket_min[b1], nb1);
    st_dev(&S.bucket_slab[b1], new_keep);
  }
}

// Persistent rounds (single shard): the grid stays resident and runs up to max_rounds
// rounds, workgroup w serving groups w, w + P, ... every round (a group's host state stays
// with one CU). Data another workgroup wrote in this launch is read with device-scope loads
// (event records, slab fills, bucket minima, the round buffers); the rest (host records,
// queues) belongs to this workgroup's groups.
// kBig: compiled with the big-slab path (launched while some slab has an extension; without
// one, the path's code cost config C 2.6 % per launch in same-box A/B, round 4)
// The persistent kernels' per-launch state, reset by the launch itself (no host memsets before
// a launch): round buffer 0 (chunk minima, counters of both barriers, spare-slab
// minimum, freed / allocated / spilled counts, exports) and the idle-gap counter, by the shard's
// bookkeeping workgroup BEFORE it counts itself into the residency census — every workgroup
// waits for the whole census, so no arrival can reach the buffers first. Buffers 1 and 2 are
// reset during rounds 0 and 1 as before.
template <uint32_t kApp>
__device__ __forceinline__ void rb_reset0(const DevSim& S, uint32_t nch) {
  using Y = RbLayout<kApp>;
  for (uint32_t i = threadIdx.x; i < nch; i += 64) {
    st_dev(&S.rb_min[(size_t)i * Y::MS], (uint64_t)INVALID);
    st_dev(&S.rb_min[(size_t)i * Y::MS + 1], (uint64_t)INVALID);
    st_dev(&S.rb_occ[(size_t)i * Y::OS], (uint64_t)0);
  }
  for (uint32_t i = threadIdx.x; i <= nch; i += 64) {
    const size_t o = (size_t)(i == nch ? RB_CH : i) * Y::CS;
    st_dev(&S.rb_cnt[o], 0u);
    if (S.rb2_cnt) st_dev(&S.rb2_cnt[o], 0u);
  }
  if (S.xout_n)
    for (uint32_t i = threadIdx.x; i < S.n_ranks; i += 64) {
      st_dev(&S.xout_n[i], 0u);
      st_dev(&S.xout_n[3 * S.n_ranks + i], 0u);  // (k_rounds_x: the per-peer totals)
    }
  if (threadIdx.x == 0) {
    st_dev(&S.rb_keep[0], (uint64_t)INVALID);
    st_dev(&S.rb_free[0], (uint64_t)0);
    st_dev(&S.rb_occ[3 * RB_CH * RB_OS_MAX], (uint64_t)0);
    st_dev(&S.rb_occ[3 * RB_CH * RB_OS_MAX + 3], (uint64_t)0);
    st_dev(&S.rb_cnt[3 * RB_CB_MAX], 0u);  // the idle-gap barrier's counter
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// A workgroup of k_rounds that gives up on a barrier (OVF_TIMEOUT) may do so after the
// bookkeeping workgroup copied the control block into host memory: it also marks the copy
// stale (the word after the epoch), and the host then reads the device's block.
static_assert(sizeof(Ctrl) % 8 == 0, "the control block is copied as 8-byte words");
constexpr uint32_t kMirrorWords = sizeof(Ctrl) / 8 + 2;  // the block, the epoch, the stale mark
__device__ __forceinline__ void fail_timeout(const DevSim& S) {
  atomicOr((unsigned int*)&S.ctrl->overflow, OVF_TIMEOUT);
  if (S.ctrl_mirror) st_sys(&S.ctrl_mirror[kMirrorWords - 1], 1ull);
}

// Residency census (thread 0 of each workgroup): the workgroup counts itself in and waits,
// bounded, for the whole grid of P; the first to see it, or to give up, sets the verdict with a
// compare-and-swap, so every workgroup acts on the same one. The arrival counter is never reset
// (the host passes its value before the launch, base) and the verdict carries the launch's epoch
// (epoch << 2 | verdict: 1 resident, 2 not). *decided: this workgroup set it.
__device__ __forceinline__ uint32_t census(SGN_GLB Ctrl* C, uint32_t P, uint32_t epoch, uint32_t base,
                                           bool* decided) {
  __hip_atomic_fetch_add(&C->res_arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t want = epoch << 2;
  uint32_t v = 0, spins = 0;
  *decided = false;
  while (((v = ld_dev(&C->res_verdict)) & ~3u) != want) {
    uint32_t nv;
    if (ld_dev(&C->res_arrive) - base >= P) {
      nv = want | 1u;
    } else if (++spins > (1u << 14)) {
      nv = want | 2u;
    } else {
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    uint32_t expect = v;
    if (__hip_atomic_compare_exchange_strong(&C->res_verdict, &expect, nv, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      *decided = true;
  }
  return v & 3u;
}

template <uint32_t kApp, bool kBig>
__global__ __launch_bounds__(64, 2) void k_rounds(const DevSim* __restrict__ Sg, uint32_t max_rounds, uint32_t epoch,
                                                  uint32_t res_base) {
  const DevSim& S = *Sg;
  SGN_GLB Ctrl* C = S.ctrl;
  SGN_EXEC_LDS(X)
  // PERIODIC (configs B, D): the per-wave statistics in LDS for the launch (B: ~70 % of the
  // PMC writes were their per-round atomics); TGEN keeps the per-round no-return adds (config
  // C: 0.45 % faster per launch without the LDS accumulator, same-box A/B)
  if constexpr (kApp == SGN_TRAFFIC_PERIODIC) {
    __shared__ uint64_t wacc_[W_N];
    X.wacc = wacc_;
    if (threadIdx.x < W_N) wacc_[threadIdx.x] = 0;
  }
  const uint32_t w = blockIdx.x, P = gridDim.x;
  // The workgroup's groups: [gq0, gq1) in steps of gqs. TGEN: w, w + P, ... (config C's server
  // groups come first in slot order and set the round's chain: dealt over every XCD). PERIODIC:
  // XCD-aware — workgroups are dealt round-robin over the 8 XCDs (blockIdx % 8; observed, used
  // for speed only), so the ones sharing blockIdx % 8 take one contiguous eighth of the groups.
  // Slots are ordered by graph node (sim_init), so an XCD's hosts cover an eighth of the nodes
  // and their sends read an eighth of the route table's rows (config D: 2 of 16 MB, L2-resident).
  // Any fixed bijection works: a group's records belong to its workgroup for the launch.
  uint32_t gq0 = w, gq1 = S.G, gqs = P;
  if constexpr (kApp == SGN_TRAFFIC_PERIODIC) {
    const uint32_t x = w & 7u, cx = (P - x + 7u) >> 3;  // this class's workgroups
    uint32_t before = 0;                                 // workgroups of the classes below x
    for (uint32_t y = 0; y < x; y++) before += (P - y + 7u) >> 3;
    const uint32_t s0 = (uint32_t)((uint64_t)S.G * before / P), s1 = (uint32_t)((uint64_t)S.G * (before + cx) / P);
    gq0 = s0 + (w >> 3);
    gq1 = s1;
    gqs = cx;
  }
  // Residency census before any simulation state is touched: the grid barrier below needs
  // every workgroup on the chip at once. Each workgroup counts itself in and waits (bounded)
  // for the rest; the first to see the whole grid, or to give up, sets the verdict with a
  // compare-and-swap, so all workgroups act on the same one. A grid that is not resident
  // leaves untouched and the host runs the rounds with per-round launches instead.
  {
    __shared__ uint32_t verdict;
    if (w == P - 1) rb_reset0<kApp>(S, (P + 63) >> 6);
    if (threadIdx.x == 0) {
      bool decided;
      verdict = census(C, P, epoch, res_base, &decided);
    }
    __syncthreads();
    if (verdict != 1) return;
  }
  const uint32_t nch = (P + 63) >> 6;
  // the workgroup that does the shared bookkeeping (the previous round's bucket minima and
  // slab table, the next round buffer's reset, the control block): the last one, whose group
  // is a client group (slots start with the TGEN servers, whose groups are the slowest)
  const uint32_t wbk = P - 1;
  // The round state every workgroup keeps for itself, in LDS (registers are the scarce
  // resource of the round kernel): the window, the spare slab, and the previous round's
  // bookkeeping that workgroup 0 does during the next round. The bucket -> slab table
  // changes by one swap per round, applied by every workgroup to its own LDS copy.
  struct RoundLDS {
    uint64_t ws, we, pend_ws, pend_we, pend_nb1, pg_avail;
    uint64_t pg_alloc, occ, nspill, hold_need;  // CoDel pages taken, calendar runs, runs spilled
    uint32_t active, ks, pend_new, pend, ngap, hold;
  };
  __shared__ RoundLDS rs;
  if (threadIdx.x == 0) {
    rs.pg_avail = ld_dev(&C->pg_avail);
    rs.ws = ld_dev(&C->ws);
    rs.we = ld_dev(&C->we);
    rs.active = ld_dev(&C->active);
    rs.ks = ld_dev(&C->keep_slab);
    rs.pend = 0;
    rs.ngap = 0;
    rs.pg_alloc = ld_dev(&C->pg_alloc);
    rs.occ = ld_dev(&C->cal_occ);
    rs.nspill = ld_dev(&C->spill_n);
    rs.hold = ld_dev(&C->hold);  // (a round still held: the launch returns at once)
    rs.hold_need = ld_dev(&C->hold_need);
  }
  // (the launch's first round number is read back at its end: nothing else writes it, and a
  // register live across the whole launch spilled the PERIODIC big-slab kernel)
  const bool lds_tab = S.NB <= LDS_BSLAB;
  if (lds_tab)
    for (uint32_t i = threadIdx.x; i < S.NB; i += 64) X.lbs[i] = (uint16_t)ld_dev(&S.bucket_slab[i]);
  init_bmin<kApp>(S, X);
  __syncthreads();
  uint32_t r = 0;
  for (; r < max_rounds; r++) {
    // (a held round: the host grows a pool between launches, then the round runs)
    if (!__builtin_amdgcn_readfirstlane((int)rs.active) || __builtin_amdgcn_readfirstlane((int)rs.hold)) break;
    const uint64_t ws = uni64(rs.ws), we = uni64(rs.we);
    const uint32_t ks = (uint32_t)__builtin_amdgcn_readfirstlane((int)rs.ks);
    const uint32_t p = r % 3;
    if (w == wbk) {
      if (rs.pend) rb_bookkeep(S, rs.pend_ws, rs.pend_we, rs.pend_nb1, rs.pend_new);
      // reset buffer (r + 1) % 3 for the next round
      const uint32_t q = (r + 1) % 3;
      for (uint32_t i = threadIdx.x; i < nch; i += 64) {
        st_dev(&S.rb_min[((size_t)q * RB_CH + i) * RbLayout<kApp>::MS], (uint64_t)INVALID);
        st_dev(&S.rb_min[((size_t)q * RB_CH + i) * RbLayout<kApp>::MS + 1], (uint64_t)INVALID);
        st_dev(&S.rb_occ[((size_t)q * RB_CH + i) * RbLayout<kApp>::OS], (uint64_t)0);
      }
      for (uint32_t i = threadIdx.x; i <= nch; i += 64)  // the grid's chunks, then the top counter
        st_dev(&S.rb_cnt[(size_t)q * RbLayout<kApp>::CB + (i == nch ? RB_CH : i) * RbLayout<kApp>::CS], 0u);
      if (threadIdx.x == 0) {
        st_dev(&S.rb_keep[q], (uint64_t)INVALID);
        st_dev(&S.rb_free[q], (uint64_t)0);
        st_dev(&S.rb_occ[3 * RB_CH * RB_OS_MAX + q], (uint64_t)0);
        st_dev(&S.rb_occ[3 * RB_CH * RB_OS_MAX + 3 + q], (uint64_t)0);
      }
    }
    // diagnostics (SGN_STAMPS): per round of this launch, {earliest start, latest arrival,
    // round edge known} on the 100 MHz clock
    SGN_GLB uint64_t* rd = S.rdbg ? S.rdbg + 3 * (size_t)(r & 127) : nullptr;
    if (rd && threadIdx.x == 0)
      __hip_atomic_fetch_min(rd, (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) {
      X.ob->keepmin = &S.rb_keep[p];
      X.ob->bbase = ws;
      X.ob->pg_avail = rs.pg_avail;
      X.ob->pg_freed = &S.rb_free[p];
      X.ob->pg_allocd = &S.rb_occ[3 * RB_CH * RB_OS_MAX + p];
      X.ob->spilled = &S.rb_occ[3 * RB_CH * RB_OS_MAX + 3 + p];
    }
    uint64_t kall = INVALID, mall = INVALID, oall = 0;
    bool arrived = false;
    for (uint32_t g = gq0; g < gq1; g += gqs) {
      uint64_t kmin, m;
      const bool lastg = g + gqs >= gq1;  // the workgroup's last group arrives
      exec_group<false, kApp, kBig>(S, g, ws, we, ks, X, &kmin, &m, [&](uint64_t k, uint64_t n, uint64_t od) {
        kall = k < kall ? k : kall;
        mall = n < mall ? n : mall;
        oall += od;
        if (lastg) {
          if (rd && threadIdx.x == 0)
            __hip_atomic_fetch_max(rd + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          flush_bmin<kApp>(S, X);
          rb_arrive<kApp>(S, p, w, P, kall, mall, oall);
          arrived = true;
        }
      });
      __syncthreads();
    }
    if (!arrived) rb_arrive<kApp>(S, p, w, P, INVALID, INVALID, 0);  // a workgroup without groups
    // grid barrier: every chunk complete, bounded
    uint32_t spins = 0;
    bool ok = true;
    while (ld_dev(&S.rb_cnt[(size_t)p * RbLayout<kApp>::CB + RB_CH * RbLayout<kApp>::CS]) < nch) {
      // (TGEN: 1563 workgroups poll one word; a longer sleep between polls leaves the memory
      // side to the last arrivals' atomics: same-box A/B on C, 3639 -> 3586 us per 100-round
      // launch; PERIODIC: 8, see RbLayout)
      __builtin_amdgcn_s_sleep(kApp == SGN_TRAFFIC_TGEN ? 16 : kApp == SGN_TRAFFIC_PERIODIC ? 8 : 1);
      if (++spins > (1u << 22)) {
        ok = false;
        break;
      }
    }
    if (!ok) {
      if (threadIdx.x == 0) fail_timeout(S);
      return;
    }
    asm volatile("" ::: "memory");
    const RbEdge e = rb_edge<kApp>(S, p, nch, ws, we);
    if (rd && w == wbk && threadIdx.x == 0) st_dev(rd + 2, (uint64_t)__builtin_amdgcn_s_memrealtime());
    // This round's bucket bookkeeping (consumed minima -> INVALID, bucket b1 -> nb1) is done by
    // workgroup 0 during the next round, with plain stores: safe while the next round's sends
    // cannot reach this round's buckets. They can after an idle gap: a send at t maps to this
    // round's bucket indices again once t >= bucketstart(ws) + NB * BW, and t < we' + max_lat.
    // Then (every workgroup decides alike) workgroup 0 does it now and a second grid barrier
    // keeps every send of the next round behind it (a lost bucket minimum).
    const uint64_t span = (uint64_t)S.NB * S.BW;
    const uint64_t bstart = SIM_START + S.bw_div.div(ws - SIM_START) * S.BW;
    const bool gap = e.active && (e.we + S.max_lat >= bstart + span || e.we + S.max_lat < e.we);
    if (gap) {
      if (w == wbk) rb_bookkeep(S, ws, we, e.nb1, ks);  // (the previous round's: done at this round's start)
      if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // workgroup 0's stores are done
        SGN_GLB uint32_t* gc = S.rb_cnt + 3 * RB_CB_MAX;
        const uint32_t target = (rs.ngap + 1) * P;
        __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t sp = 0;
        while (ld_dev(gc) < target && ++sp < (1u << 24)) __builtin_amdgcn_s_sleep(2);
        if (sp >= (1u << 24)) fail_timeout(S);
        rs.ngap++;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      // the spare slab set (survivors + this round's new runs for b1) becomes bucket b1
      const uint32_t b1 = bucket_of(S, we - 1);
      const uint32_t slab_b1 = lds_tab ? X.lbs[b1] : ld_dev(&S.bucket_slab[b1]);
      if (lds_tab) X.lbs[b1] = (uint16_t)ks;
      rs.pend = gap ? 0u : 1u;
      rs.pend_ws = ws;
      rs.pend_we = we;
      rs.pend_nb1 = e.nb1;
      rs.pend_new = ks;
      rs.ks = slab_b1;
      rs.ws = e.ws;
      rs.we = e.we;
      rs.active = e.active;
      rs.pg_avail += e.nfree;  // this round's freed pages (all written: barrier)
      rs.pg_alloc += e.nalloc;
      rs.occ += e.occd;
      rs.nspill += e.nspill;
      if (e.active) {  // the next round's guards: every workgroup decides alike (same values)
        const uint64_t need = codel_round_bound(S, rs.occ, e.ws, e.we);
        rs.hold = (pages_free(rs.pg_avail, rs.pg_alloc) < need ? HOLD_CODEL : 0u) | (rs.nspill ? HOLD_SPILL : 0u);
        rs.hold_need = need;
      }
      if (w == wbk) {
        st_dev(&C->last_min_next, e.min_next);
        st_dev(&C->prev_we, we);
      }
    }
    __syncthreads();
  }
  // the launch's per-wave statistics, in the slot of this workgroup's first group (the host sums
  // the slots; the mapping is a bijection, so gq0 < G is this workgroup's alone — a forced grid
  // larger than G has workgroups w >= G; one without groups has nothing to flush)
  __syncthreads();
  if (X.wacc && threadIdx.x < W_N && X.wacc[threadIdx.x] && gq0 < gq1) {
    const uint32_t k = threadIdx.x;
    if (k == W_MAXFILL)
      __hip_atomic_fetch_max(&S.w_cnt[k * S.G + gq0], X.wacc[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      cnt_add(&S.w_cnt[k * S.G + gq0], X.wacc[k]);
  }
  // the last round's bookkeeping and the host-visible control block
  if (w == wbk) {
    if (rs.pend) rb_bookkeep(S, rs.pend_ws, rs.pend_we, rs.pend_nb1, rs.pend_new);
    if (threadIdx.x == 0) {
      st_dev(&C->keep_slab, rs.ks);
      st_dev(&C->ws, rs.ws);
      st_dev(&C->we, rs.we);
      st_dev(&C->active, rs.active);
      st_dev(&C->rounds, ld_dev(&C->rounds) + r);
      st_dev(&C->pg_avail, rs.pg_avail);
      st_dev(&C->cal_occ, rs.occ);
      if (rs.hold) {
        st_dev(&C->hold, rs.hold);
        st_dev(&C->hold_need, rs.hold_need);
      }
    }
    // ... and its copy in host memory: after the last barrier no other workgroup writes the
    // control block (their counters and flags arrived with them)
    if (S.ctrl_mirror) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      constexpr uint32_t NW = sizeof(Ctrl) / 8;
      for (uint32_t i = threadIdx.x; i < NW; i += 64) st_sys(&S.ctrl_mirror[i], ld_dev(&((SGN_GLB uint64_t*)C)[i]));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (threadIdx.x == 0) st_sys(&S.ctrl_mirror[NW], (uint64_t)epoch);
    }
  }
}

// ---- persistent multi-shard rounds (k_rounds_x) ----
// N shards, each on its own GPU (one launch per GPU) or, for the one-GPU rehearsal, on its own
// range of workgroups of ONE launch. A round of shard s is the single-shard persistent round
// (k_rounds) plus the exchange that replaces the RCCL send/recv and k_import:
//  1. execute: runs for another shard's hosts go straight into that shard's inbox slot for this
//     shard and round parity (peer-mapped memory, system-scope write-through stores), counted
//     per peer in local counters (Worker::send_packet pushes into the destination host's queue
//     from any thread: core/worker.rs:603-613);
//  2. the local barrier (k_rounds' chunk counters) and the local round edge (rb_edge: this
//     shard's minima, the runs it exported included);
//  3. the shard's last workgroup writes one 128-B message per shard (its own included) into the
//     receivers' inboxes — run count, min next event, min used latency, the pool figures every
//     shard needs for the same hold decisions — and then, after every store has completed, the
//     message's tag (the global round number);
//  4. every workgroup waits for the N messages of its own inbox and computes the next window
//     from them: the min over messages is the min over all pending events (each message counts
//     its shard's, exported runs included), i.e. the RCCL min all-reduce of the north star and
//     Controller::manager_finished_current_round (controller.rs:88-112) over the global min;
//  5. the workgroups file the runs of their inbox into the local calendar (k_import's work) and
//     meet at a second local barrier before the next round's gathers read the slabs.
// Inbox slots alternate by round parity: a sender writes round r + 1's runs while the receiver
// may still be filing round r's. Rounds that would need more than a slot, or a larger pool, or a
// re-layout, are held on every shard alike (the same messages, the same decisions) and the host
// completes them between launches.
constexpr uint32_t XR_MAX = 8;  // shards of a persistent multi-shard run (one MI355X node)
// The round-edge messages across GPUs: a system-scope release before them (kept: it costs
// nothing measurable), and no system-scope acquire after them. The acquire (buffer_inv sc0 sc1
// in every workgroup, every round) cost 9 us per round on the two-process rehearsal (41.6 ->
// 50.6 us, profiles/r06/xfence_ab.txt), and every byte it would order is read by system-coherent
// loads anyway: the tags by an asm global_load sc0 sc1 followed by s_waitcnt vmcnt(0), so every
// later load issues after the tag was read, and the bins and slots by sc0 sc1 loads of uncached
// memory (no cache can hold an older copy). SGN_XACQ builds it in (for that price), SGN_XNOFENCE
// builds neither (experiments only, build_exp.sh).
#ifdef SGN_XNOFENCE
constexpr bool kXFenceRel = false, kXFenceAcq = false;
#elif defined(SGN_XACQ)
constexpr bool kXFenceRel = true, kXFenceAcq = true;
#else
constexpr bool kXFenceRel = true, kXFenceAcq = false;
#endif
#ifdef SGN_KX_NOBIG  // cost experiment only (build_exp.sh): k_rounds_x without the big-slab path
constexpr bool kKxBig = false;
#else
constexpr bool kKxBig = true;
#endif
// imports of a round up to this many runs are filed by their own workgroups at the next round's
// start (each workgroup scans them all: ~64 KB), more are shared out before a second barrier
// (DevSim::xown; SGN_XOWN: a test hook, 0 = always shared)
constexpr uint32_t kOwnFile = 2048;
// inbox bins: runs per (round parity, sender, receiving host group). Config C at 8 shards sends
// a group ~0.6 runs per sender and round, config D ~8; a fuller bin sends the rest to the slot.
constexpr uint32_t kXBin = 32;
// shards of up to this many workgroups arrive on one counter (k_rounds' chunk counters take
// two returning atomics for the last arrival; at config C's ~200 workgroups per shard, spread
// over the round's ~15 us of arrivals, one counter does not queue)
constexpr uint32_t kXFlat = 256;
constexpr uint64_t kXWaitTicks = 2000000000ull;  // 20 s on the 100 MHz clock: a peer that never
                                                 // answers is an error (OVF_TIMEOUT), not a hang
// the census across GPUs: 60 s, so that shards whose launches start far apart (one of them
// re-laying its calendar out or growing a pool first) wait instead of failing
constexpr uint64_t kXCensusTicks = 6000000000ull;

template <uint32_t kApp>
__device__ __forceinline__ bool rb_wait(SGN_GLB uint32_t* top, uint32_t nch) {
  uint32_t spins = 0;
  while (ld_dev(top) < nch) {
    __builtin_amdgcn_s_sleep(kApp == SGN_TRAFFIC_TGEN ? 16 : kApp == SGN_TRAFFIC_PERIODIC ? 8 : 1);
    if (++spins > (1u << 22)) return false;
  }
  return true;
}

// the second local barrier (after the imports): chunk counters, then the top counter
template <uint32_t kApp>
__device__ __forceinline__ void rb2_arrive(const DevSim& S, uint32_t p, uint32_t w, uint32_t nw) {
  if (threadIdx.x != 0) return;
  using Y = RbLayout<kApp>;
  const uint32_t ch = w >> 6;
  const uint32_t csz = min(64u, nw - (ch << 6));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's imports are in place
  SGN_GLB uint32_t* cnt = S.rb2_cnt + (size_t)p * Y::CB;
  const uint32_t c = __hip_atomic_fetch_add(&cnt[ch * Y::CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (c == csz - 1) (void)__hip_atomic_fetch_add(&cnt[RB_CH * Y::CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the local arrival of k_rounds_x (k_rounds' chunk counters): *last = 1 for the workgroup whose
// count completes the shard's barrier (it computes the round edge and sends the messages)
template <uint32_t kApp>
__device__ __forceinline__ void rb_arrive_x(const DevSim& S, uint32_t p, uint32_t w, uint32_t nw, uint64_t kmin,
                                            uint64_t m, uint64_t occd, uint32_t* last, const uint32_t* xc) {
  // this workgroup's runs per peer this round (LDS, bins and slots) into the shard's totals
  if (xc && threadIdx.x < S.n_ranks && threadIdx.x != S.rank) {
    const uint32_t v = xc[threadIdx.x];
    if (v)
      (void)__hip_atomic_fetch_add(&S.xout_n[(size_t)(3 + p) * S.n_ranks + threadIdx.x], v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x != 0) return;
  const uint32_t ch = w >> 6;
  const uint32_t csz = min(64u, nw - (ch << 6));
  const uint32_t nch = (nw + 63) >> 6;
  using Y = RbLayout<kApp>;
  SGN_GLB uint64_t* mn = S.rb_min + ((size_t)p * RB_CH + ch) * Y::MS;
  if (kmin != INVALID) min_nr(mn, kmin);
  if (m != INVALID) min_nr(mn + 1, m);
  if (occd) cnt_add(&S.rb_occ[((size_t)p * RB_CH + ch) * Y::OS], occd);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this round's stores and atomics done
  SGN_GLB uint32_t* cnt = S.rb_cnt + (size_t)p * Y::CB;
  uint32_t l = 0;
  if (nw <= kXFlat) {  // one counter: the last arrival learns it in one round trip
    l = __hip_atomic_fetch_add(&cnt[RB_CH * Y::CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nw - 1 ? 1u : 0u;
  } else {
    const uint32_t c = __hip_atomic_fetch_add(&cnt[ch * Y::CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c == csz - 1)
      l = __hip_atomic_fetch_add(&cnt[RB_CH * Y::CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nch - 1 ? 1u : 0u;
  }
  *last = l;
}

// a 16-byte message granule {value, tag}: one load (device scope: sc1; system: sc0 sc1)
__device__ __forceinline__ u64x2 ld_gran16(SGN_GLB const uint64_t* p, bool sys) {
  u64x2 v;
  if (sys)
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"((uint64_t)p) : "memory");
  else
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"((uint64_t)p) : "memory");
  return v;
}

template <uint32_t kApp>
__global__ __launch_bounds__(64, 2) void k_rounds_x(const XLaunch* __restrict__ L, uint32_t max_rounds) {
  // this workgroup's shard and its place in the shard's range
  const uint32_t nl = L->n_local;
  uint32_t si = 0;
  while (si + 1 < nl && blockIdx.x >= L->base[si + 1]) si++;
  const DevSim& S = *(const DevSim*)L->S[si];
  SGN_GLB Ctrl* C = S.ctrl;
  const uint32_t w_i = blockIdx.x - L->base[si], P_i = L->base[si + 1] - L->base[si];
  SGN_EXEC_LDS(X)
  if constexpr (kApp == SGN_TRAFFIC_PERIODIC) {
    __shared__ uint64_t wacc_[W_N];
    X.wacc = wacc_;
    if (threadIdx.x < W_N) wacc_[threadIdx.x] = 0;
  }
  // the workgroup's groups, as in k_rounds
  uint32_t gq0_i = w_i, gq1_i = S.G, gqs_i = P_i;
  if constexpr (kApp == SGN_TRAFFIC_PERIODIC) {
    const uint32_t x = w_i & 7u, cx = (P_i - x + 7u) >> 3;
    uint32_t before = 0;
    for (uint32_t y = 0; y < x; y++) before += (P_i - y + 7u) >> 3;
    const uint32_t s0 = (uint32_t)((uint64_t)S.G * before / P_i), s1 = (uint32_t)((uint64_t)S.G * (before + cx) / P_i);
    gq0_i = s0 + (w_i >> 3);
    gq1_i = s1;
    gqs_i = cx;
  }
  const uint32_t w = w_i, P = P_i, gq0 = gq0_i, gq1 = gq1_i, gqs = gqs_i;
  const uint32_t R = S.n_ranks, me = S.rank;
  const uint32_t nch = (P + 63) >> 6;
  const uint32_t wbk = P - 1;  // this shard's bookkeeping workgroup (and its messages)
  // residency census over the whole launch (the control block of its first shard), then, one
  // shard per GPU, over the shards: every shard publishes its verdict to every inbox and waits for
  // all of them — a grid that is not resident anywhere makes every shard fall back alike
  {
    __shared__ uint32_t verdict;
    SGN_GLB Ctrl* C0 = L->S[0]->ctrl;
    const uint32_t ep32 = (uint32_t)L->epoch << 2;
    if (w == P - 1 && !L->refuse) rb_reset0<kApp>(S, (P + 63) >> 6);
    if (threadIdx.x == 0) {
      bool decided = true;
      // (a refused launch is one workgroup on a GPU that cannot hold the grid: it only tells the
      // peers, so that every shard falls back together — ADVICE r5)
      uint32_t v = L->refuse ? 2u : census(C0, gridDim.x, (uint32_t)L->epoch, L->res_base, &decided);
      if (L->refuse) st_dev(&C->res_verdict, ep32 | 2u);
      if (L->peers_census) {
        const uint64_t ep = L->epoch << 2;
        if (decided) {
          // the deciding workgroup tells every shard (its own inbox too), then combines the
          // peers' verdicts for its whole shard under ONE deadline: a peer that is not resident,
          // or never answers, stops this shard too
          for (uint32_t q = 0; q < R; q++) st_sys(S.xp[q].cen, ep | v);
          if (v == 1) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (uint32_t q = 0; q < R && v == 1; q++) {
              uint64_t c;
              while (((c = ld_sys(&S.xin_cen[q])) >> 2) != L->epoch) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > kXCensusTicks) {
                  c = ep | 2;
                  atomicOr((unsigned int*)&C->overflow, OVF_TIMEOUT);
                  break;
                }
                __builtin_amdgcn_s_sleep(8);
              }
              if ((c & 3) != 1) v = 3;
            }
          }
          st_dev(&C->res_xverdict, ep32 | v);
        } else if (v == 1) {
          // the other workgroups act on the decider's combined verdict only (its deadline, then
          // a margin: they never time out on their own before it does)
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          uint32_t c;
          while (((c = ld_dev(&C->res_xverdict)) & ~3u) != ep32) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 2 * kXCensusTicks) {
              c = ep32 | 3u;
              atomicOr((unsigned int*)&C->overflow, OVF_TIMEOUT);
              break;
            }
            __builtin_amdgcn_s_sleep(8);
          }
          v = c & 3u;
        }
      }
      verdict = v;
    }
    __syncthreads();
    if (verdict != 1) {
      if (verdict == 3 && w == P - 1 && threadIdx.x == 0) st_dev(&C->res_verdict, ep32 | 3u);
      return;
    }
  }
  struct RoundLDS {
    uint64_t ws, we, pend_ws, pend_we, pend_nb1, pg_avail;
    uint64_t pg_alloc, occ, hold_need;
    uint32_t active, ks, pend, pend_new, ngap, hold;
    // runs to file from the inbox slots this round: in all, and from each shard (nin, from the
    // exchange until they are filed); while the workgroup executes, nin counts its runs to each
    // shard instead (OutboxHdr::xc; reset after the filing, flushed at the arrival)
    uint32_t n_in, nin[XR_MAX];
    uint32_t fpend, fbuf;        // imports left for the next round's start (and their slot parity;
                                 // their horizon: the round pend_ws started)
    uint32_t last;               // this workgroup arrived last at the shard's local barrier
  };
  __shared__ RoundLDS rs;
  if (threadIdx.x == 0) {
    rs.pg_avail = ld_dev(&C->pg_avail);
    rs.ws = ld_dev(&C->ws);
    rs.we = ld_dev(&C->we);
    rs.active = ld_dev(&C->active);
    rs.ks = ld_dev(&C->keep_slab);
    rs.pend = 0;
    rs.ngap = 0;
    rs.pg_alloc = ld_dev(&C->pg_alloc);
    rs.occ = ld_dev(&C->cal_occ);
    rs.hold = ld_dev(&C->hold);
    rs.hold_need = ld_dev(&C->hold_need);
    rs.fpend = 0;
    rs.n_in = 0;
    rs.last = 0;
    rs.pend_ws = rs.ws;
    // (every spill-area entry so far may hold an import a gather must read: the re-layout at a
    // held edge empties the area)
    X.big->spill_imp = ld_dev(&C->spill_n);
  }
  const uint64_t rounds0 = ld_dev(&C->rounds);
  // the calendar horizon of a round starting at ws0 (OutboxHdr::hz)
  auto hz_of = [&](uint64_t ws0) { return SIM_START + (S.bw_div.div(ws0 - SIM_START) + S.NB) * S.BW; };
  // this workgroup's share of the senders' bin counters of round parity k (zeroed in the round
  // before their next use: no workgroup of this shard sends with them then)
  auto bin_counters_reset = [&](uint32_t k) {
    if (!S.xin_bins) return;
    const uint32_t nb = R * S.xgx;
    for (uint32_t i = w * 64 + threadIdx.x; i < nb; i += P * 64) st_dev(&S.xbin_n[(size_t)k * nb + i], 0u);
  };
  // The runs other shards sent this shard (inbox slot parity fbuf, rs.nin per sender) into the
  // calendar with the bucket -> slab table as it is now; their bucket minima except for the
  // buckets of the window [nws, nwe) they will be gathered in (its first bucket's minimum is not
  // read while it is the window's, and its last bucket's later runs join the kept minimum).
  // own: this workgroup's groups only (every workgroup scans every run: no barrier needed
  // before its own gathers); else a share of all of them (then a barrier).
  auto file_in = [&](uint32_t fbuf, uint64_t fhz, uint64_t nws, uint64_t nwe, bool own) {
    uint32_t ln = threadIdx.x;
    asm volatile("" : "+v"(ln));
    const uint32_t sb0 = bucket_of(S, nws), sbn = ((bucket_of(S, nwe - 1) - sb0) & (S.NB - 1)) + 1;
    const uint32_t n = rs.n_in;
    for (uint32_t i = (own ? 0u : w * 64) + ln; i < n; i += own ? 64u : P * 64) {
      uint32_t q = 0, off = i;
      while (off >= rs.nin[q]) off -= rs.nin[q++];
      SGN_GLB const EvRec* src = S.xin_runs + ((size_t)fbuf * R + q) * S.xislot + off;
      const EvRec ev = S.xsys ? ld_sys_rec(src) : ld_dev_rec(src);
      const uint32_t g = (ev.dst - S.lo) >> S.gsh;
      if (own && (g < gq0 || g >= gq1 || (g - gq0) % gqs != 0)) continue;
      if (ev.time >= fhz) {
        if ((atomicOr(&C->overflow, OVF_HORIZON) & OVF_HORIZON) == 0) C->overflow_info = ev.dst;
        continue;
      }
      const uint32_t b = bucket_of(S, ev.time);
      const size_t idx = (size_t)X.lbs[b] * S.G + g;
      const uint32_t pos = atomicAdd(&S.slab_n[idx], 1u);
      if (((b - sb0) & (S.NB - 1)) >= sbn) min_nr(&S.bucket_min[b], ev.time);
      if (pos < S.CAP)
        st_dev_rec(S.pool + idx * S.CAP + pos, ev);
      else  // the extension, or the spill area: the gathers read it there, and the spill flag
            // holds the round after on every shard for the re-layout
        place_overflow(S, nullptr, (uint32_t)idx, pos, ev);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  for (uint32_t i = threadIdx.x; i < S.NB; i += 64) X.lbs[i] = (uint16_t)ld_dev(&S.bucket_slab[i]);
  init_bmin<kApp>(S, X);
  __syncthreads();
  uint32_t r = 0;
  for (; r < max_rounds; r++) {
    if (!__builtin_amdgcn_readfirstlane((int)rs.active) || __builtin_amdgcn_readfirstlane((int)rs.hold)) break;
    const uint64_t ws = uni64(rs.ws), we = uni64(rs.we);
    const uint32_t ks = (uint32_t)__builtin_amdgcn_readfirstlane((int)rs.ks);
    const uint32_t p = r % 3;
    if (w == wbk) {
      if (rs.pend) rb_bookkeep(S, rs.pend_ws, rs.pend_we, rs.pend_nb1, rs.pend_new);
      // reset buffer (r + 1) % 3 for the next round: minima, counters, both barriers, exports
      const uint32_t q = (r + 1) % 3;
      for (uint32_t i = threadIdx.x; i < nch; i += 64) {
        st_dev(&S.rb_min[((size_t)q * RB_CH + i) * RbLayout<kApp>::MS], (uint64_t)INVALID);
        st_dev(&S.rb_min[((size_t)q * RB_CH + i) * RbLayout<kApp>::MS + 1], (uint64_t)INVALID);
        st_dev(&S.rb_occ[((size_t)q * RB_CH + i) * RbLayout<kApp>::OS], (uint64_t)0);
      }
      for (uint32_t i = threadIdx.x; i <= nch; i += 64) {
        const size_t o = (size_t)q * RbLayout<kApp>::CB + (i == nch ? RB_CH : i) * RbLayout<kApp>::CS;
        st_dev(&S.rb_cnt[o], 0u);
        st_dev(&S.rb2_cnt[o], 0u);
      }
      for (uint32_t i = threadIdx.x; i < R; i += 64) {
        st_dev(&S.xout_n[q * R + i], 0u);
        st_dev(&S.xout_n[(3 + q) * R + i], 0u);
      }
      if (threadIdx.x == 0) {
        st_dev(&S.rb_keep[q], (uint64_t)INVALID);
        st_dev(&S.rb_free[q], (uint64_t)0);
        st_dev(&S.rb_occ[3 * RB_CH * RB_OS_MAX + q], (uint64_t)0);
        st_dev(&S.rb_occ[3 * RB_CH * RB_OS_MAX + 3 + q], (uint64_t)0);
      }
    }
    // (the bins this round's gathers read were filled with parity (rounds0 + r) & 1 last round;
    // the next round sends with it again)
    bin_counters_reset((uint32_t)((rounds0 + r) & 1));
    if (threadIdx.x == 0) {
      X.ob->keepmin = &S.rb_keep[p];
      X.ob->bbase = ws;
      X.ob->pg_avail = rs.pg_avail;
      X.ob->pg_freed = &S.rb_free[p];
      X.ob->pg_allocd = &S.rb_occ[3 * RB_CH * RB_OS_MAX + p];
      X.ob->spilled = &S.rb_occ[3 * RB_CH * RB_OS_MAX + 3 + p];
      X.ob->xn = S.xout_n + (size_t)p * R;
      X.ob->xc = S.xin_bins ? rs.nin : nullptr;
      X.ob->xbuf = (uint32_t)((rounds0 + r + 1) & 1);
    }
    // diagnostics (SGN_STAMPS=2): per round of this launch, on the 100 MHz clock: {earliest start,
    // latest local arrival, local barrier seen (last workgroup), its messages sent, latest "all
    // messages seen", latest imports filed, latest second barrier seen}
    // (SGN_STAMPS=3: every workgroup's own stamps, plain stores: [128 rounds][2048][8])
    SGN_GLB uint64_t* rd = S.rdbg ? S.rdbg + (S.rdbg_wg ? ((size_t)(r & 127) * 2048 + w) * 8 : 8 * (size_t)(r & 127)) : nullptr;
    auto stamp = [&](uint32_t i, bool mx) {
      if (rd && threadIdx.x == 0) {
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        if (S.rdbg_wg)
          rd[i] = t;
        else if (mx)
          __hip_atomic_fetch_max(rd + i, (unsigned long long)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
          __hip_atomic_fetch_min(rd + i, (unsigned long long)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    };
    stamp(0, false);
    // the previous round's imports for this workgroup's groups (few of them: every workgroup
    // scans them all instead of a second barrier), before its gathers read the slabs
    if (uni32(rs.fpend)) {
      file_in(rs.fbuf, hz_of(rs.pend_ws), ws, we, true);
      __syncthreads();
      if (threadIdx.x == 0) {
        X.big->spill_imp = ld_dev(&C->spill_n);
        rs.fpend = 0;
      }
      __syncthreads();
    }
    if (threadIdx.x < XR_MAX) rs.nin[threadIdx.x] = 0;  // (now the per-peer send counts: xc)
    // ---- 1. execute this workgroup's groups, then arrive (the last arrival learns it is) ----
    uint64_t kall = INVALID, mall = INVALID, oall = 0;
    bool arrived = false;
    for (uint32_t g = gq0; g < gq1; g += gqs) {
      uint64_t kmin, m;
      const bool lastg = g + gqs >= gq1;
      exec_group<false, kApp, kKxBig, true>(S, g, ws, we, ks, X, &kmin, &m, [&](uint64_t k, uint64_t n, uint64_t od) {
        kall = k < kall ? k : kall;
        mall = n < mall ? n : mall;
        oall += od;
        if (lastg) {
          flush_bmin<kApp>(S, X);
          stamp(1, true);
          rb_arrive_x<kApp>(S, p, w, P, kall, mall, oall, &rs.last, X.ob->xc);
          arrived = true;
        }
      });
      __syncthreads();
    }
    if (!arrived) rb_arrive_x<kApp>(S, p, w, P, INVALID, INVALID, 0, &rs.last, nullptr);
    __syncthreads();
    const uint64_t tag = rounds0 + r + 1;  // the global round number + 1 (the same on every shard)
    const uint32_t buf = (uint32_t)(tag & 1);
    // (the lane index laundered every round: the compiler would otherwise hoist this section's
    // lane-dependent values out of the round loop and keep them in registers through the
    // execute phase, where the round kernels have none to spare)
    uint32_t lane = threadIdx.x;
    asm volatile("" : "+v"(lane));
    // ---- 2. the shard's last arrival: its round edge, and its message to every shard ----
    if (uni32(rs.last)) {
      stamp(2, true);
      // the message's own inputs beside the round edge's loads (no dependent round trips)
      SGN_GLB uint64_t* hm = nullptr;
      uint64_t cnt = 0, tot = 0;  // runs to the peer: in its slot; in all (bins and slot)
      if (lane < R) hm = S.xp[lane].hdr[buf];
      if (lane < R && lane != me) {
        cnt = ld_dev(&S.xout_n[(size_t)p * R + lane]);
        tot = S.xin_bins ? (uint64_t)ld_dev(&S.xout_n[(size_t)(3 + p) * R + lane]) : cnt;
      }
      const uint64_t spilled = ld_dev(&C->spill_n);
      const uint64_t mu = ld_dev(&C->min_used);
      const RbEdge e = rb_edge<kApp>(S, p, nch, ws, we);  // (its window: this shard's view only)
      uint64_t xmax = cnt, xsum = tot;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = shfl_xor64(xmax, off);
        xmax = o > xmax ? o : xmax;
        xsum += shfl_xor64(xsum, off);
      }
      if (kXFenceRel && S.xsys) {
        // System-scope release before the message (the peers are other GPUs): every run this
        // shard stored into a peer's bins or slot was a write-through sc0 sc1 store whose wave
        // waited for it (s_waitcnt vmcnt(0)) before arriving, and the arrivals completed before
        // this workgroup learned it is last; the fence writes back anything else of this XCD's
        // L2 and orders it all before the message words. (The wait after it is explicit: the
        // compiler may drop its own, MI355X_MICROARCH.md "compiler hazard".)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (lane < R) {
        const uint64_t v[XH_N] = {cnt, e.min_next, mu, xmax, spilled ? 1ull : 0ull,
                                  pages_free(rs.pg_avail + e.nfree, rs.pg_alloc + e.nalloc),
                                  rs.occ + e.occd, xsum, (uint64_t)S.G * S.CAP + S.ext_total, S.nH,
                                  e.nb1, e.occd, e.nalloc, e.nfree, tot};
        // every 8-byte word tagged (xh_lo / xh_hi): across GPUs each is its own 8-byte atomic
        // store, so no receiver relies on a 16-byte store arriving untorn over xGMI
        if (S.xsys) {
#pragma unroll
          for (uint32_t k = 0; k < XH_N; k++) {
            st_sys(hm + 2 * k, xh_lo(v[k], tag));
            st_sys(hm + 2 * k + 1, xh_hi(v[k], tag));
          }
        } else {
#pragma unroll
          for (uint32_t k = 0; k < XH_N; k++) st_wt16(hm + 2 * k, xh_lo(v[k], tag), xh_hi(v[k], tag));
        }
      }
      stamp(3, true);
    }
    // ---- 3. every shard's message (granule q + 8 j: words 2 j, 2 j + 1 of sender q) ----
    uint64_t ga = 0, gb = 0;
    {
      const uint32_t q = lane & 7, jj = lane >> 3;
      const bool mine = q < R && 2 * jj < XH_N;
      SGN_GLB const uint64_t* h = S.xin_hdr + ((size_t)buf * R + q) * XH_WORDS + 4 * jj;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      bool ok = true;
      // every workgroup of every shard waits here: only the first granule of each message is
      // polled (R lanes; a poll of every granule by every workgroup swamped the L2 channel that
      // holds them), then every granule is read once and its tag checked (re-read if late)
      while (true) {
        bool good = true;
        if (lane < R) {
          const u64x2 x = ld_gran16(S.xin_hdr + ((size_t)buf * R + lane) * XH_WORDS, S.xsys != 0);
          good = xh_ok(x.x, x.y, tag);
        }
        if (__ballot(!good) == 0) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kXWaitTicks) {
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(kApp == SGN_TRAFFIC_TGEN ? 8 : 4);
      }
      while (ok) {
        bool good = true;
        if (mine) {
          const u64x2 x = ld_gran16(h, S.xsys != 0), y = ld_gran16(h + 2, S.xsys != 0);
          ga = xh_val(x.x, x.y);
          gb = xh_val(y.x, y.y);
          good = xh_ok(x.x, x.y, tag) && (2 * jj + 1 >= XH_N || xh_ok(y.x, y.y, tag));
        }
        if (__ballot(!good) == 0) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kXWaitTicks) ok = false;
      }
      if (!ok) {
        if (lane == 0) atomicOr((unsigned int*)&C->overflow, OVF_TIMEOUT);
        return;
      }
      // (a system-scope acquire here: not built by default, see kXFenceAcq)
      if (kXFenceAcq && S.xsys) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      stamp(4, true);
      // the words into LDS (the event list's space, free between rounds): word k of sender q
      // at [k][q], read below as broadcasts (a shuffle per word and sender serialised ~200
      // cross-lane reads on the round's critical path)
      uint64_t* mw = (uint64_t*)X.lev;
      if (mine) {
        mw[(2 * jj) * XR_MAX + q] = ga;
        if (2 * jj + 1 < XH_N) mw[(2 * jj + 1) * XR_MAX + q] = gb;
      }
      __syncthreads();
    }
    // word k of sender q
    auto xw = [&](uint32_t k, uint32_t q) { return ((const uint64_t*)X.lev)[k * XR_MAX + q]; };
    uint64_t gm = INVALID, gmu = INVALID, xs = 0, xmax = 0;
    uint32_t spill_any = 0, nin_l = 0;
    uint64_t bin_l = 0;  // (lane q: runs sender q put in this shard's bins)
    for (uint32_t q = 0; q < R; q++) {
      const uint64_t a0 = xw(XH_MIN, q), a1 = xw(XH_MU, q), a2 = xw(XH_XSUM, q), a3 = xw(XH_XMAX, q);
      const uint64_t a4 = xw(XH_SPILL, q), a5 = xw(XH_CNT, q), a6 = xw(XH_TOT, q);
      gm = a0 < gm ? a0 : gm;
      gmu = a1 < gmu ? a1 : gmu;
      xs += a2;
      xmax = a3 > xmax ? a3 : xmax;
      spill_any |= a4 ? 1u : 0u;
      if (lane == q && q != me) {
        nin_l = (uint32_t)min(a5, (uint64_t)S.xislot);
        bin_l = a6 - a5;
      }
    }
    // Runahead::get (runahead.rs:44-57) over the global min used latency; the controller
    // (controller.rs:88-112) over the global min next event
    const uint64_t min_next = gm;  // (each message's minimum is already unwrapped: EMU_MAX = none)
    uint64_t ra = (S.dynamic && gmu != INVALID) ? gmu : S.min_possible;
    ra = ra > S.runahead_cfg ? ra : S.runahead_cfg;
    uint64_t ne = min_next + ra;
    if (ne < min_next || ne > EMU_MAX) ne = EMU_MAX;
    ne = ne < S.end_time ? ne : S.end_time;
    const uint32_t active = min_next < ne ? 1u : 0u;
    // the next round's guards, evaluated for every shard from the messages alike (k_import's):
    // CoDel pages for the next window's due runs (occupancy plus everything exported this round,
    // a bound on what any shard receives), a re-layout after spills, the inbox slots
    uint32_t hflags = 0;
    uint64_t own_need = 0;
    if (active) {
      const uint32_t nbk = ((bucket_of(S, ne - 1) - bucket_of(S, min_next)) & (S.NB - 1)) + 1;
      for (uint32_t q = 0; q < R; q++) {
        const uint64_t occ = xw(XH_OCC, q) + xs, capb = (uint64_t)nbk * xw(XH_CAPB, q) + xs;
        const uint64_t need = codel_pages_bound(occ < capb ? occ : capb, xw(XH_NH, q));
        if (xw(XH_PFREE, q) < need) hflags |= HOLD_CODEL;
        if (q == me) own_need = need;
      }
      if (spill_any) hflags |= HOLD_SPILL;
      if (xmax > S.xislot) hflags |= HOLD_XSLOT;
      else if (2 * xmax > S.xislot) hflags |= HOLD_XGROW;
    }
    // this shard's own round edge, from its message to itself
    const uint64_t e_nb1 = xw(XH_NB1, me), e_occd = xw(XH_OCCD, me), e_nalloc = xw(XH_NALLOC, me),
                   e_nfree = xw(XH_NFREE, me);
    uint32_t n_in = nin_l;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      n_in += __shfl_xor(n_in, off, 64);
      bin_l += shfl_xor64(bin_l, off);
    }
    // the idle-gap case of k_rounds: the bookkeeping now, and a local barrier before any send of
    // the next round can reach this round's bucket indices again
    const uint64_t span = (uint64_t)S.NB * S.BW;
    const uint64_t bstart = SIM_START + S.bw_div.div(ws - SIM_START) * S.BW;
    const bool gap = active && (ne + S.max_lat >= bstart + span || ne + S.max_lat < ne);
    if (gap) {
      if (w == wbk) rb_bookkeep(S, ws, we, e_nb1, ks);
      if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        SGN_GLB uint32_t* gc = S.rb_cnt + 3 * RB_CB_MAX;
        const uint32_t target = (rs.ngap + 1) * P;
        __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t sp = 0;
        while (ld_dev(gc) < target && ++sp < (1u << 24)) __builtin_amdgcn_s_sleep(2);
        if (sp >= (1u << 24)) atomicOr((unsigned int*)&C->overflow, OVF_TIMEOUT);
        rs.ngap++;
      }
    }
    if (lane < XR_MAX) rs.nin[lane] = nin_l;  // (lanes >= R hold 0)
    __syncthreads();
    const uint32_t b1 = bucket_of(S, we - 1);
    if (threadIdx.x == 0) {
      // the spare slab set (survivors + this round's new runs for b1) becomes bucket b1
      const uint32_t slab_b1 = X.lbs[b1];
      X.lbs[b1] = (uint16_t)ks;
      rs.pend = gap ? 0u : 1u;
      rs.pend_ws = ws;
      rs.pend_we = we;
      rs.pend_nb1 = e_nb1;
      rs.pend_new = ks;
      rs.ks = slab_b1;
      rs.ws = min_next;
      rs.we = ne;
      rs.active = active;
      rs.pg_avail += e_nfree;
      rs.pg_alloc += e_nalloc;
      rs.occ += e_occd + n_in + bin_l;  // (every import counts from here: slots and bins)
      rs.n_in = n_in;
      rs.hold = hflags;
      rs.hold_need = own_need;
      rs.last = 0;
      if (w == wbk) {
        st_dev(&C->last_min_next, min_next);
        st_dev(&C->prev_we, we);
        if (gmu != INVALID) min_nr(&C->min_used, gmu);  // (the next rounds' messages carry it)
        // the largest per-peer count any shard produced (the host sizes the inbox slots by it)
        (void)__hip_atomic_fetch_max(&C->xhwm, xmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
    // ---- 5. the runs other shards sent this shard: a few are filed by their own workgroups at
    // the next round's start; many are shared out now and a second local barrier follows ----
    if (uni32(rs.n_in)) {
      if (uni32(rs.n_in) <= S.xown) {
        if (threadIdx.x == 0) {
          rs.fpend = 1;
          rs.fbuf = buf;
        }
        __syncthreads();
      } else {
        file_in(buf, hz_of(ws), uni64(rs.ws), uni64(rs.we), false);
        stamp(5, true);
        rb2_arrive<kApp>(S, p, w, P);
        if (!rb_wait<kApp>(&S.rb2_cnt[(size_t)p * RbLayout<kApp>::CB + RB_CH * RbLayout<kApp>::CS], nch)) {
          if (threadIdx.x == 0) atomicOr((unsigned int*)&C->overflow, OVF_TIMEOUT);
          return;
        }
        stamp(6, true);
        if (threadIdx.x == 0) X.big->spill_imp = ld_dev(&C->spill_n);  // (imports past their slab)
        __syncthreads();
      }
    }
    stamp(7, true);
  }
  // imports left for a next round this launch does not run: shared out now (the launch's end is
  // the barrier)
  if (uni32(rs.fpend)) file_in(rs.fbuf, hz_of(uni64(rs.pend_ws)), uni64(rs.ws), uni64(rs.we), false);
  // ... and the last round's bins of this workgroup's groups (file_in's rules: the launch's end
  // leaves every bin empty and every counter zero, whatever runs next)
  if (S.xin_bins) {
    const uint32_t ib = (uint32_t)((rounds0 + r) & 1);
    const uint64_t nws = uni64(rs.ws), nwe = uni64(rs.we), fhz = hz_of(uni64(rs.pend_ws));
    const uint32_t sb0 = bucket_of(S, nws), sbn = ((bucket_of(S, nwe - 1) - sb0) & (S.NB - 1)) + 1;
    uint32_t ln = threadIdx.x;
    asm volatile("" : "+v"(ln));
    const uint32_t bsh = R <= 2 ? 5u : R <= 4 ? 4u : 3u, E = 1u << bsh, q = ln >> bsh, e = ln & (E - 1);
    const bool on = q < R && q != me && e < S.xbk;
    bool spilled = false;
    for (uint32_t g = gq0; g < gq1; g += gqs) {
      SGN_GLB EvRec* bp = on ? S.xin_bins + (((size_t)ib * R + q) * S.G + g) * S.xbk + e : nullptr;
      bool more = on;
      for (uint32_t e0 = 0; e0 < S.xbk; e0 += E) {
        EvRec ev{};
        if (more) ev = S.xsys ? ld_sys_rec(bp + e0) : ld_dev_rec(bp + e0);
        const bool ok = more && ev.pc != 0;
        if (ok) {
          SGN_GLB uint64_t* pw = (SGN_GLB uint64_t*)(bp + e0) + 3;
          if (S.xsys) st_sys(pw, 0ull); else st_dev(pw, (uint64_t)0);
          if (ev.time >= fhz) {
            if ((atomicOr(&C->overflow, OVF_HORIZON) & OVF_HORIZON) == 0) C->overflow_info = ev.dst;
          } else {
            const uint32_t b = bucket_of(S, ev.time);
            const size_t idx = (size_t)X.lbs[b] * S.G + g;
            const uint32_t pos = atomicAdd(&S.slab_n[idx], 1u);
            if (((b - sb0) & (S.NB - 1)) >= sbn) min_nr(&S.bucket_min[b], ev.time);
            if (pos < S.CAP) {
              st_dev_rec(S.pool + idx * S.CAP + pos, ev);
            } else {
              place_overflow(S, nullptr, (uint32_t)idx, pos, ev);
              spilled = true;
            }
          }
        }
        const uint64_t m = __ballot(ok && e == E - 1);
        if (!m) break;
        more = on && ((m >> (q * E + E - 1)) & 1ull) && e0 + E + e < S.xbk;
      }
    }
    bin_counters_reset(ib);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // (runs past their slab: the next launch's gathers read the spill area up to here)
    if (__ballot(spilled) && threadIdx.x == 0)
      (void)__hip_atomic_fetch_max(&C->spill_imp, ld_dev(&C->spill_n), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the launch's per-wave statistics (k_rounds)
  __syncthreads();
  if (X.wacc && threadIdx.x < W_N && X.wacc[threadIdx.x] && gq0 < gq1) {
    const uint32_t k = threadIdx.x;
    if (k == W_MAXFILL)
      __hip_atomic_fetch_max(&S.w_cnt[k * S.G + gq0], X.wacc[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      cnt_add(&S.w_cnt[k * S.G + gq0], X.wacc[k]);
  }
  if (w == wbk) {
    if (rs.pend) rb_bookkeep(S, rs.pend_ws, rs.pend_we, rs.pend_nb1, rs.pend_new);
    if (threadIdx.x == 0) {
      st_dev(&C->keep_slab, rs.ks);
      st_dev(&C->ws, rs.ws);
      st_dev(&C->we, rs.we);
      st_dev(&C->active, rs.active);
      st_dev(&C->rounds, rounds0 + r);
      st_dev(&C->pg_avail, rs.pg_avail);
      st_dev(&C->cal_occ, rs.occ);
      (void)__hip_atomic_fetch_max(&C->spill_imp, X.big->spill_imp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (rs.hold) {
        st_dev(&C->hold, rs.hold);
        st_dev(&C->hold_need, rs.hold_need);
      }
    }
  }
}

// Multi-shard round edge, after the exchange: the runs other shards sent this round into the
// local calendar, then the window advance from every shard's message. k_execute's last wave
// already did the local bucket bookkeeping, so every run goes to its bucket's current slab
// set (runs for the window's last bucket into the spare slab, like local sends).
// The advance (Controller::manager_finished_current_round, controller.rs:88-112, over the
// global {min next event, min used latency}: each message's minimum counts every pending
// event of its shard, exported runs included, so the min over messages is what an all-reduce
// would give) is done by the LAST block to finish: every block has read the window that just
// ran before it counts itself in, so no block sees the new one. One kernel per round edge.
__device__ __forceinline__ void advance_window(const DevSim& S, Ctrl* C) {
  uint64_t m = INVALID, mu = INVALID;
  for (uint32_t p = 0; p < S.n_ranks; p++) {
    const uint64_t* msg = (const uint64_t*)(S.xin + (size_t)p * (S.xslot + XHDR));
    const uint64_t a = msg[1], b = msg[2];
    m = a < m ? a : m;
    mu = b < mu ? b : mu;
    S.xout_n[p] = 0;  // the next round's sends count from zero
  }
  if (S.dynamic && mu != INVALID && mu < C->min_used) C->min_used = mu;
  const uint64_t min_next = m == INVALID ? EMU_MAX : m;
  C->last_min_next = min_next;
  // Runahead::get (runahead.rs:44-57)
  uint64_t ra = (S.dynamic && C->min_used != INVALID) ? C->min_used : S.min_possible;
  ra = ra > S.runahead_cfg ? ra : S.runahead_cfg;
  uint64_t ne = min_next + ra;
  if (ne < min_next || ne > EMU_MAX) ne = EMU_MAX;
  ne = ne < S.end_time ? ne : S.end_time;
  C->active = min_next < ne ? 1u : 0u;
  C->prev_we = C->we;
  C->ws = min_next;
  C->we = ne;
  C->round_min = INVALID;
  C->rounds++;
}

// few blocks: the round's received runs are a few thousand, and every block counts itself in
// with a device atomic on one word
constexpr uint32_t kImportBlocks = 16;
__global__ __launch_bounds__(256) void k_import(DevSim S) {
  Ctrl* C = S.ctrl;
  // every block reads the same values: nothing changes them before all blocks count in
  if (!C->active || C->xspill || C->hold) return;
  // The send/recv moved the first C->xsz runs of each slot. If any shard had more for some
  // peer (the messages carry every shard's maximum), the round is held on every shard alike:
  // nothing is imported, the window stays, and the host completes the round with a
  // full-slot exchange and this kernel again (comm_complete_spill). Counts above the slot
  // itself are an overflow the sender already reported.
  uint64_t gm = 0;
  for (uint32_t r = 0; r < S.n_ranks; r++) {
    const uint64_t x = ((const uint64_t*)(S.xin + (size_t)r * (S.xslot + XHDR)))[3] & 0xFFFFFFFFull;
    gm = x > gm ? x : gm;
  }
  const uint32_t sz = C->xsz;
  // (gm > xslot: some shard spilled runs past a slot; the host grows the slots, then completes)
  const bool hold = gm > sz && (sz < S.xslot || gm > S.xslot);
  // the window that just ran (still C->ws): the same horizon as sends
  const uint64_t hz = SIM_START + (S.bw_div.div(C->ws - SIM_START) + S.NB) * S.BW;
  uint32_t filed = 0;
  for (uint32_t r = 0; r < S.n_ranks && !hold; r++) {
    if (r == S.rank) continue;
    const EvRec* blk = S.xin + (size_t)r * (S.xslot + XHDR);  // message, then the runs
    const uint32_t n = (uint32_t)min(((const uint64_t*)blk)[0], (uint64_t)S.xslot);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += gridDim.x * blockDim.x) {
      const EvRec e = blk[XHDR + i];
      if (e.time >= hz) {
        if ((atomicOr(&C->overflow, OVF_HORIZON) & OVF_HORIZON) == 0) C->overflow_info = e.dst;
        continue;
      }
      const uint32_t b = bucket_of(S, e.time);
      const size_t idx = (size_t)S.bucket_slab[b] * S.G + ((e.dst - S.lo) >> S.gsh);
      const uint32_t pos = atomicAdd(&S.slab_n[idx], 1u);
      atomicMin((unsigned long long*)&S.bucket_min[b], (unsigned long long)e.time);
      if (pos < S.CAP)
        S.pool[idx * S.CAP + pos] = e;
      else  // the extension, or the spill area: the next round's gather reads it (lossless), and
            // the spill flag holds the round after that on every shard for the re-layout
        place_overflow(S, nullptr, (uint32_t)idx, pos, e);
      filed++;
    }
  }
  __shared__ uint32_t last, bfiled;
  if (threadIdx.x == 0) bfiled = 0;
  __syncthreads();
  if (filed) atomicAdd(&bfiled, filed);
  __syncthreads();  // this block's reads of C->ws are done
  if (threadIdx.x == 0) {
    if (bfiled) (void)atomicAdd((unsigned long long*)&C->cal_occ, (unsigned long long)bfiled);  // (completes first)
    last = atomicAdd(&C->imp_done, 1u) == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  C->imp_done = 0;
  // the spill-area entries the next round's gathers scan for runs imported past their slab
  C->spill_imp = ld_dev(&S.ctrl->spill_n);
  if (gm > C->xhwm) C->xhwm = gm;
  if (hold) {
    C->xspill = 1;
    return;
  }
  advance_window(S, C);
  if (!C->active) return;
  // the next round's guards, evaluated for EVERY shard from the messages alike (so all shards
  // hold the same round, or none): a shard's CoDel pages may not cover the next window's due
  // runs — its occupancy plus everything exported this round (a bound on what it received)
  // and at most its slabs of the window's buckets — or some shard spilled runs
  uint64_t xs = 0;
  for (uint32_t q = 0; q < S.n_ranks; q++) xs += ((const uint64_t*)(S.xin + (size_t)q * (S.xslot + XHDR)))[6];
  const uint32_t nbk = ((bucket_of(S, C->we - 1) - bucket_of(S, C->ws)) & (S.NB - 1)) + 1;
  uint32_t hflags = 0;
  uint64_t own = 0;
  for (uint32_t q = 0; q < S.n_ranks; q++) {
    const uint64_t* msg = (const uint64_t*)(S.xin + (size_t)q * (S.xslot + XHDR));
    // (msg[7]: the shard's runs per bucket, extensions included; imported runs may go past it)
    const uint64_t occ = msg[5] + xs, capb = (uint64_t)nbk * msg[7] + xs;
    const uint64_t need = codel_pages_bound(occ < capb ? occ : capb, S.rank_lo[q + 1] - S.rank_lo[q]);
    if (msg[4] < need) hflags |= HOLD_CODEL;
    if ((msg[3] >> 32) & 1) hflags |= HOLD_SPILL;
    if (q == S.rank) own = need;
  }
  if (hflags) {
    C->hold = hflags;
    C->hold_need = own;
  }
}

// CoDel control-law self test (f64 sqrt/div/round on the device vs the host).
__global__ void k_codel_law_test(uint64_t n, uint64_t* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = codel_law(SIM_START, i) - SIM_START;
}

// sgn_submit: each datagram becomes an event record of its source host in the calendar
// bucket of its send time (validated on the host: owned source, time within the horizon).
__global__ void k_inject(const DevSim* Sp, const EvRec* recs, uint32_t n) {
  const DevSim& S = *Sp;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const EvRec r = recs[i];
  const uint32_t g = (r.dst - S.lo) >> S.gsh;
  const uint32_t b = bucket_of(S, r.time);
  const size_t idx = (size_t)S.bucket_slab[b] * S.G + g;
  const uint32_t pos = atomicAdd(&S.slab_n[idx], 1u);
  atomicMin((unsigned long long*)&S.bucket_min[b], (unsigned long long)r.time);
  (void)atomicAdd((unsigned long long*)&S.ctrl->cal_occ, 1ULL);
  if (pos < S.CAP)
    S.pool[idx * S.CAP + pos] = r;
  else
    place_overflow(S, nullptr, (uint32_t)idx, pos, r);  // (a spill: sgn_submit re-lays out right after)
}

// Calendar re-layout (a held round edge after a spill, or sgn_submit): every slab's runs into
// the new layout — slabs of cap runs, and extensions (ext: offset | capacity << 40) for the hot
// ones — then the spilled runs after them. Order inside a slab is free (the gather sorts by
// Shadow's key); slab_n already counts every run of a slab, spilled ones included.
__device__ __forceinline__ EvRec* relayout_dst(EvRec* pool, uint32_t cap, const uint64_t* ext, EvRec* ext_pool,
                                               uint64_t idx, uint32_t j) {
  return j < cap ? pool + idx * cap + j : ext_pool + (ext[idx] & EXT_OFF_MASK) + (j - cap);
}
// the pool part of every slab (thread = (slab, position)); sets each slab's respill cursor
__global__ void k_relayout(const EvRec* __restrict__ old_pool, uint32_t old_cap, const uint64_t* __restrict__ old_ext,
                           EvRec* pool, uint32_t cap, const uint64_t* __restrict__ ext, EvRec* ext_pool,
                           const uint32_t* __restrict__ slab_n, uint32_t* cursor, uint64_t n_slabs) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t idx = t / old_cap;
  const uint32_t j = (uint32_t)(t % old_cap);
  if (idx >= n_slabs) return;
  const uint32_t fill = slab_n[idx];
  if (j < min(fill, old_cap)) *relayout_dst(pool, cap, ext, ext_pool, idx, j) = old_pool[idx * old_cap + j];
  if (j == 0) cursor[idx] = min(fill, old_cap + (old_ext ? (uint32_t)(old_ext[idx] >> 40) : 0u));
}
// the old extensions' runs (thread = (hot slab k of the list, position))
__global__ void k_relayout_ext(const uint64_t* __restrict__ hot, uint64_t n_hot, uint32_t max_ecap,
                               const EvRec* __restrict__ old_ext_pool, const uint64_t* __restrict__ old_ext,
                               uint32_t old_cap, EvRec* pool, uint32_t cap, const uint64_t* __restrict__ ext,
                               EvRec* ext_pool, const uint32_t* __restrict__ slab_n) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t k = t / max_ecap;
  const uint32_t j = (uint32_t)(t % max_ecap);
  if (k >= n_hot) return;
  const uint64_t idx = hot[k], x = old_ext[idx];
  const uint32_t fill = slab_n[idx];
  if (j < (uint32_t)(x >> 40) && old_cap + j < fill)
    *relayout_dst(pool, cap, ext, ext_pool, idx, old_cap + j) = old_ext_pool[(x & EXT_OFF_MASK) + j];
}
__global__ void k_respill(const EvRec* __restrict__ spill, const uint32_t* __restrict__ spill_idx, uint64_t n,
                          EvRec* pool, uint32_t cap, const uint64_t* __restrict__ ext, EvRec* ext_pool,
                          uint32_t* cursor, uint32_t* lost) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t idx = spill_idx[i];
  if (idx & SPILL_PEER) return;  // a run for another shard (grow_exchange_slot), or one a gather took
  const uint32_t pos = atomicAdd(&cursor[idx], 1u);
  const uint32_t room = cap + (ext ? (uint32_t)(ext[idx] >> 40) : 0u);
  if (pos < room)
    *relayout_dst(pool, cap, ext, ext_pool, idx, pos) = spill[i];
  else  // the host sized every slab for its fill (room >= fill): a violation is an error, never
        // a silent loss (relayout_calendar reads this count)
    atomicAdd(lost, 1u);
}

// sgn_rng_*: draws of host Xoshiro256++ streams (the state stays on the device). One thread
// per requested host (hosts distinct, checked on the host): its count[i] draws go to
// out[off[i] ..), in stream order.
__global__ void k_rng(const DevSim* Sp, const uint32_t* hosts, const uint32_t* count,
                      const uint64_t* off, uint32_t n, uint64_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  SGN_GLB HostRec* R = Sp->hrec + hosts[i];
  // (the state's two chunks: in the tiles, or in the record's hot line)
  SGN_GLB uint64_t* rg0 = Sp->htile ? Sp->htile + 2 * hot_idx(hosts[i], 0) : &R->rng[0];
  SGN_GLB uint64_t* rg1 = Sp->htile ? Sp->htile + 2 * hot_idx(hosts[i], 1) : &R->rng[2];
  uint64_t s0 = rg0[0], s1 = rg0[1], s2 = rg1[0], s3 = rg1[1];
  uint64_t* o = out + off[i];
  for (uint32_t k = 0; k < count[i]; k++) {
    o[k] = rotl64(s0 + s3, 23) + s0;
    const uint64_t t = s1 << 17;
    s2 ^= s0;
    s3 ^= s1;
    s1 ^= s2;
    s0 ^= s3;
    s2 ^= t;
    s3 = rotl64(s3, 45);
  }
  rg0[0] = s0;
  rg0[1] = s1;
  rg1[0] = s2;
  rg1[1] = s3;
  R->rng_pos += count[i];
}

// CPU-held host RNG states back into the records (sgn_rng_* single draws): per entry
// {slot, s0..s3, draws}; the stream position advances by the draws made on the CPU
__global__ void k_rng_set(const DevSim* Sp, const uint64_t* st, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t* e = st + 6 * (size_t)i;
  SGN_GLB HostRec* R = Sp->hrec + (uint32_t)e[0];
  SGN_GLB uint64_t* rg0 = Sp->htile ? Sp->htile + 2 * hot_idx((uint32_t)e[0], 0) : &R->rng[0];
  SGN_GLB uint64_t* rg1 = Sp->htile ? Sp->htile + 2 * hot_idx((uint32_t)e[0], 1) : &R->rng[2];
  rg0[0] = e[1];
  rg0[1] = e[2];
  rg1[0] = e[3];
  rg1[1] = e[4];
  R->rng_pos += e[5];
}

// Host::next_event_time (host.rs:832-834) for the owned HostIds [lo, lo + n), between rounds:
// the earliest local event (the host record's slots) ...
__global__ void k_next_local(const DevSim* Sp, uint32_t lo, uint32_t n, uint64_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t slot = Sp->sid_of[lo + i] - Sp->lo;
  const HostRec& r = Sp->hrec[slot];
  const uint64_t m0 = Sp->htile ? Sp->htile[2 * hot_idx(slot, 2) + 1] : r.st2;                   // st2
  const uint32_t flg = Sp->htile ? (uint32_t)Sp->htile[2 * hot_idx(slot, 7) + 1] : r.flags;     // flags
  uint64_t m = m0;
  if (Sp->tkind != SGN_TRAFFIC_PERIODIC || (flg & F_COLD)) {  // (else both relays idle)
    m = r.st0 < m ? r.st0 : m;
    m = r.st1 < m ? r.st1 : m;
  }
  out[i] = m;
}
// ... and the earliest pending packet event: one wave per (bucket, host group) slab,
// atomicMin into the destination's slot of out when it is in the range. Between rounds every
// pending event is in a bucket's slab (the spare slab set is empty).
__global__ void k_next_packet(const DevSim* Sp, uint32_t lo, uint32_t n, uint32_t g0, uint32_t ng,
                              uint64_t* out) {
  const DevSim& S = *Sp;
  const uint32_t w = blockIdx.x;  // (bucket, group) pair
  const uint32_t b = w / ng, g = g0 + w % ng;
  const size_t idx = (size_t)S.bucket_slab[b] * S.G + g;
  const uint32_t fill = S.slab_n[idx];
  const uint64_t x = S.ext && fill > S.CAP ? S.ext[idx] : 0ULL;
  const uint32_t np = min(fill, S.CAP), ne = min(fill - np, (uint32_t)(x >> 40));
  for (uint32_t j = threadIdx.x; j < np + ne; j += blockDim.x) {
    const EvRec& e = j < np ? S.pool[idx * S.CAP + j] : S.ext_pool[(x & EXT_OFF_MASK) + j - np];
    const uint32_t d = S.host_of[e.dst - S.lo];
    if (d >= lo && d < lo + n) atomicMin((unsigned long long*)&out[d - lo], (unsigned long long)e.time);
  }
}

}  // namespace sgn

// ====================================================================================
// Host side: sim init, round launch, readback
// ====================================================================================
using namespace sgn;

namespace {

inline uint64_t host_splitmix(uint64_t& s) {
  s += 0x9e3779b97f4a7c15ULL;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

template <typename T>
T* dalloc(sgn_ctx* ctx, size_t n) {
  return (T*)dev_alloc(ctx, n * sizeof(T));
}

enum { K_EXECUTE = 0, K_IMPORT, K_NUM };
const char* kKernelNames[K_NUM] = {"k_execute", "k_import"};

int launch_round(sgn_ctx* ctx);

// dynamic LDS of k_execute / k_rounds: CAP event runs + two u16 index arrays
// (the u16 index arrays are padded to 8 bytes so the optional bucket-minimum table that
// follows them is aligned)
inline size_t exec_lds_bytes(uint32_t cap, uint32_t agg_nb = 0) {
  return exec_lds_runs_bytes(cap) + (agg_nb ? (size_t)(agg_nb + 1) * 4 : 0);
}
constexpr uint32_t kPersistRounds = 128;  // rounds per persistent launch (then a host sync)
constexpr uint64_t kTimeEvery = 8;        // per-round launches: one timed in kTimeEvery

}  // namespace


namespace {

// the round kernels of the simulation's traffic kind (k_execute: traced or lean)
template <bool kTrace>
const void* execute_fn_t(uint32_t kind) {
  if (kind == SGN_TRAFFIC_TGEN) return (const void*)k_execute<kTrace, SGN_TRAFFIC_TGEN>;
  if (kind == SGN_TRAFFIC_EXTERNAL) return (const void*)k_execute<kTrace, SGN_TRAFFIC_EXTERNAL>;
  return (const void*)k_execute<kTrace, SGN_TRAFFIC_PERIODIC>;
}
const void* execute_fn(uint32_t kind, bool trace) {
  return trace ? execute_fn_t<true>(kind) : execute_fn_t<false>(kind);
}
template <bool kBig>
const void* rounds_fn_t(uint32_t kind) {
  if (kind == SGN_TRAFFIC_TGEN) return (const void*)k_rounds<SGN_TRAFFIC_TGEN, kBig>;
  if (kind == SGN_TRAFFIC_EXTERNAL) return (const void*)k_rounds<SGN_TRAFFIC_EXTERNAL, kBig>;
  return (const void*)k_rounds<SGN_TRAFFIC_PERIODIC, kBig>;
}
// the persistent kernel with the big-slab path only while a slab can hold more than CAP runs
bool rounds_big(const sgn_ctx* ctx) { return ctx->ext_slabs > 0; }
const void* rounds_fn(uint32_t kind, bool big) { return big ? rounds_fn_t<true>(kind) : rounds_fn_t<false>(kind); }
template <bool kTrace>
void launch_k_execute_t(sgn_ctx* ctx, hipStream_t st) {
  const uint32_t k = ctx->S.tkind;
  const dim3 grid(ctx->S.G), block(64);
  const size_t lds = exec_lds_bytes(ctx->S.CAP, ctx->S.agg_bmin ? ctx->S.NB : 0);
  const DevSim* d = (const DevSim*)ctx->d_S;
  if (k == SGN_TRAFFIC_TGEN)
    hipLaunchKernelGGL((k_execute<kTrace, SGN_TRAFFIC_TGEN>), grid, block, lds, st, d);
  else if (k == SGN_TRAFFIC_EXTERNAL)
    hipLaunchKernelGGL((k_execute<kTrace, SGN_TRAFFIC_EXTERNAL>), grid, block, lds, st, d);
  else
    hipLaunchKernelGGL((k_execute<kTrace, SGN_TRAFFIC_PERIODIC>), grid, block, lds, st, d);
}
void launch_k_execute(sgn_ctx* ctx, hipStream_t st) {
  if (ctx->S.trace_on)
    launch_k_execute_t<true>(ctx, st);
  else
    launch_k_execute_t<false>(ctx, st);
}
template <bool kBig>
void launch_k_rounds_t(sgn_ctx* ctx, uint32_t n) {
  const uint32_t k = ctx->S.tkind;
  const dim3 grid(ctx->persist_grid), block(64);
  const size_t lds = exec_lds_bytes(ctx->S.CAP, ctx->S.agg_bmin ? ctx->S.NB : 0);
  const DevSim* d = (const DevSim*)ctx->d_S;
  // (the census: this launch's epoch, and the arrivals of the launches before it)
  const uint32_t ep = ++ctx->res_epoch, base = ctx->res_base;
  ctx->res_base += ctx->persist_grid;
  if (k == SGN_TRAFFIC_TGEN)
    hipLaunchKernelGGL((k_rounds<SGN_TRAFFIC_TGEN, kBig>), grid, block, lds, ctx->stream, d, n, ep, base);
  else if (k == SGN_TRAFFIC_EXTERNAL)
    hipLaunchKernelGGL((k_rounds<SGN_TRAFFIC_EXTERNAL, kBig>), grid, block, lds, ctx->stream, d, n, ep, base);
  else
    hipLaunchKernelGGL((k_rounds<SGN_TRAFFIC_PERIODIC, kBig>), grid, block, lds, ctx->stream, d, n, ep, base);
}
// the census verdict of the last persistent launch: 1 resident, 2 not (0: none recorded)
uint32_t census_verdict(const sgn_ctx* ctx, uint32_t epoch) {
  const uint32_t v = ctx->h_ctrl->res_verdict;
  return (v >> 2) == (epoch & 0x3FFFFFFFu) ? (v & 3u) : 0u;
}
void launch_k_rounds(sgn_ctx* ctx, uint32_t n) {
  if (rounds_big(ctx))
    launch_k_rounds_t<true>(ctx, n);
  else
    launch_k_rounds_t<false>(ctx, n);
}

int launch_round(sgn_ctx* ctx) {
  // a multi-shard round needs its exchange transport before anything is launched
  if (ctx->nranks > 1 && !ctx->comm)
    return set_error(ctx, SGN_ESTATE, "multi-shard round without an RCCL communicator");
  hipStream_t st = ctx->stream;
  // per-round launches time one round in kTimeEvery: an event record is a barrier packet
  // with a cache write-back, and around every launch it cost 20 % of the rounds (eager) or
  // 45 % (graph batches) on config C; a sample gives the kernel's average duration
  const bool timed = ctx->capturing || (ctx->t_seq++ % kTimeEvery) == 0;
  if (timed) time_begin(ctx, K_EXECUTE);
  launch_k_execute(ctx, st);
  if (timed) time_end(ctx);
  if (!ctx->capturing) ctx->kt[K_EXECUTE].total++;
  if (ctx->nranks > 1) {
    // exchange + import + local finalize + all-reduce(min) + advance (comm.cpp)
    int rc = comm_round_exchange(ctx);
    if (rc) return rc;
  } else {
    // single shard: k_execute's last wave runs the round edge (finalize_fused)
  }
  SGN_HIP(ctx, hipGetLastError());
  ctx->rounds_enqueued++;
  return 0;
}

// Resident workgroups of a round kernel on this GPU (0: unknown): the occupancy query,
// capped by LDS per CU (the device attribute: 160 KiB on gfx950) — LDS is allocated per
// workgroup in 512-byte granules (a 23184-byte workgroup fits 6 per CU, not 7: a grid sized
// for 7 was not resident and its barrier timed out)
uint64_t resident_wg(sgn_ctx* ctx, const void* fn, size_t dyn) {
  int occ = 0, ncu = 0, lds_cu = 0;
  hipFuncAttributes fa{};
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 64, dyn) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess ||
      hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, ctx->device) != hipSuccess ||
      hipFuncGetAttributes(&fa, fn) != hipSuccess || occ <= 0 || ncu <= 0 || lds_cu <= 0)
    return 0;
  const size_t lds_wg = (fa.sharedSizeBytes + dyn + 511) / 512 * 512;
  ctx->lds_per_cu = (uint32_t)lds_cu;
  return (uint64_t)std::min<int>(occ, (int)((size_t)lds_cu / lds_wg)) * (uint64_t)ncu;
}

// The largest slab capacity whose round-kernel LDS fits one workgroup (calendar re-layout).
uint32_t max_slab_capacity(sgn_ctx* ctx, const DevSim& S) {
  int per_block = 0;
  if (hipDeviceGetAttribute(&per_block, hipDeviceAttributeMaxSharedMemoryPerBlock, ctx->device) != hipSuccess ||
      per_block <= 0)
    per_block = 64 * 1024;
  size_t st = 0;
  for (const void* fn : {rounds_fn(S.tkind, false), rounds_fn(S.tkind, true), execute_fn(S.tkind, S.trace_on)}) {
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, fn) == hipSuccess) st = std::max<size_t>(st, fa.sharedSizeBytes);
  }
  uint32_t cap = CAP_MIN;
  while (cap < (1u << 15) && st + exec_lds_bytes(cap * 2, S.NB) <= (size_t)per_block) cap *= 2;
  // test hook: a lower limit, so that hot slabs take extensions and the big-slab path at small sizes
  if (const char* e = getenv("SGN_SLAB_LIM")) cap = std::max<uint32_t>(16, std::min<uint32_t>(cap, (uint32_t)atoi(e)));
  return cap;
}

// The round kernels' shapes for the calendar as it is now (sim_init, and after a re-layout):
// the LDS table of bucket minima ((NB + 1) x 4 bytes per workgroup, flush_bmin) is used when
// it costs no resident workgroups where they count — the round kernels' grids stay as large
// (config C has no LDS to spare: its 1563 groups need 7 workgroups per CU), or the grid
// exceeds the chip either way (config D); SGN_AGG_BMIN=0/1 overrides — and the persistent
// grid (single shard): entirely resident, with workgroups looping over groups when G exceeds
// it. Persistent rounds keep the bucket -> slab table in LDS (each workgroup applies the
// round's swap itself), so they need NB <= LDS_BSLAB; longer calendars run one launch per
// round, and so does a traced run (k_rounds is built without the per-packet trace).
void size_round_kernels(sgn_ctx* ctx, DevSim& S) {
  const uint64_t G = S.G, NB = S.NB;
  bool agg = S.tkind == SGN_TRAFFIC_PERIODIC;  // the kernels fold in LDS for PERIODIC traffic (kAggBmin)
  for (const void* fn : {rounds_fn(S.tkind, false), rounds_fn(S.tkind, true), execute_fn(S.tkind, S.trace_on)}) {
    const uint64_t r0 = resident_wg(ctx, fn, exec_lds_bytes(S.CAP)), r1 = resident_wg(ctx, fn, exec_lds_bytes(S.CAP, S.NB));
    if (!r0 || std::min<uint64_t>(G, r1) < std::min<uint64_t>(G, r0)) agg = false;
  }
  if (const char* e = getenv("SGN_AGG_BMIN")) agg = atoi(e) != 0;
  if ((NB + 1) * S.BW >= (1ULL << 32)) agg = false;  // offsets from the window start must fit u32
  S.agg_bmin = agg ? 1u : 0u;
  ctx->persist_grid = 0;
  if (ctx->nranks == 1 && NB <= LDS_BSLAB && !S.trace_on && !ctx->persist_off &&
      !(getenv("SGN_PERSISTENT") && atoi(getenv("SGN_PERSISTENT")) == 0)) {
    // (resident for either variant: a re-layout that adds slab extensions switches to kBig)
    const size_t lds = exec_lds_bytes(S.CAP, S.agg_bmin ? S.NB : 0);
    const uint64_t res = std::min(resident_wg(ctx, rounds_fn(S.tkind, false), lds), resident_wg(ctx, rounds_fn(S.tkind, true), lds));
    if (res) {
      ctx->persist_grid = (uint32_t)std::min<uint64_t>(G, res);
      // test hook: a smaller grid makes every workgroup serve several groups per round
      if (const char* e = getenv("SGN_PERSIST_GRID"))
        ctx->persist_grid = std::max<uint32_t>(1, std::min<uint32_t>(ctx->persist_grid, (uint32_t)atoi(e)));
      // test hook: an oversized grid (not resident) exercises the residency census fallback
      if (const char* e = getenv("SGN_PERSIST_GRID_FORCE")) ctx->persist_grid = (uint32_t)atoi(e);
    }
  }
  if (ctx->persist_grid > 64 * RB_CH) ctx->persist_grid = 64 * RB_CH;
}

int check_overflow(sgn_ctx* ctx) {
  const Ctrl& c = *ctx->h_ctrl;
  if (c.overflow == 0) return 0;
  std::string what;
  if (c.overflow & OVF_BUCKET) what += " calendar bucket (raise sgn_sim_config.event_capacity)";
  if (c.overflow & OVF_CODEL) what += " CoDel page pool (raise sgn_sim_config.codel_cap)";
  if (c.overflow & OVF_SEG) what += " due-event segment buffer";
  if (c.overflow & OVF_EXCHANGE) what += " exchange slot (raise exchange_slot_events)";
  if (c.overflow & OVF_TRACE) what += " trace buffer";
  if (c.overflow & OVF_TIMEOUT) what += " persistent grid barrier timed out (grid not resident)";
  if (c.overflow & OVF_HORIZON) what += " event calendar horizon (a delivery beyond the calendar's buckets)";
  if (c.overflow & OVF_DRAIN) what += " drain buffer (raise sgn_drain_enable's capacity or drain more often)";
  return set_error(ctx, SGN_EOVERFLOW,
                   "device capacity exceeded:" + what + " (info " +
                       std::to_string(c.overflow_info) + "); results are invalid");
}

int sync_ctrl(sgn_ctx* ctx) {
  if (!ctx->failed.empty()) return set_error(ctx, SGN_ESTATE, "simulation unusable: " + ctx->failed);
  SGN_HIP(ctx, hipMemcpyAsync(ctx->h_ctrl, ctx->S.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost,
                              ctx->stream));
  SGN_HIP(ctx, hipStreamSynchronize(ctx->stream));
  time_collect(ctx);
  return check_overflow(ctx);
}
// After a persistent launch of census epoch ep: its own copy of the control block when it wrote
// one (no device-to-host copy on the launch edge), else sync_ctrl.
int sync_ctrl_persist(sgn_ctx* ctx, uint32_t ep) {
  if (!ctx->failed.empty()) return set_error(ctx, SGN_ESTATE, "simulation unusable: " + ctx->failed);
  if (!ctx->h_mirror) return sync_ctrl(ctx);
  SGN_HIP(ctx, hipStreamSynchronize(ctx->stream));
  constexpr size_t NW = sizeof(Ctrl) / 8;
  if (__atomic_load_n(&ctx->h_mirror[NW], __ATOMIC_ACQUIRE) != ep || ctx->h_mirror[kMirrorWords - 1])
    return sync_ctrl(ctx);
  std::memcpy(ctx->h_ctrl, ctx->h_mirror, sizeof(Ctrl));
  time_collect(ctx);
  return check_overflow(ctx);
}

// ---- pools that grow (the reference's queues are unbounded): run at a held round edge ----
int upload_sim(sgn_ctx* ctx) {
  SGN_HIP(ctx, hipMemcpy(ctx->d_S, &ctx->S, sizeof(DevSim), hipMemcpyHostToDevice));
  drop_graph(ctx);  // captured batches hold k_import's by-value DevSim
  return 0;
}

// The calendar re-laid out after runs went past their slabs (a held round edge, or sgn_submit).
// The slab capacity CAP doubles while more than 1/256 of the slabs (and more than 16) would
// still overflow, up to what one workgroup's LDS orders at once; the few hot slabs past it get
// extensions of 1.5x their fill (a slab keeps the capacity it had). Every run moves into the
// new layout, the spilled runs after them; the spill area empties, and grows when it was more
// than a quarter full. Device memory grows with the hot slabs only (sizing every
// slab for the fullest cost config D ~8 -> ~16 GB for one hot slab).
int relayout_calendar(sgn_ctx* ctx) {
  DevSim& S = ctx->S;
  Ctrl& c = *ctx->h_ctrl;
  const uint64_t n_slabs = (uint64_t)(S.NB + 1) * S.G;
  if (c.spill_n > S.spill_cap)
    return set_error(ctx, SGN_EOVERFLOW, "calendar spill area exhausted within one round (" +
                                             std::to_string(c.spill_n) + " runs, capacity " +
                                             std::to_string(S.spill_cap) + ")");
  const uint64_t nsp = c.spill_n;
  std::vector<uint32_t> fill(n_slabs);
  SGN_HIP(ctx, hipMemcpy(fill.data(), (const void*)S.slab_n, n_slabs * 4, hipMemcpyDeviceToHost));
  const std::vector<uint64_t>& oext = ctx->h_ext;  // (empty: no extensions yet)
  auto oecap = [&](uint64_t i) -> uint64_t { return oext.empty() ? 0 : oext[i] >> 40; };
  // the new slab capacity
  const uint32_t lim = std::max(S.CAP, max_slab_capacity(ctx, S));
  const uint64_t few = std::max<uint64_t>(16, n_slabs / 256);
  uint32_t cap = S.CAP;
  size_t mfree = 0, mtot = 0;
  if (hipMemGetInfo(&mfree, &mtot) != hipSuccess) mfree = 0;
  while (cap * 2 <= lim && n_slabs * cap * 2 * sizeof(EvRec) < mfree / 2) {
    uint64_t over = 0;
    for (uint64_t i = 0; i < n_slabs; i++) over += fill[i] > cap;
    if (over <= few) break;
    cap *= 2;
  }
  // extensions: hot slabs keep room for 1.5x their fill, and never less than they had
  std::vector<uint64_t> next(n_slabs, 0), hot_old;
  uint64_t etot = 0, nhot = 0, max_oecap = 0;
  for (uint64_t i = 0; i < n_slabs; i++) {
    const uint64_t had = oecap(i) ? S.CAP + oecap(i) : 0;
    if (oecap(i)) {
      hot_old.push_back(i);
      max_oecap = std::max(max_oecap, oecap(i));
    }
    // (a slab that fits the slab capacity or what it had keeps that; one that outgrew both gets
    // 1.5x its fill — growth follows the fill, not the number of re-layouts)
    const uint64_t need = fill[i] <= std::max<uint64_t>(had, cap) ? had : fill[i] + fill[i] / 2;
    if (need <= cap) continue;
    const uint64_t e = ((need - cap) + 63) / 64 * 64;
    if (e >= (1ULL << 24))
      return set_error(ctx, SGN_EOVERFLOW, "a calendar slab above 2^24 runs (slab " + std::to_string(i) + ", fill " +
                                               std::to_string(fill[i]) + ", had " + std::to_string(had) + ", cap " +
                                               std::to_string(S.CAP) + " -> " + std::to_string(cap) + ")");
    next[i] = etot | (e << 40);
    etot += e;
    nhot++;
  }
  if (etot >= (1ULL << 40)) return set_error(ctx, SGN_EOVERFLOW, "calendar extensions above 2^40 runs");
  const bool changed = cap != S.CAP || next != (oext.empty() ? std::vector<uint64_t>(n_slabs, 0) : oext);
  if (changed) {
    EvRec* np = cap != S.CAP ? (EvRec*)dev_alloc(ctx, n_slabs * cap * sizeof(EvRec), false) : (EvRec*)S.pool;
    EvRec* nep = etot ? (EvRec*)dev_alloc(ctx, etot * sizeof(EvRec), false) : nullptr;
    uint64_t* nxt = etot ? (uint64_t*)dev_alloc(ctx, n_slabs * 8, false) : nullptr;
    uint32_t* cur = (uint32_t*)dev_alloc(ctx, (n_slabs + 1) * 4, false);  // + k_respill's lost-run count
    uint64_t* dhot = hot_old.empty() ? nullptr : (uint64_t*)dev_alloc(ctx, hot_old.size() * 8, false);
    auto undo = [&]() {
      if (np && np != (EvRec*)S.pool) dev_free(ctx, np, n_slabs * cap * sizeof(EvRec));
      if (nep) dev_free(ctx, nep, etot * sizeof(EvRec));
      if (nxt) dev_free(ctx, nxt, n_slabs * 8);
      if (cur) dev_free(ctx, cur, (n_slabs + 1) * 4);
      if (dhot) dev_free(ctx, dhot, hot_old.size() * 8);
    };
    if (!np || (etot && (!nep || !nxt)) || !cur || (!hot_old.empty() && !dhot)) {
      undo();
      return set_error(ctx, SGN_ENOMEM, "device allocation failed (calendar re-layout)");
    }
    if (nxt) SGN_HIP(ctx, hipMemcpy(nxt, next.data(), n_slabs * 8, hipMemcpyHostToDevice));
    if (dhot) SGN_HIP(ctx, hipMemcpy(dhot, hot_old.data(), hot_old.size() * 8, hipMemcpyHostToDevice));
    SGN_HIP(ctx, hipMemsetAsync(cur + n_slabs, 0, 4, ctx->stream));
    // the pool part moves only when the slabs grow (in place it stays where it is)
    const uint64_t nt = n_slabs * S.CAP;
    if (np != (EvRec*)S.pool) {
      hipLaunchKernelGGL(k_relayout, dim3((uint32_t)((nt + 255) / 256)), dim3(256), 0, ctx->stream,
                         (const EvRec*)S.pool, S.CAP, (const uint64_t*)S.ext, np, cap, (const uint64_t*)nxt, nep,
                         (const uint32_t*)S.slab_n, cur, n_slabs);
    } else {
      std::vector<uint32_t> hc(n_slabs);
      for (uint64_t i = 0; i < n_slabs; i++) hc[i] = (uint32_t)std::min<uint64_t>(fill[i], S.CAP + oecap(i));
      SGN_HIP(ctx, hipMemcpy(cur, hc.data(), n_slabs * 4, hipMemcpyHostToDevice));
    }
    if (!hot_old.empty()) {
      const uint64_t ne = hot_old.size() * max_oecap;
      hipLaunchKernelGGL(k_relayout_ext, dim3((uint32_t)((ne + 255) / 256)), dim3(256), 0, ctx->stream,
                         (const uint64_t*)dhot, (uint64_t)hot_old.size(), (uint32_t)max_oecap,
                         (const EvRec*)S.ext_pool, (const uint64_t*)S.ext, S.CAP, np, cap, (const uint64_t*)nxt, nep,
                         (const uint32_t*)S.slab_n);
    }
    if (nsp)
      hipLaunchKernelGGL(k_respill, dim3((uint32_t)((nsp + 255) / 256)), dim3(256), 0, ctx->stream,
                         (const EvRec*)S.spill, (const uint32_t*)S.spill_idx, nsp, np, cap, (const uint64_t*)nxt,
                         nep, cur, cur + n_slabs);
    SGN_HIP(ctx, hipGetLastError());
    SGN_HIP(ctx, hipStreamSynchronize(ctx->stream));
    uint32_t lost = 0;
    SGN_HIP(ctx, hipMemcpy(&lost, cur + n_slabs, 4, hipMemcpyDeviceToHost));
    if (lost) {
      ctx->failed = "calendar re-layout lost " + std::to_string(lost) + " spilled runs (slab sizing)";
      return set_error(ctx, SGN_EOVERFLOW, ctx->failed);
    }
    if (np != (EvRec*)S.pool) dev_free(ctx, (void*)S.pool, n_slabs * S.CAP * sizeof(EvRec));
    if (S.ext_pool) dev_free(ctx, (void*)S.ext_pool, S.ext_total * sizeof(EvRec));
    if (S.ext) dev_free(ctx, (void*)S.ext, n_slabs * 8);
    dev_free(ctx, cur, (n_slabs + 1) * 4);
    if (dhot) dev_free(ctx, dhot, hot_old.size() * 8);
    if (cap != S.CAP) ctx->cal_grows++;
    S.pool = (decltype(S.pool))np;
    S.CAP = cap;
    S.ext = (decltype(S.ext))nxt;
    S.ext_pool = (decltype(S.ext_pool))nep;
    S.ext_total = etot;
    ctx->h_ext = etot ? next : std::vector<uint64_t>();
    ctx->ext_slabs = nhot;
    S.gspec = std::min<uint32_t>(S.gspec, S.CAP);
    size_round_kernels(ctx, S);
  }
  ctx->cal_spill_runs += nsp;
  // the spill area: emptied; grown when this round used more than a quarter of it
  if (nsp > S.spill_cap / 4) {
    const uint64_t ncap = std::min<uint64_t>(1ULL << 30, std::max<uint64_t>(2 * S.spill_cap, 4 * nsp));
    EvRec* sp = (EvRec*)dev_alloc(ctx, ncap * sizeof(EvRec), false);
    uint32_t* si = (uint32_t*)dev_alloc(ctx, ncap * 4, false);
    if (sp && si) {
      dev_free(ctx, (void*)S.spill, S.spill_cap * sizeof(EvRec));
      dev_free(ctx, (void*)S.spill_idx, S.spill_cap * 4);
      S.spill = (decltype(S.spill))sp;
      S.spill_idx = (decltype(S.spill_idx))si;
      S.spill_cap = ncap;
      ctx->spill_grows++;
    } else {  // (the area as it was still works)
      if (sp) dev_free(ctx, sp, ncap * sizeof(EvRec));
      if (si) dev_free(ctx, si, ncap * 4);
    }
  }
  const uint64_t zero[2] = {0, 0};
  SGN_HIP(ctx, hipMemcpy((char*)S.ctrl + offsetof(Ctrl, spill_n), zero, 8, hipMemcpyHostToDevice));
  SGN_HIP(ctx, hipMemcpy((char*)S.ctrl + offsetof(Ctrl, spill_imp), zero, 8, hipMemcpyHostToDevice));
  c.spill_n = 0;
  c.spill_imp = 0;
  return upload_sim(ctx);
}

// the CoDel pages the round of the current window may take (codel_round_bound, host form)
uint64_t codel_need_host(const sgn_ctx* ctx) {
  const DevSim& S = ctx->S;
  const Ctrl& c = *ctx->h_ctrl;
  if (!c.active || c.we <= c.ws) return 0;
  auto bk = [&](uint64_t t) { return (uint32_t)((t - SIM_START) / S.BW) & (S.NB - 1); };
  const uint64_t nbk = ((bk(c.we - 1) - bk(c.ws)) & (S.NB - 1)) + 1;
  return codel_pages_bound(std::min<uint64_t>(c.cal_occ, nbk * S.G * S.CAP + S.ext_total), S.nH);
}

// A CoDel page pool with at least `extra` more free pages (and at least double the size): the
// pages keep their indices (host records and chains stay valid), the free ring is rebuilt as
// its current entries followed by the new pages.
int grow_codel(sgn_ctx* ctx, uint64_t extra) {
  DevSim& S = ctx->S;
  Ctrl& c = *ctx->h_ctrl;
  if (c.pg_avail != c.pg_tail)
    return set_error(ctx, SGN_ESTATE, "CoDel pool growth outside a round edge");
  const uint64_t P = S.cq_pages;
  const uint64_t P2 = std::max<uint64_t>(2 * P, P + extra + extra / 2 + 64);
  if (P2 >= (1ULL << 28)) return set_error(ctx, SGN_EOVERFLOW, "CoDel page pool above 2^28 pages");
  CodelEnt* ne = (CodelEnt*)dev_alloc(ctx, P2 * CQ_PAGE * sizeof(CodelEnt), false);
  uint32_t* nn = (uint32_t*)dev_alloc(ctx, P2 * 4, true);
  uint32_t* nf = (uint32_t*)dev_alloc(ctx, P2 * 4, false);
  if (!ne || !nn || !nf) return set_error(ctx, SGN_ENOMEM, "device allocation failed (CoDel pool growth)");
  SGN_HIP(ctx, hipMemcpy(ne, (const void*)S.codel, P * CQ_PAGE * sizeof(CodelEnt), hipMemcpyDeviceToDevice));
  SGN_HIP(ctx, hipMemcpy(nn, (const void*)S.cq_next, P * 4, hipMemcpyDeviceToDevice));
  std::vector<uint32_t> ring(P), fr;
  SGN_HIP(ctx, hipMemcpy(ring.data(), (const void*)S.cq_free, P * 4, hipMemcpyDeviceToHost));
  fr.reserve(P2);
  for (uint64_t i = c.pg_alloc; i < c.pg_tail; i++) fr.push_back(ring[i % P]);
  for (uint64_t pg = P; pg < P2; pg++) fr.push_back((uint32_t)pg);
  const uint64_t nfree = fr.size();
  fr.resize(P2, 0);
  SGN_HIP(ctx, hipMemcpy(nf, fr.data(), P2 * 4, hipMemcpyHostToDevice));
  dev_free(ctx, (void*)S.codel, P * CQ_PAGE * sizeof(CodelEnt));
  dev_free(ctx, (void*)S.cq_next, P * 4);
  dev_free(ctx, (void*)S.cq_free, P * 4);
  S.codel = (decltype(S.codel))ne;
  S.cq_next = (decltype(S.cq_next))nn;
  S.cq_free = (decltype(S.cq_free))nf;
  S.cq_pages = (uint32_t)P2;
  ctx->codel_allocs_before += c.pg_alloc;
  c.pg_alloc = 0;
  c.pg_tail = c.pg_avail = nfree;
  SGN_HIP(ctx, hipMemcpy((char*)S.ctrl + offsetof(Ctrl, pg_alloc), &c.pg_alloc, 3 * 8, hipMemcpyHostToDevice));
  ctx->codel_grows++;
  return upload_sim(ctx);
}

// Multi-shard: a round in which some shard had more runs for a peer than a slot holds (the
// messages carry every shard's largest count, so every shard grows alike to twice that):
// the slots grow, keeping each outgoing block's message and runs, and the runs that went to
// the spill area (tagged SPILL_PEER | peer) follow them; comm_complete_spill then moves the
// whole slots and completes the round.
int grow_exchange_slot_impl(sgn_ctx* ctx) {
  DevSim& S = ctx->S;
  const uint64_t hwm = ctx->h_ctrl->xhwm;
  uint64_t ns = S.xslot;
  while (ns < 2 * hwm) ns *= 2;
  if (ns > (1ULL << 26)) return set_error(ctx, SGN_EOVERFLOW, "exchange slot above 2^26 runs per peer");
  const size_t ob = XHDR + (size_t)S.xslot, nb = XHDR + (size_t)ns, R = S.n_ranks;
  EvRec* nxo = (EvRec*)dev_alloc(ctx, R * nb * sizeof(EvRec), true);
  EvRec* nxi = (EvRec*)dev_alloc(ctx, R * nb * sizeof(EvRec), true);
  if (!nxo || !nxi) return set_error(ctx, SGN_ENOMEM, "device allocation failed (exchange slot growth)");
  // (xin too: this shard's own message sits in its incoming block)
  for (size_t p = 0; p < R; p++) {
    SGN_HIP(ctx, hipMemcpy(nxo + p * nb, (const void*)(S.xout + p * ob), ob * sizeof(EvRec), hipMemcpyDeviceToDevice));
    SGN_HIP(ctx, hipMemcpy(nxi + p * nb, (const void*)(S.xin + p * ob), ob * sizeof(EvRec), hipMemcpyDeviceToDevice));
  }
  const uint64_t n = std::min<uint64_t>(ctx->h_ctrl->spill_n, S.spill_cap);
  if (n) {
    std::vector<uint32_t> idx(n);
    std::vector<EvRec> rec(n);
    SGN_HIP(ctx, hipMemcpy(idx.data(), (const void*)S.spill_idx, n * 4, hipMemcpyDeviceToHost));
    SGN_HIP(ctx, hipMemcpy(rec.data(), (const void*)S.spill, n * sizeof(EvRec), hipMemcpyDeviceToHost));
    std::vector<std::vector<EvRec>> per(R);
    for (uint64_t i = 0; i < n; i++)
      if ((idx[i] & SPILL_PEER) && idx[i] != SPILL_DEAD) per[idx[i] & ~SPILL_PEER].push_back(rec[i]);
    for (size_t p = 0; p < R; p++)
      if (!per[p].empty())
        SGN_HIP(ctx, hipMemcpy(nxo + p * nb + ob, per[p].data(), per[p].size() * sizeof(EvRec), hipMemcpyHostToDevice));
  }
  dev_free(ctx, (void*)S.xout, R * ob * sizeof(EvRec));
  dev_free(ctx, (void*)S.xin, R * ob * sizeof(EvRec));
  S.xout = (decltype(S.xout))nxo;
  S.xin = (decltype(S.xin))nxi;
  S.xslot = (uint32_t)ns;
  ctx->xslot = ns;
  ctx->xslot_grows++;
  if (int rc = xpeer_upload(ctx)) return rc;  // (the send blocks moved)
  return upload_sim(ctx);
}

// A round edge held the rounds (Ctrl::hold; nothing of the next round has run): the calendar
// is re-laid out after a spill, the CoDel pool grows until its free pages cover the next
// round's bound, and the rounds are released. (Multi-shard: every shard holds the same round;
// each grows what it needs.)
int resolve_hold(sgn_ctx* ctx) {
  Ctrl& c = *ctx->h_ctrl;
  if (!c.hold) {
    // (multi-shard: runs k_import spilled hold nothing; re-laid out at the batch's sync)
    return c.spill_n ? relayout_calendar(ctx) : 0;
  }
  int rc = 0;
  if (c.spill_n && (rc = relayout_calendar(ctx))) return rc;
  // (the bound again for the layout as it is now: spilled runs may be due in the held round)
  const uint64_t need = std::max(c.hold_need, codel_need_host(ctx));
  const uint64_t free = c.pg_avail > c.pg_alloc ? c.pg_avail - c.pg_alloc : 0;
  if (free < need && (rc = grow_codel(ctx, need - free))) return rc;
  ctx->rounds_held++;
  c.hold = 0;
  c.hold_need = 0;
  SGN_HIP(ctx, hipMemcpy((char*)ctx->S.ctrl + offsetof(Ctrl, hold), &c.hold, 4, hipMemcpyHostToDevice));
  return 0;
}

// Event-record nodes around the timed kernel nodes of a captured batch (a captured
// hipEventRecord yields no timing on ROCm 7.2; explicit record nodes do).
int add_timing_nodes(sgn_ctx* ctx, hipGraph_t g) {
  const bool all = ctx->flags & SGN_CREATE_TIME_KERNELS;
  const bool exec = ctx->flags & SGN_CREATE_TIME_EXECUTE;
  ctx->graph_timed.clear();
  if (!all && !exec) return 0;
  const void* fn[K_NUM] = {execute_fn(ctx->S.tkind, ctx->S.trace_on), (const void*)k_import};
  size_t n = 0;
  SGN_HIP(ctx, hipGraphGetNodes(g, nullptr, &n));
  std::vector<hipGraphNode_t> nodes(n);
  SGN_HIP(ctx, hipGraphGetNodes(g, nodes.data(), &n));
  size_t ev = 0;
  uint32_t tseen[K_NUM] = {};
  for (hipGraphNode_t node : nodes) {
    hipGraphNodeType t;
    SGN_HIP(ctx, hipGraphNodeGetType(node, &t));
    if (t != hipGraphNodeTypeKernel) continue;
    hipKernelNodeParams p;
    SGN_HIP(ctx, hipGraphKernelNodeGetParams(node, &p));
    int kid = -1;
    for (int k = 0; k < K_NUM; k++)
      if (p.func == fn[k]) kid = k;
    if (kid < 0 || (!all && kid != K_EXECUTE)) continue;
    if ((tseen[kid]++ % kTimeEvery) != 0) continue;  // a sample (launch_round's note)
    if (ev >= ctx->ev_pool.size()) {
      hipEvent_t a, b;
      SGN_HIP(ctx, hipEventCreate(&a));
      SGN_HIP(ctx, hipEventCreate(&b));
      ctx->ev_pool.push_back({a, b});
    }
    size_t nd = 0, nn = 0;
    SGN_HIP(ctx, hipGraphNodeGetDependencies(node, nullptr, &nd));
    std::vector<hipGraphNode_t> deps(nd);
    if (nd) SGN_HIP(ctx, hipGraphNodeGetDependencies(node, deps.data(), &nd));
    SGN_HIP(ctx, hipGraphNodeGetDependentNodes(node, nullptr, &nn));
    std::vector<hipGraphNode_t> outs(nn);
    if (nn) SGN_HIP(ctx, hipGraphNodeGetDependentNodes(node, outs.data(), &nn));
    hipGraphNode_t a, b;
    SGN_HIP(ctx, hipGraphAddEventRecordNode(&a, g, nd ? deps.data() : nullptr, nd, ctx->ev_pool[ev].first));
    SGN_HIP(ctx, hipGraphAddDependencies(g, &a, &node, 1));
    SGN_HIP(ctx, hipGraphAddEventRecordNode(&b, g, &node, 1, ctx->ev_pool[ev].second));
    for (hipGraphNode_t o : outs) SGN_HIP(ctx, hipGraphAddDependencies(g, &b, &o, 1));
    ctx->graph_timed.push_back({kid, ev});
    ev++;
  }
  return 0;
}

}  // namespace

namespace sgn {

void time_begin(sgn_ctx* ctx, int kernel) {
  if (ctx->capturing) return;  // graph mode: event-record nodes are added after capture
  const bool all = ctx->flags & SGN_CREATE_TIME_KERNELS;
  const bool exec = (ctx->flags & SGN_CREATE_TIME_EXECUTE) && kernel == K_EXECUTE;
  if (!all && !exec) return;
  if (ctx->ev_next >= ctx->ev_pool.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
    ctx->ev_pool.push_back({a, b});
  }
  hipEventRecord(ctx->ev_pool[ctx->ev_next].first, ctx->stream);
  ctx->ev_pending.push_back({kernel, ctx->ev_next});
}

void time_end(sgn_ctx* ctx) {
  if (ctx->capturing) return;
  if (!(ctx->flags & (SGN_CREATE_TIME_KERNELS | SGN_CREATE_TIME_EXECUTE))) return;
  if (ctx->ev_pending.empty() || ctx->ev_pending.back().second != ctx->ev_next) return;
  hipEventRecord(ctx->ev_pool[ctx->ev_next].second, ctx->stream);
  ctx->ev_next++;
}

void time_collect(sgn_ctx* ctx) {
  if (!(ctx->flags & (SGN_CREATE_TIME_KERNELS | SGN_CREATE_TIME_EXECUTE))) return;
  if (ctx->graph_pending) {
    // events recorded by the replayed graph's event-record nodes
    for (auto& p : ctx->graph_timed) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, ctx->ev_pool[p.second].first,
                              ctx->ev_pool[p.second].second) == hipSuccess) {
        ctx->kt[p.first].ms += ms;
        ctx->kt[p.first].launches++;
      }
    }
    ctx->graph_pending = false;
  }
  for (auto& p : ctx->ev_pending) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, ctx->ev_pool[p.second].first, ctx->ev_pool[p.second].second) ==
        hipSuccess) {
      ctx->kt[p.first].ms += ms;
      ctx->kt[p.first].launches++;
    }
  }
  ctx->ev_pending.clear();
  ctx->ev_next = 0;
}

int ctrl_sync(sgn_ctx* ctx) { return sync_ctrl(ctx); }
int grow_exchange_slot(sgn_ctx* ctx) { return grow_exchange_slot_impl(ctx); }
int resolve_pools(sgn_ctx* ctx) { return resolve_hold(ctx); }

void drop_graph(sgn_ctx* ctx) {
  if (ctx->gexec) hipGraphExecDestroy(ctx->gexec);
  if (ctx->graph) hipGraphDestroy(ctx->graph);
  ctx->gexec = nullptr;
  ctx->graph = nullptr;
  ctx->gbatch = 0;
  ctx->gsz = 0;
  ctx->graph_timed.clear();
  ctx->graph_pending = false;
}

// ---- persistent multi-shard rounds (k_rounds_x): host side ----
// Inbox layout (one uncached allocation per shard): headers [2][R][XH_WORDS], census words [R]
// (padded to a line), runs [2][R][xislot].
// (then the bins: [2][R][G][xbk] runs, G = the receiving shard's host groups)
XLay xlay(uint32_t R, uint64_t xislot, uint32_t G, uint32_t xbk) {
  XLay l;
  l.hdr = 0;
  l.cen = (size_t)2 * R * XH_WORDS * 8;
  l.runs = l.cen + ((size_t)R * 8 + 127) / 128 * 128;
  l.bins = l.runs + (size_t)2 * R * xislot * sizeof(EvRec);
  l.bytes = l.bins + (size_t)2 * R * G * xbk * sizeof(EvRec);
  return l;
}

void xinbox_release(sgn_ctx* ctx) {
  for (void* p : ctx->x_opened)
    if (p) (void)hipIpcCloseMemHandle(p);
  ctx->x_opened.clear();
  if (ctx->xin_mem) {
    (void)hipFree(ctx->xin_mem);
    ctx->sim_bytes -= std::min<uint64_t>(ctx->sim_bytes, ctx->xin_bytes);
  }
  ctx->xin_mem = nullptr;
  ctx->xin_bytes = 0;
  ctx->x_base.clear();
  ctx->x_mapped = false;
}

// A (new) inbox of xislot runs per sender and round parity, zeroed (no tag matches a round).
// Uncached device memory: peers' stores reach it over xGMI and no L2 — the writer's or this
// GPU's — keeps a copy, so the tags polled and the runs read here are the memory's. The old
// inbox and the peer mappings go (the caller maps the new ones).
int xinbox_alloc(sgn_ctx* ctx, uint64_t xislot) {
  DevSim& S = ctx->S;
  const XLay l = xlay(ctx->nranks, xislot, S.G, S.xbk);
  void* p = nullptr;
  // (a local group's shards share this GPU: ordinary device memory, device-scope accesses;
  // one shard per GPU: uncached, the peers write it over xGMI)
  S.xsys = ctx->comm_local ? 0u : 1u;
  hipError_t e = S.xsys ? hipExtMallocWithFlags(&p, l.bytes, hipDeviceMallocUncached) : hipMalloc(&p, l.bytes);
  if (e != hipSuccess) return set_error(ctx, SGN_ENOMEM, std::string("inbox allocation: ") + hipGetErrorString(e));
  if ((e = hipMemset(p, 0, l.bytes)) != hipSuccess) {
    (void)hipFree(p);
    return hip_fail(ctx, e, "hipMemset (inbox)");
  }
  xinbox_release(ctx);
  ctx->xin_mem = p;
  ctx->xin_bytes = l.bytes;
  ctx->sim_bytes += l.bytes;
  S.xin_hdr = (decltype(S.xin_hdr))((char*)p + l.hdr);
  S.xin_cen = (decltype(S.xin_cen))((char*)p + l.cen);
  S.xin_runs = (decltype(S.xin_runs))((char*)p + l.runs);
  S.xislot = (uint32_t)xislot;
  S.xin_bins = S.xbk ? (decltype(S.xin_bins))((char*)p + l.bins) : nullptr;
  return 0;
}

// This shard's XPeer table: its slot, header and census word in every shard's inbox
// (ctx->x_base, by rank; none before the mapping) and the RCCL transport's send blocks.
int xpeer_upload(sgn_ctx* ctx) {
  DevSim& S = ctx->S;
  const uint32_t R = ctx->nranks, s = ctx->rank;
  std::vector<XPeer> xp(R);
  std::memset(xp.data(), 0, R * sizeof(XPeer));
  for (uint32_t q = 0; q < R; q++) {
    XPeer& x = xp[q];
    char* b = q < ctx->x_base.size() ? ctx->x_base[q] : nullptr;
    const uint32_t Gq = q < ctx->x_G.size() ? ctx->x_G[q] : 0;
    const XLay l = xlay(R, S.xislot, Gq, S.xbk);  // (receiver q's inbox)
    if (b) {
      for (uint32_t k = 0; k < 2; k++) {
        x.runs[k] = (std::remove_reference_t<decltype(x.runs[k])>)((EvRec*)(b + l.runs) + ((size_t)k * R + s) * S.xislot);
        x.hdr[k] = (std::remove_reference_t<decltype(x.hdr[k])>)((uint64_t*)(b + l.hdr) + ((size_t)k * R + s) * XH_WORDS);
        if (S.xbk)
          x.bins[k] = (std::remove_reference_t<decltype(x.bins[k])>)((EvRec*)(b + l.bins) + ((size_t)k * R + s) * Gq * S.xbk);
      }
      x.cen = (decltype(x.cen))((uint64_t*)(b + l.cen) + s);
    }
    if (S.xout) x.runs[2] = (std::remove_reference_t<decltype(x.runs[2])>)((EvRec*)S.xout + (size_t)q * (S.xslot + XHDR) + XHDR);
  }
  SGN_HIP(ctx, hipMemcpy(ctx->d_xp, xp.data(), R * sizeof(XPeer), hipMemcpyHostToDevice));
  return 0;
}

// The persistent multi-shard path runs where the persistent kernel would (the bucket -> slab
// table in LDS, no per-packet trace) unless refused before or switched off (SGN_XPERSIST=0 or
// SGN_PERSISTENT=0: per-round launches and the RCCL / local-copy exchange).
bool xpersist_possible(sgn_ctx* ctx) {
  // (read per call, like the single-shard path's SGN_PERSISTENT: a test that changes either
  // variable within one process must see it — ADVICE r5)
  const bool off = (getenv("SGN_XPERSIST") && atoi(getenv("SGN_XPERSIST")) == 0) ||
                   (getenv("SGN_PERSISTENT") && atoi(getenv("SGN_PERSISTENT")) == 0);
  return ctx->nranks > 1 && ctx->nranks <= XR_MAX && ctx->sim_ready && ctx->xin_mem && ctx->S.NB <= LDS_BSLAB &&
         !ctx->S.trace_on &&
         !ctx->x_off && !ctx->persist_off && !off;
}

// runs into this shard's calendar at a held round edge (k_inject: the bucket's current slab)
int inject_runs(sgn_ctx* ctx, const std::vector<EvRec>& runs) {
  if (runs.empty()) return 0;
  void* d = nullptr;
  SGN_HIP(ctx, hipMalloc(&d, runs.size() * sizeof(EvRec)));
  hipError_t e = hipMemcpy(d, runs.data(), runs.size() * sizeof(EvRec), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_inject, dim3((uint32_t)((runs.size() + 255) / 256)), dim3(256), 0, ctx->stream,
                       (const DevSim*)ctx->d_S, (const EvRec*)d, (uint32_t)runs.size());
    e = hipStreamSynchronize(ctx->stream);
  }
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(ctx, e, "inject_runs");
  return 0;
}

namespace {
const void* rounds_x_fn(uint32_t kind) {
  if (kind == SGN_TRAFFIC_TGEN) return (const void*)k_rounds_x<SGN_TRAFFIC_TGEN>;
  if (kind == SGN_TRAFFIC_EXTERNAL) return (const void*)k_rounds_x<SGN_TRAFFIC_EXTERNAL>;
  return (const void*)k_rounds_x<SGN_TRAFFIC_PERIODIC>;
}

// One k_rounds_x launch of up to n rounds over the shards sh (all on sh[0]'s GPU and stream).
// Returns 1 when no resident grid can be sized (the caller falls back to per-round launches).
int x_launch(const std::vector<sgn_ctx*>& sh, bool peers, uint32_t n) {
  sgn_ctx* c0 = sh[0];
  const uint32_t kind = c0->S.tkind;
  size_t lds = 0;
  uint64_t sumG = 0;
  for (sgn_ctx* c : sh) {
    lds = std::max(lds, exec_lds_bytes(c->S.CAP, c->S.agg_bmin ? c->S.NB : 0));
    sumG += c->S.G;
  }
  const uint64_t res = resident_wg(c0, rounds_x_fn(kind), lds) / std::max<uint32_t>(1, peers ? c0->x_share : 1);
  // A refusal is decided here, from this GPU's LDS and residency alone (CAP may differ between
  // shards after their re-layouts). A local group falls back at once; one shard per GPU must not,
  // or its peers would launch and wait for it: it launches ONE workgroup that publishes "not
  // resident" to every peer's census word, and every shard falls back together.
  bool refuse = !res || res < sh.size();
  // (test hook: this rank refuses as if its GPU could not hold the grid)
  if (peers && getenv("SGN_XREFUSE_RANK") && atoi(getenv("SGN_XREFUSE_RANK")) == (int)c0->rank) refuse = true;
  if (refuse && !peers) return 1;
  if (!c0->x_hxl) SGN_HIP(c0, hipHostMalloc(&c0->x_hxl, sizeof(XLaunch), 0));
  XLaunch& xl = *(XLaunch*)c0->x_hxl;
  std::memset(&xl, 0, sizeof(xl));
  xl.n_local = (uint32_t)sh.size();
  xl.peers_census = peers ? 1u : 0u;
  xl.refuse = refuse ? 1u : 0u;
  xl.epoch = ++c0->x_epoch;
  uint32_t b = 0;
  const char* cap_env = getenv("SGN_PERSIST_GRID");
  for (size_t i = 0; i < sh.size(); i++) {
    sgn_ctx* c = sh[i];
    uint64_t P = std::max<uint64_t>(1, std::min<uint64_t>(c->S.G, res * c->S.G / sumG));
    if (cap_env) P = std::max<uint64_t>(1, std::min<uint64_t>(P, (uint64_t)atoi(cap_env)));
    P = std::min<uint64_t>(P, 64 * RB_CH);
    if (refuse) P = 1;
    xl.base[i] = b;
    xl.S[i] = (std::remove_reference_t<decltype(xl.S[i])>)c->d_S;
    b += (uint32_t)P;
    c->x_grid = (uint32_t)P;
    const DevSim& S = c->S;
    (void)S;  // (no per-launch memsets: each shard's launch resets its round buffers itself)
  }
  xl.base[sh.size()] = b;
  xl.res_base = c0->res_base;  // (the census counts in the first shard's control block)
  if (!refuse) c0->res_base += b;  // (a refused launch runs no census)
  if (refuse) lds = 0;             // (its one workgroup leaves before touching the dynamic LDS)
  SGN_HIP(c0, hipMemcpyAsync(c0->d_xl, &xl, sizeof(XLaunch), hipMemcpyHostToDevice, c0->stream));
  time_begin(c0, K_EXECUTE);
  const dim3 grid(b), block(64);
  const XLaunch* d = (const XLaunch*)c0->d_xl;
  if (kind == SGN_TRAFFIC_TGEN)
    hipLaunchKernelGGL((k_rounds_x<SGN_TRAFFIC_TGEN>), grid, block, lds, c0->stream, d, n);
  else if (kind == SGN_TRAFFIC_EXTERNAL)
    hipLaunchKernelGGL((k_rounds_x<SGN_TRAFFIC_EXTERNAL>), grid, block, lds, c0->stream, d, n);
  else
    hipLaunchKernelGGL((k_rounds_x<SGN_TRAFFIC_PERIODIC>), grid, block, lds, c0->stream, d, n);
  time_end(c0);
  c0->kt[K_EXECUTE].total++;
  SGN_HIP(c0, hipGetLastError());
  for (sgn_ctx* c : sh) {
    c->x_launches++;
    c->x_mode = 2;
  }
  return 0;
}

// A round edge held by k_rounds_x (every shard the same flags): runs past an inbox slot go from
// the senders' spill areas into their shards' calendars, and the inboxes grow; then each shard's
// own pools (resolve_hold). sh: every shard of the group (local) or this GPU's one (peers).
int x_resolve(const std::vector<sgn_ctx*>& sh, bool peers) {
  uint32_t hold = 0;
  uint64_t hwm = 0;
  for (sgn_ctx* c : sh) {
    hold |= c->h_ctrl->hold;
    hwm = std::max<uint64_t>(hwm, c->h_ctrl->xhwm);
  }
  const uint32_t xf = HOLD_XSLOT | HOLD_XGROW;
  if (!(hold & xf)) {
    for (sgn_ctx* c : sh)
      if (int rc = resolve_hold(c)) return rc;
    return 0;
  }
  for (sgn_ctx* c : sh) {  // the inbox flags are this function's: cleared before any growth
    c->h_ctrl->hold &= ~xf;
    SGN_HIP(c, hipMemcpy((char*)c->S.ctrl + offsetof(Ctrl, hold), &c->h_ctrl->hold, 4, hipMemcpyHostToDevice));
  }
  if (hold & HOLD_XSLOT) {
    // each sender's runs past a peer's slot (spill-area entries tagged SPILL_PEER | peer)
    std::vector<std::vector<std::vector<EvRec>>> out(sh.size());
    for (size_t i = 0; i < sh.size(); i++) {
      sgn_ctx* c = sh[i];
      const DevSim& S = c->S;
      out[i].assign(c->nranks, {});
      const uint64_t n = std::min<uint64_t>(c->h_ctrl->spill_n, S.spill_cap);
      if (!n) continue;
      std::vector<uint32_t> idx(n);
      std::vector<EvRec> rec(n);
      SGN_HIP(c, hipMemcpy(idx.data(), (const void*)S.spill_idx, n * 4, hipMemcpyDeviceToHost));
      SGN_HIP(c, hipMemcpy(rec.data(), (const void*)S.spill, n * sizeof(EvRec), hipMemcpyDeviceToHost));
      bool any = false;
      for (uint64_t k = 0; k < n; k++)
        if ((idx[k] & SPILL_PEER) && idx[k] != SPILL_DEAD) {
          out[i][idx[k] & ~SPILL_PEER].push_back(rec[k]);
          idx[k] = SPILL_DEAD;
          any = true;
        }
      if (any) SGN_HIP(c, hipMemcpy((void*)S.spill_idx, idx.data(), n * 4, hipMemcpyHostToDevice));
    }
    if (!peers) {
      for (size_t i = 0; i < sh.size(); i++)
        for (uint32_t q = 0; q < sh[i]->nranks; q++) {
          sh[q]->x_moved += out[i][q].size();
          if (int rc = inject_runs(sh[q], out[i][q])) return rc;
        }
    } else {
      std::vector<EvRec> in;
      if (int rc = comm_xmove_spills(sh[0], out[0], &in)) return rc;
      sh[0]->x_moved += in.size();
      if (int rc = inject_runs(sh[0], in)) return rc;
    }
    for (sgn_ctx* c : sh) c->x_over_rounds++;
  }
  // larger inboxes: 4x the largest per-peer count any round produced (every shard sees the same
  // maximum: the same size everywhere), at least twice the slot
  uint64_t ns = sh[0]->S.xislot;
  do ns *= 2;
  while (ns < 4 * hwm);
  if (ns > (1ULL << 26)) return set_error(sh[0], SGN_EOVERFLOW, "inbox slot above 2^26 runs per sender");
  for (sgn_ctx* c : sh)
    if (int rc = xinbox_alloc(c, ns)) return rc;
  if (!peers) {
    std::vector<char*> base(sh.size());
    for (size_t i = 0; i < sh.size(); i++) base[sh[i]->rank] = (char*)sh[i]->xin_mem;
    for (sgn_ctx* c : sh) {
      c->x_base = base;
      if (int rc = xpeer_upload(c)) return rc;
      c->x_mapped = true;
    }
  } else {
    if (int rc = comm_xpeer_map(sh[0])) return rc;
    if (!sh[0]->x_mapped) return set_error(sh[0], SGN_EDEVICE, "inbox growth: the peers' new inboxes could not be mapped");
  }
  for (sgn_ctx* c : sh) {
    c->x_grows++;
    if (int rc = upload_sim(c)) return rc;
    if (int rc = sync_ctrl(c)) return rc;  // (the injected runs' occupancy and spills)
    if (int rc = resolve_hold(c)) return rc;
  }
  return 0;
}
}  // namespace

// Rounds through k_rounds_x until max_rounds, the end, or a refused census (every shard's x_off
// set: the caller goes on with per-round launches). sh: the shards of one launch — a local
// group's (rank order) or this GPU's one (peers: the census and messages cross GPUs).
int run_xpersist(const std::vector<sgn_ctx*>& sh, bool peers, uint64_t max_rounds, uint64_t* rounds_done) {
  sgn_ctx* c0 = sh[0];
  for (sgn_ctx* c : sh)
    if (int rc = sync_ctrl(c)) return rc;
  const uint64_t r_start = c0->h_ctrl->rounds;
  uint64_t enq = 0;
  int rc = 0;
  // (a round still held from an earlier call: its pools first)
  if (!rc) rc = x_resolve(sh, peers);
  while (!rc && c0->h_ctrl->active && enq < max_rounds) {
    const uint32_t n = (uint32_t)std::min<uint64_t>(kPersistRounds, max_rounds - enq);
    const int lr = x_launch(sh, peers, n);
    if (lr < 0) return lr;
    if (lr == 0) SGN_HIP(c0, hipStreamSynchronize(c0->stream));
    for (sgn_ctx* c : sh)
      if ((rc = sync_ctrl(c))) break;
    if (rc) break;
    if (lr == 1 || census_verdict(c0, (uint32_t)c0->x_epoch) != 1) {
      // not resident (here or on a peer): nothing ran; per-round launches from now on
      for (sgn_ctx* c : sh) {
        c->x_off = true;
        c->x_mode = 1;
        c->persist_fallbacks++;
      }
      break;
    }
    rc = x_resolve(sh, peers);
    enq = c0->h_ctrl->rounds - r_start;
  }
  for (sgn_ctx* c : sh)  // (the per-round path counts its sends in row 0 from zero)
    if (c->S.xout_n) (void)hipMemsetAsync((void*)c->S.xout_n, 0, (6 * (size_t)c->nranks + 8) * 4, c->stream);
  if (rounds_done) *rounds_done = c0->h_ctrl->rounds - r_start;
  return rc;
}

void free_sim(sgn_ctx* ctx) {
  drop_graph(ctx);
  xinbox_release(ctx);
  if (ctx->x_hxl) (void)hipHostFree(ctx->x_hxl);
  ctx->x_hxl = nullptr;
  ctx->d_xp = ctx->d_xl = nullptr;  // (in allocs)
  ctx->x_mapped = false;
  ctx->rng_held.clear();
  if (ctx->d_rng_stage) hipFree(ctx->d_rng_stage);
  ctx->d_rng_stage = nullptr;
  ctx->rng_stage_cap = 0;
  for (void* p : ctx->allocs) hipFree(p);
  ctx->allocs.clear();
  ctx->sim_bytes = 0;
  if (ctx->d_stage) hipFree(ctx->d_stage);
  ctx->d_stage = nullptr;
  ctx->stage_cap = 0;
  if (ctx->h_ctrl) {
    hipHostFree(ctx->h_ctrl);
    ctx->h_ctrl = nullptr;
  }
  if (ctx->h_mirror) {
    hipHostFree(ctx->h_mirror);
    ctx->h_mirror = nullptr;
  }
  ctx->ctrl_fresh = false;
  ctx->sim_ready = false;
}

}  // namespace sgn

extern "C" {

int sgn_trace_enable(sgn_ctx* ctx, uint64_t capacity) {
  if (!ctx) return SGN_EINVAL;
  if (ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "sgn_trace_enable must precede sgn_sim_init");
  ctx->trace_cap = capacity;
  return 0;
}

int sgn_sim_init(sgn_ctx* ctx, const sgn_sim_config* cfg, const sgn_traffic* tr) {
  if (ctx) ctx->ctrl_fresh = false;  // (it may change the device control block)
  if (!ctx || !cfg || !tr) return SGN_EINVAL;
  if (!ctx->routes_ready) return set_error(ctx, SGN_ESTATE, "sgn_routes_build must precede sgn_sim_init");
  if (!ctx->hosts_ready) return set_error(ctx, SGN_ESTATE, "sgn_hosts_set must precede sgn_sim_init");
  if (tr->kind != SGN_TRAFFIC_PERIODIC && tr->kind != SGN_TRAFFIC_TGEN &&
      tr->kind != SGN_TRAFFIC_EXTERNAL)
    return set_error(ctx, SGN_EINVAL, "unknown traffic kind");
  if (cfg->out_fifo_cap == 0 || cfg->codel_cap == 0)
    return set_error(ctx, SGN_EINVAL, "out_fifo_cap and codel_cap must be >= 1");
  if (tr->kind == SGN_TRAFFIC_PERIODIC && tr->payload_len > 0xFFFFu)
    return set_error(ctx, SGN_EINVAL, "payload_len must fit a UDP datagram");
  if (tr->kind == SGN_TRAFFIC_TGEN && (tr->n_servers == 0 || !tr->server_hosts))
    return set_error(ctx, SGN_EINVAL, "TGEN traffic needs servers");
  if (tr->kind == SGN_TRAFFIC_TGEN && tr->req_payload > 0xFFFFu)
    return set_error(ctx, SGN_EINVAL, "req_payload must fit a UDP datagram");
  if (ctx->sim_ready) free_sim(ctx);
  SGN_HIP(ctx, hipSetDevice(ctx->device));

  DevSim S{};
  const uint32_t nH = ctx->hi - ctx->lo;
  const uint32_t N = ctx->n_all;
  ctx->persist_off = false;
  ctx->res_epoch = ctx->res_base = 0;  // (the new control block's census words are zero)
  ctx->codel_grows = ctx->cal_grows = ctx->cal_spill_runs = ctx->xslot_grows = ctx->rounds_held = 0;
  ctx->codel_allocs_before = 0;
  ctx->ext_slabs = ctx->spill_grows = 0;
  ctx->h_ext.clear();
  ctx->failed.clear();
  S.n_all = N;
  S.lo = ctx->lo;
  S.nH = nH;
  S.U = ctx->U;
  S.end_time = SIM_START + cfg->stop_time_ns;
  S.boot_end = SIM_START + cfg->bootstrap_end_ns;
  S.runahead_cfg = cfg->runahead_ns;
  S.dynamic = cfg->use_dynamic_runahead ? 1 : 0;
  S.fifo_cap = cfg->out_fifo_cap;
  if (cfg->interface_qdisc > SGN_QDISC_ROUND_ROBIN) return set_error(ctx, SGN_EINVAL, "unknown interface_qdisc");
  S.qdisc_rr = cfg->interface_qdisc == SGN_QDISC_ROUND_ROBIN ? 1u : 0u;
  // CoDel page pool: codel_cap run slots per host on average, at least one page per host
  // (its first) plus 64 to share
  {
    const uint64_t pages = std::max<uint64_t>((uint64_t)nH + 64, ((uint64_t)nH * cfg->codel_cap + CQ_PAGE - 1) / CQ_PAGE);
    if (pages >= (1ULL << 28)) return set_error(ctx, SGN_EINVAL, "codel_cap: CoDel page pool above 2^28 pages");
    S.cq_pages = (uint32_t)pages;
  }
  S.trace_on = ctx->trace_cap > 0;
  S.tkind = tr->kind;
  S.payload_len = tr->payload_len;
  S.unknown_permille = tr->unknown_dst_permille;
  S.req_payload = tr->req_payload;
  S.n_servers = tr->kind == SGN_TRAFFIC_TGEN ? tr->n_servers : 0;
  S.flow_seed = tr->flow_seed;
  S.period = tr->period_ns;
  S.period_jitter = tr->period_jitter_ns;
  for (int i = 0; i < 3; i++) S.file_bytes[i] = tr->file_bytes[i];

  const uint64_t min_possible = ctx->lat_min, max_lat = ctx->lat_max;
  S.min_possible = min_possible;
  S.max_lat = max_lat;
  if (min_possible == 0) return set_error(ctx, SGN_EINVAL, "route latency 0 (Runahead::new asserts)");

  // routing (device copies made by sgn_routes_build)
  S.rlat = (decltype(S.rlat))ctx->d_lat;
  S.rloss = (decltype(S.rloss))ctx->d_loss;
  uint32_t* d_unode = dalloc<uint32_t>(ctx, N);
  uint32_t* d_ip = dalloc<uint32_t>(ctx, N);
  uint32_t* d_dk = dalloc<uint32_t>(ctx, ctx->dns_key.size());
  uint32_t* d_dv = dalloc<uint32_t>(ctx, ctx->dns_val.size());
  if (!d_unode || !d_ip || !d_dk || !d_dv) return set_error(ctx, SGN_ENOMEM, "device allocation failed");
  SGN_HIP(ctx, hipMemcpy(d_unode, ctx->unode.data(), N * 4, hipMemcpyHostToDevice));
  SGN_HIP(ctx, hipMemcpy(d_ip, ctx->ip.data(), N * 4, hipMemcpyHostToDevice));
  SGN_HIP(ctx, hipMemcpy(d_dk, ctx->dns_key.data(), ctx->dns_key.size() * 4, hipMemcpyHostToDevice));
  SGN_HIP(ctx, hipMemcpy(d_dv, ctx->dns_val.data(), ctx->dns_val.size() * 4, hipMemcpyHostToDevice));
  S.unode = (decltype(S.unode))d_unode;
  S.ip = (decltype(S.ip))d_ip;
  S.dns_key = (decltype(S.dns_key))d_dk;
  S.dns_val = (decltype(S.dns_val))d_dv;
  S.dns_mask = ctx->dns_mask;
  std::vector<uint8_t> is_server(N, 0);
  if (tr->kind == SGN_TRAFFIC_TGEN) {
    uint32_t* d_sv = dalloc<uint32_t>(ctx, tr->n_servers);
    if (!d_sv) return set_error(ctx, SGN_ENOMEM, "device allocation failed");
    for (uint32_t i = 0; i < tr->n_servers; i++) {
      if (tr->server_hosts[i] >= N) return set_error(ctx, SGN_EINVAL, "server host out of range");
      is_server[tr->server_hosts[i]] = 1;
    }
    SGN_HIP(ctx, hipMemcpy(d_sv, tr->server_hosts, tr->n_servers * 4, hipMemcpyHostToDevice));
    S.servers = (decltype(S.servers))d_sv;
  }

  // ---- host slots: every shard's HostId range, permuted so that hosts of one kind share
  // waves (TGEN: servers by uplink, then clients by downlink; otherwise by bandwidth, then by
  // graph node: a wave's sends then read one row of the route table, and an XCD's workgroups
  // a few hundred rows instead of all of them — config D's ~1 k hosts per node fill whole
  // waves, so its random-peer route lookups become L2 hits). The
  // permutation only places hosts on lanes; semantics follow HostIds. SGN_HOST_ORDER=id keeps
  // HostId order (test hook). Every shard computes every shard's permutation (same inputs).
  {
    const bool by_id = getenv("SGN_HOST_ORDER") && std::string(getenv("SGN_HOST_ORDER")) == "id";
    ctx->sid_of.assign(N, 0);
    std::vector<uint32_t> order;
    for (uint32_t rk = 0; rk < ctx->nranks; rk++) {
      uint32_t lo = 0, hi = 0;
      sgn_shard_range(N, rk, ctx->nranks, &lo, &hi);
      order.resize(hi - lo);
      for (uint32_t i = lo; i < hi; i++) order[i - lo] = i;
      if (!by_id) {
        auto key = [&](uint32_t i) {
          if (tr->kind == SGN_TRAFFIC_TGEN)
            return std::make_tuple(is_server[i] ? 0u : 1u, is_server[i] ? ctx->bw_up[i] : ctx->bw_down[i], (uint64_t)i);
          return std::make_tuple(0u, ctx->bw_up[i] ^ (ctx->bw_down[i] << 1), (uint64_t)ctx->unode[i] << 32 | i);
        };
        std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
      }
      for (uint32_t k = 0; k < hi - lo; k++) ctx->sid_of[order[k]] = lo + k;
      if (rk == ctx->rank) ctx->host_of = order;
    }
  }
  // ---- per-host state records (one per slot), initialised on the host ----
  std::vector<HostRec> recs(nH);
  std::vector<HostConst> hk(nH);
  std::vector<uint64_t> nextloc(nH, INVALID);
  std::memset(recs.data(), 0, recs.size() * sizeof(HostRec));
  std::memset(hk.data(), 0, hk.size() * sizeof(HostConst));
  for (uint32_t h = 0; h < nH; h++) {
    const uint32_t g = ctx->host_of[h];
    HostRec& r = recs[h];
    HostConst& k = hk[h];
    k.gid = r.k_gid = g;
    k.ip = r.k_ip = ctx->ip[g];
    k.unode = r.k_unode = ctx->unode[g];
    // Xoshiro256PlusPlus::seed_from_u64 (SplitMix64 fill), host.rs:234
    uint64_t sm = ctx->seed[g];
    for (int i = 0; i < 4; i++) r.rng[i] = host_splitmix(sm);
    r.st0 = r.st1 = r.st2 = INVALID;
    // create_token_bucket (relay/mod.rs:278-288) for inet_out (up) and inet_in (down)
    for (int w = 0; w < 2; w++) {
      const uint64_t bps = (w == 0 ? ctx->bw_up[g] : ctx->bw_down[g]) / 8;
      const uint64_t inc = std::max<uint64_t>(1, bps / 1000);
      k.tb_inc[w] = r.k_tbinc[w] = inc;  // (capacity = inc + MTU, the bucket starts full)
      r.tb_bal[w] = inc + SGN_CONFIG_MTU;
      r.tb_last[w] = SIM_START;
    }
    for (int i = 0; i < 3; i++) r.dig[i] = SGN_DIGEST_SEED;
    r.rc_dst = NO_HOST;  // empty route cache
    r.cq_head = h * CQ_PAGE;  // CoDel chain: page h
    r.cq_tp = h;
    if (is_server[g]) r.flags |= F_SERVER;
    const bool has_app = tr->kind == SGN_TRAFFIC_PERIODIC || (tr->kind == SGN_TRAFFIC_TGEN && !is_server[g]);
    if (has_app) {
      r.flags |= F_HAS_APP;
      const uint64_t t = SIM_START + sgn_app_start_rel(tr->flow_seed, g, tr->start_ns, tr->start_jitter_ns);
      const uint64_t e = r.eid++;
      if (t < S.end_time) {
        r.st2 = t;
        r.se2 = e;
        nextloc[h] = t;
      }
    }
  }
  auto up64 = [&](const std::vector<uint64_t>& v, auto* out) -> int {
    *out = (std::remove_reference_t<decltype(*out)>)dalloc<uint64_t>(ctx, v.size());
    if (!*out) return set_error(ctx, SGN_ENOMEM, "device allocation failed");
    SGN_HIP(ctx, hipMemcpy((void*)*out, v.data(), v.size() * 8, hipMemcpyHostToDevice));
    return 0;
  };
  auto up32 = [&](const std::vector<uint32_t>& v, auto* out) -> int {
    *out = (std::remove_reference_t<decltype(*out)>)dalloc<uint32_t>(ctx, v.size());
    if (!*out) return set_error(ctx, SGN_ENOMEM, "device allocation failed");
    SGN_HIP(ctx, hipMemcpy((void*)*out, v.data(), v.size() * 4, hipMemcpyHostToDevice));
    return 0;
  };
  int rc = 0;
  if ((rc = up32(ctx->sid_of, &S.sid_of)) || (rc = up32(ctx->host_of, &S.host_of))) return rc;
  {  // the packet path's peer and route forms (send_batch: two loads per route-cache miss)
    std::vector<uint64_t> pe(N);
    for (uint32_t i = 0; i < N; i++) pe[i] = (uint64_t)ctx->sid_of[i] | ((uint64_t)ctx->unode[i] << 32);
    if ((rc = up64(pe, &S.peer))) return rc;
    // the 4-byte form when slot ids and node indices fit together (sid < N, node < U)
    uint32_t sb = 1, ub = 1;
    while (sb < 32 && (1ull << sb) < N) sb++;
    while (ub < 32 && (1ull << ub) < ctx->U) ub++;
    S.peer32 = nullptr;
    S.peer_sb = sb;
    if (sb + ub <= 32 && !getenv("SGN_PEER64")) {
      std::vector<uint32_t> p32(N);
      for (uint32_t i = 0; i < N; i++) p32[i] = ctx->sid_of[i] | (ctx->unode[i] << sb);
      if ((rc = up32(p32, &S.peer32))) return rc;
    }
    if ((rc = ensure_host_routes(ctx))) return rc;
    const size_t UU = (size_t)ctx->U * ctx->U;
    std::vector<RouteEnt> re(UU);
    for (size_t i = 0; i < UU; i++) {
      // reliability = (f64)(1.0f - loss) (worker.rs:363-371), exactly as the device would
      volatile float rel32 = 1.0f - ctx->h_loss[i];
      re[i].lat = ctx->h_lat[i];
      re[i].T = (uint64_t)((double)rel32 * 9007199254740992.0);
    }
    RouteEnt* d = (RouteEnt*)dev_alloc(ctx, UU * sizeof(RouteEnt), false);
    if (!d) return set_error(ctx, SGN_ENOMEM, "device allocation failed (route table)");
    SGN_HIP(ctx, hipMemcpy(d, re.data(), UU * sizeof(RouteEnt), hipMemcpyHostToDevice));
    S.route = (decltype(S.route))d;
  }
  S.hrec = (decltype(S.hrec))dalloc<HostRec>(ctx, nH);
  S.codel = (decltype(S.codel))dalloc<CodelEnt>(ctx, (size_t)S.cq_pages * CQ_PAGE);
  S.cq_next = (decltype(S.cq_next))dalloc<uint32_t>(ctx, S.cq_pages);
  {  // host slot h starts with page h; pages nH.. are the free ring's first entries
    std::vector<uint32_t> fr(S.cq_pages, 0);
    for (uint32_t i = 0; i + nH < S.cq_pages; i++) fr[i] = nH + i;
    if ((rc = up32(fr, &S.cq_free))) return rc;
  }
  S.rb_free = (decltype(S.rb_free))dalloc<uint64_t>(ctx, 3);
  S.fifo = (decltype(S.fifo))dalloc<FifoEnt>(ctx, (size_t)nH * cfg->out_fifo_cap);
  S.fifo_addr = nullptr;
  if (ctx->trace_cap) {
    S.fifo_addr = (decltype(S.fifo_addr))dalloc<uint32_t>(ctx, (size_t)nH * cfg->out_fifo_cap);
    if (!S.fifo_addr) return set_error(ctx, SGN_ENOMEM, "device allocation failed (trace)");
  }
  if (!S.hrec || !S.codel || !S.fifo || !S.cq_next || !S.rb_free)
    return set_error(ctx, SGN_ENOMEM, "device allocation failed (host state)");
  SGN_HIP(ctx, hipMemcpy((void*)S.hrec, recs.data(), recs.size() * sizeof(HostRec), hipMemcpyHostToDevice));
  S.htile = nullptr;
  if (tr->kind == SGN_TRAFFIC_PERIODIC) {  // the hot lines, tiled (kSoa)
    const size_t nt = ((size_t)nH + 63) / 64;
    std::vector<uint64_t> tile(nt * 8 * 64 * 2, 0);
    for (uint32_t h = 0; h < nH; h++)
      for (uint32_t c = 0; c < 8; c++) std::memcpy(&tile[2 * hot_idx(h, c)], (const char*)&recs[h] + 16 * c, 16);
    S.htile = (decltype(S.htile))dalloc<uint64_t>(ctx, tile.size());
    if (!S.htile) return set_error(ctx, SGN_ENOMEM, "device allocation failed (host tiles)");
    SGN_HIP(ctx, hipMemcpy((void*)S.htile, tile.data(), tile.size() * 8, hipMemcpyHostToDevice));
  }
  {
    HostConst* dk = dalloc<HostConst>(ctx, nH);
    S.n_cnt = (decltype(S.n_cnt))dalloc<uint64_t>(ctx, (size_t)N_CNT * nH);
    S.maxq = (decltype(S.maxq))dalloc<uint32_t>(ctx, nH);
    if (!dk || !S.n_cnt || !S.maxq) return set_error(ctx, SGN_ENOMEM, "device allocation failed (host state)");
    SGN_HIP(ctx, hipMemcpy(dk, hk.data(), hk.size() * sizeof(HostConst), hipMemcpyHostToDevice));
    S.hconst = (decltype(S.hconst))dk;
  }
  if ((rc = up64(nextloc, &S.nextloc))) return rc;
  S.npeer = nullptr;
  if (tr->kind == SGN_TRAFFIC_PERIODIC) {  // every app counter starts at 0
    std::vector<uint32_t> np(nH);
    for (uint32_t h = 0; h < nH; h++) {
      uint32_t peer = NO_HOST, uip = 0;
      np[h] = sgn_periodic_dst(tr->flow_seed, ctx->host_of[h], 0, N, tr->unknown_dst_permille, &peer, &uip) ? peer : NO_HOST;
    }
    if ((rc = up32(np, &S.npeer))) return rc;
  }

  // ---- calendar: bucket width >= any window length, horizon > max latency ----
  // The shortest possible window (Runahead::get, runahead.rs:44-57): a window spans at least
  // one bucket, and in dynamic mode possibly many (executed bucket by bucket).
  uint64_t BW = std::max<uint64_t>(1, std::max(min_possible, cfg->runahead_ns));
  // Every pending event lies in [ws, we + max_lat): sends happen before the window end and
  // arrive at most max_lat later (worker.rs:386-390). A static window is BW long; a dynamic
  // one is max(min used latency, configured runahead) (runahead.rs:44-57), i.e. up to
  // max(max_lat, runahead). The calendar spans that plus one partial bucket at each end;
  // send_batch checks the horizon on the device (OVF_HORIZON), so a violation is reported.
  // The persistent kernel resets a round's consumed buckets during the next round, so one more
  // window of slack keeps the next round's sends off them (see k_rounds).
  const uint64_t wmax = cfg->use_dynamic_runahead ? std::max<uint64_t>(BW, std::max(max_lat, cfg->runahead_ns)) : BW;
  uint64_t NB = (3 * wmax + max_lat) / BW + 8;
  if (NB > (1u << 20)) return set_error(ctx, SGN_EINVAL, "calendar would need > 2^20 buckets");
  while (NB & (NB - 1)) NB += NB & (~NB + 1);  // round up to a power of two
  // hosts per k_execute wave: fewer than 64 spreads the (divergent, per-lane serial) host
  // work of a round over more waves; sgn_sim_config.hosts_per_wave (0 = default 64)
  uint32_t gsz = cfg->hosts_per_wave ? cfg->hosts_per_wave : 64;
  if (const char* e = getenv("SGN_HOSTS_PER_WAVE")) gsz = (uint32_t)atoi(e);
  if (gsz == 0 || gsz > GROUP_MAX || (gsz & (gsz - 1)))
    return set_error(ctx, SGN_EINVAL, "hosts_per_wave must be a power of two in [1, 64]");
  S.gsh = (uint32_t)__builtin_ctz(gsz);
  const uint64_t G = (nH + gsz - 1) / gsz;
  uint64_t cap = cfg->event_capacity ? cfg->event_capacity : (1ULL << 22);
  uint64_t CAP = cap / ((NB + 1) * G);
  CAP = std::max<uint64_t>(CAP_MIN, std::min<uint64_t>(CAP_MAX, CAP));
  // test hook: small slabs, so that rounds spill runs and the calendar is re-laid out
  if (const char* e = getenv("SGN_SLAB_CAP")) CAP = std::max<uint64_t>(16, std::min<uint64_t>(CAP_MAX, atoll(e)));
  S.NB = (uint32_t)NB;
  S.G = (uint32_t)G;
  S.CAP = (uint32_t)CAP;
  S.BW = BW;
  S.bw_div.init(BW);
  S.div_n.init(std::max<uint64_t>(1, N));
  S.div_1000.init(1000);
  S.div_ns.init(std::max<uint64_t>(1, S.n_servers));
  S.pool = (decltype(S.pool))dalloc<EvRec>(ctx, (NB + 1) * G * CAP);
  S.w_cnt = (decltype(S.w_cnt))dalloc<uint64_t>(ctx, W_N * G);
  if (!S.w_cnt) return set_error(ctx, SGN_ENOMEM, "device allocation failed (wave slots)");
  S.slab_n = (decltype(S.slab_n))dalloc<uint32_t>(ctx, (NB + 1) * G);
  if (!S.pool || !S.slab_n) return set_error(ctx, SGN_ENOMEM, "device allocation failed (event calendar)");
  std::vector<uint32_t> bslab(NB);
  for (uint64_t b = 0; b < NB; b++) bslab[b] = (uint32_t)b;
  if ((rc = up32(bslab, &S.bucket_slab))) return rc;
  std::vector<uint64_t> bmin(NB, INVALID);
  if ((rc = up64(bmin, &S.bucket_min))) return rc;
  // SGN_STAMPS=1: per-group stamps; =2: also the persistent kernel's per-round timeline (one
  // atomic min and max per workgroup and round on shared words: it slows the rounds it times)
  if (const char* e = getenv("SGN_STAMPS")) {
    S.stamps = (decltype(S.stamps))dalloc<uint64_t>(ctx, SGN_STAMP_WORDS * G);
    if (atoi(e) >= 2) {
      S.rdbg_wg = atoi(e) >= 3 ? 1u : 0u;
      S.rdbg = (decltype(S.rdbg))dalloc<uint64_t>(ctx, S.rdbg_wg ? (size_t)8 * 128 * 2048 : 8 * 128);
    }
  }
  if (ctx->trace_cap) {
    S.trace = (decltype(S.trace))dalloc<sgn_trace_rec>(ctx, ctx->trace_cap);
    if (!S.trace) return set_error(ctx, SGN_ENOMEM, "device allocation failed (trace)");
    S.trace_cap = ctx->trace_cap;
  }
  ctx->handles.clear();
  ctx->drain_held.clear();
  ctx->submit_seq.assign(nH, 0u);
  if (tr->kind == SGN_TRAFFIC_EXTERNAL) {
    const uint64_t dc = ctx->drain_cap ? ctx->drain_cap : (1ULL << 20);
    S.drain = (decltype(S.drain))dalloc<sgn_drain_rec>(ctx, dc);
    if (!S.drain) return set_error(ctx, SGN_ENOMEM, "device allocation failed (drain buffer)");
    S.drain_cap = dc;
  }
  // multi-GPU exchange slots
  S.n_ranks = ctx->nranks;
  S.rank = ctx->rank;
  {
    std::vector<uint32_t> rl(ctx->nranks + 1);
    for (uint32_t r = 0; r <= ctx->nranks; r++) {
      uint32_t lo = 0, hi = 0;
      sgn_shard_range(N, r < ctx->nranks ? r : ctx->nranks - 1, ctx->nranks, &lo, &hi);
      rl[r] = r < ctx->nranks ? lo : N;
    }
    if ((rc = up32(rl, &S.rank_lo))) return rc;
  }
  if (ctx->nranks > 1) {
    if (!ctx->comm && !ctx->comm_local)
      return set_error(ctx, SGN_ESTATE, "multi-shard context needs sgn_comm_init (or sgn_comm_init_local) before sgn_sim_init");
    S.xslot = (uint32_t)ctx->xslot;
    // per peer a block of 1 + xslot records: the 32-byte round-edge message, then the runs
    S.xout = (decltype(S.xout))dalloc<EvRec>(ctx, (size_t)ctx->nranks * (ctx->xslot + XHDR));
    S.xin = (decltype(S.xin))dalloc<EvRec>(ctx, (size_t)ctx->nranks * (ctx->xslot + XHDR));
    // (per-round launches count in row 0; k_rounds_x in row round % 3)
    // (k_rounds_x: rows [3][n_ranks] of slot counts, then [3][n_ranks] of totals, bins included)
    S.xout_n = (decltype(S.xout_n))dalloc<uint32_t>(ctx, ctx->nranks * 6 + 8);
    S.xin_n = (decltype(S.xin_n))dalloc<uint32_t>(ctx, ctx->nranks * 2 + 8);
    if (!S.xout || !S.xin || !S.xout_n || !S.xin_n) return set_error(ctx, SGN_ENOMEM, "device allocation failed (exchange)");
    // persistent rounds: the second barrier's counters, the XPeer table, the launch descriptor
    // and this shard's inbox (SGN_XISLOT: a smaller first slot, a test hook for the growth path)
    S.rb2_cnt = (decltype(S.rb2_cnt))dalloc<uint32_t>(ctx, 3 * RB_CB_MAX);
    ctx->d_xp = dalloc<XPeer>(ctx, ctx->nranks);
    ctx->d_xl = dalloc<XLaunch>(ctx, 1);
    if (!S.rb2_cnt || !ctx->d_xp || !ctx->d_xl) return set_error(ctx, SGN_ENOMEM, "device allocation failed (exchange)");
    S.xp = (decltype(S.xp))ctx->d_xp;
    S.xown = kOwnFile;
    if (const char* e = getenv("SGN_XOWN")) S.xown = (uint32_t)atoi(e);
    // inbox bins: xbk runs per (parity, sender, receiving group), a power of two;
    // SGN_XBIN: another size, 0 = none (every import through the slots)
    ctx->x_G.assign(ctx->nranks, 0u);
    S.xgx = 0;
    for (uint32_t q = 0; q < ctx->nranks; q++) {
      uint32_t lo = 0, hi = 0;
      sgn_shard_range(N, q, ctx->nranks, &lo, &hi);
      ctx->x_G[q] = (hi - lo + gsz - 1) / gsz;
      S.xgx = std::max(S.xgx, ctx->x_G[q]);
    }
    S.xbk = kXBin;
    if (const char* e = getenv("SGN_XBIN")) {  // (a test hook: small bins send runs to the slots)
      const uint32_t v = (uint32_t)atoi(e);
      S.xbk = 0;
      if (v) {
        S.xbk = 1;
        while (S.xbk < v && S.xbk < (1u << 12)) S.xbk *= 2;
      }
    }
    S.xbin_n = nullptr;
    if (S.xbk) {
      S.xbin_n = (decltype(S.xbin_n))dalloc<uint32_t>(ctx, (size_t)2 * ctx->nranks * S.xgx);
      if (!S.xbin_n) return set_error(ctx, SGN_ENOMEM, "device allocation failed (inbox bin counters)");
    }
    uint64_t xis = ctx->xslot;
    if (const char* e = getenv("SGN_XISLOT")) xis = std::max<uint64_t>(1, std::min<uint64_t>(xis, (uint64_t)atoll(e)));
    ctx->S = S;  // (xinbox_alloc / xpeer_upload work on ctx->S)
    if ((rc = xinbox_alloc(ctx, xis)) || (rc = xpeer_upload(ctx))) return rc;
    S = ctx->S;
    ctx->x_off = false;
    ctx->x_mode = 1;
    ctx->x_epoch = ctx->x_grows = ctx->x_over_rounds = ctx->x_moved = ctx->x_launches = 0;
    for (sgn_ctx* g : ctx->group)  // (a local group maps every member's inbox at its next run)
      if (g) g->x_mapped = false;
  }
  Ctrl c{};
  c.ws = SIM_START;  // initial window (manager.rs:506-509)
  c.we = SIM_START + 1;
  c.active = 1;
  c.round_min = INVALID;
  c.min_used = INVALID;
  c.keep_slab = (uint32_t)NB;
  c.keep_min = INVALID;
  c.last_min_next = INVALID;
  c.prev_we = SIM_START;
  c.pg_tail = c.pg_avail = S.cq_pages - nH;  // the free ring holds the pages beyond the hosts' first
  // multi-shard exchange size: RCCL rounds start at min(slot, kXszInit) runs per peer and
  // grow with the high-water mark; a local shard group copies counts, so it uses the slot
  ctx->xsz_cur = ctx->nranks > 1 ? (ctx->comm_local ? (uint32_t)ctx->xslot
                                                    : (uint32_t)std::min<uint64_t>(ctx->xslot, kXszInit))
                                 : 0;
  // test hook: a small first size makes the first rounds hold and complete (spill path)
  if (const char* e = getenv("SGN_XSZ_INIT"))
    if (ctx->nranks > 1 && !ctx->comm_local)
      ctx->xsz_cur = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ctx->xslot, (uint64_t)atoll(e)));
  ctx->x_spills = ctx->x_bytes = 0;
  c.xsz = ctx->xsz_cur;
  S.ctrl = (decltype(S.ctrl))dalloc<Ctrl>(ctx, 1);
  if (!S.ctrl) return set_error(ctx, SGN_ENOMEM, "device allocation failed");
  SGN_HIP(ctx, hipMemcpy(S.ctrl, &c, sizeof(c), hipMemcpyHostToDevice));
  if (!ctx->h_ctrl) SGN_HIP(ctx, hipHostMalloc((void**)&ctx->h_ctrl, sizeof(Ctrl), 0));
  static_assert(sizeof(Ctrl) % 8 == 0, "the control block's copy is written in u64 words");
  if (!ctx->h_mirror) SGN_HIP(ctx, hipHostMalloc((void**)&ctx->h_mirror, kMirrorWords * 8, 0));
  std::memset(ctx->h_mirror, 0, kMirrorWords * 8);
  {
    void* dm = nullptr;
    SGN_HIP(ctx, hipHostGetDevicePointer(&dm, ctx->h_mirror, 0));
    S.ctrl_mirror = (decltype(S.ctrl_mirror))dm;
  }
  *ctx->h_ctrl = c;
  S.fuse_finalize = ctx->nranks == 1 ? 1u : 0u;
  // PERIODIC traffic: each host receives ~BW / period runs per bucket, so a group's slab holds
  // ~gsz * BW / period; when that is a full wave (config D: 64 hosts, one send per window) all
  // 64 lanes load speculatively and the second round trip goes (same-box A/B: D +1.3 %, while
  // B's ~2-run slabs measured 1 % slower at 64 and unchanged at 4 and 8)
  // (round 4: from 4 up, twice the expected fill: config B's ~2-run slabs of 16 hosts read 4
  // records instead of 16 — its PMC traffic was 3.4x the algorithmic bytes, mostly these
  // speculative heads, while B's time measured the same at 4, 8 and 16 in round 3)
  S.gspec = GATHER_SPEC;
  if (S.tkind == SGN_TRAFFIC_PERIODIC && S.period) {
    const uint64_t fill = ((uint64_t)gsz * BW + S.period - 1) / S.period;
    S.gspec = 4;
    while (S.gspec < 64 && S.gspec < 2 * fill) S.gspec *= 2;
  }
  if (const char* e = getenv("SGN_GATHER_SPEC")) S.gspec = std::min<uint32_t>(64, (uint32_t)atoi(e));
  S.gspec = (uint32_t)std::min<uint64_t>(S.gspec, S.CAP);  // speculative loads stay inside the slab
  size_round_kernels(ctx, S);
  // persistent-round buffers (three, by round % 3): chunk minima + keep minima, counters
  S.rb_min = (decltype(S.rb_min))dalloc<uint64_t>(ctx, 3 * RB_CH * RB_MS_MAX + 4);
  S.rb_keep = S.rb_min + 3 * RB_CH * RB_MS_MAX;
  S.rb_cnt = (decltype(S.rb_cnt))dalloc<uint32_t>(ctx, 3 * RB_CB_MAX + 1);
  S.rb_occ = (decltype(S.rb_occ))dalloc<uint64_t>(ctx, 3 * RB_CH * RB_OS_MAX + 6);
  if (!S.rb_min || !S.rb_cnt || !S.rb_occ) return set_error(ctx, SGN_ENOMEM, "device allocation failed");
  S.fin_cnt = (decltype(S.fin_cnt))dalloc<uint32_t>(ctx, (G + 63) / 64 + 1);
  S.fin_occ = (decltype(S.fin_occ))dalloc<uint64_t>(ctx, (G + 63) / 64);
  if (!S.fin_occ) return set_error(ctx, SGN_ENOMEM, "device allocation failed");
  // the calendar's spill area: runs whose slab is full until the next re-layout (a round edge
  // holds right after a spill); sized for an eighth of the slabs, at least 2^16 runs
  S.spill_cap = std::max<uint64_t>(1u << 16, std::min<uint64_t>(1u << 24, (NB + 1) * G * CAP / 8));
  S.spill = (decltype(S.spill))dev_alloc(ctx, S.spill_cap * sizeof(EvRec), false);
  S.spill_idx = (decltype(S.spill_idx))dev_alloc(ctx, S.spill_cap * 4, false);
  if (!S.spill || !S.spill_idx) return set_error(ctx, SGN_ENOMEM, "device allocation failed (spill area)");
  {
    std::vector<uint64_t> inv((G + 63) / 64, INVALID);
    if ((rc = up64(inv, &S.fin_keep)) || (rc = up64(inv, &S.fin_next))) return rc;
  }
  if (!S.fin_cnt) return set_error(ctx, SGN_ENOMEM, "device allocation failed");
  ctx->d_S = dalloc<DevSim>(ctx, 1);
  if (!ctx->d_S) return set_error(ctx, SGN_ENOMEM, "device allocation failed");
  SGN_HIP(ctx, hipMemcpy(ctx->d_S, &S, sizeof(S), hipMemcpyHostToDevice));
  SGN_HIP(ctx, hipDeviceSynchronize());
  ctx->S = S;
  ctx->sim_ready = true;
  ctx->rounds_enqueued = 0;
  for (int i = 0; i < K_NUM; i++) ctx->kt[i] = {kKernelNames[i], 0, 0.0, 0};
  return 0;
}

int sgn_window(sgn_ctx* ctx, uint64_t* start, uint64_t* end, int32_t* active) {
  if (!ctx || !ctx->sim_ready) return ctx ? set_error(ctx, SGN_ESTATE, "no simulation") : SGN_EINVAL;
  int rc = sync_ctrl(ctx);
  if (start) *start = ctx->h_ctrl->ws;
  if (end) *end = ctx->h_ctrl->we;
  if (active) *active = (int32_t)ctx->h_ctrl->active;
  return rc;
}

int sgn_round(sgn_ctx* ctx, uint64_t* min_next) {
  if (ctx) ctx->ctrl_fresh = false;  // (it may change the device control block)
  if (!ctx || !ctx->sim_ready) return ctx ? set_error(ctx, SGN_ESTATE, "no simulation") : SGN_EINVAL;
  if (int e = rng_release(ctx)) return e;
  if (ctx->comm_local)
    return set_error(ctx, SGN_ESTATE, "a local shard group runs with sgn_run_local_group, not sgn_round");
  int rc = sync_ctrl(ctx);
  if (rc) return rc;
  if (!ctx->h_ctrl->active) return set_error(ctx, SGN_ESTATE, "simulation already finished");
  if (ctx->h_ctrl->hold && (rc = resolve_hold(ctx))) return rc;  // (an earlier growth failed)
  if ((rc = launch_round(ctx))) return rc;
  rc = sync_ctrl(ctx);
  if (!rc && ctx->h_ctrl->xspill) rc = comm_complete_spill(ctx);
  if (!rc) rc = resolve_hold(ctx);
  if (min_next) *min_next = ctx->h_ctrl->last_min_next;
  return rc;
}

int sgn_run(sgn_ctx* ctx, uint64_t max_rounds, uint64_t* rounds_done) {
  if (!ctx || !ctx->sim_ready) return ctx ? set_error(ctx, SGN_ESTATE, "no simulation") : SGN_EINVAL;
  if (int e = rng_release(ctx)) return e;
  if (ctx->comm_local)
    return set_error(ctx, SGN_ESTATE, "a local shard group runs with sgn_run_local_group, not sgn_run");
  // (the control block as the last sgn_run left it, unless a call since may have changed it)
  int rc = ctx->ctrl_fresh ? 0 : sync_ctrl(ctx);
  ctx->ctrl_fresh = false;
  if (rc) return rc;
  // a round still held (an earlier pool growth failed and the caller runs again): grow first
  if ((ctx->h_ctrl->hold || ctx->h_ctrl->spill_n) && (rc = resolve_hold(ctx))) return rc;
  const uint64_t r_start = ctx->h_ctrl->rounds;
  uint64_t enq = 0;
  // Rounds are enqueued in batches with one host synchronisation per batch (the window
  // lives on the device; kernels of rounds past the end return at once). On a single
  // shard a full batch is one hipGraph replay: the round's launches are captured once.
  const uint64_t batch = 32;
  // SGN_GRAPH=1: a full batch is captured once as a hipGraph and replayed (multi-shard over
  // RCCL too: each round's k_execute, the grouped send/recv — RCCL records its kernels in the
  // graph — and k_import). Off by default: measured on config C with per-round launches,
  // replays are no faster than eager launches (38.9 vs 38.9 us per round untimed), and the
  // event-record nodes that time a sample of the rounds slow the replay (1.35 vs 1.47 G
  // packet events/s); the host enqueues eager rounds faster than the GPU runs them.
  const bool graph = ctx->use_graph && (ctx->nranks == 1 || ctx->comm) &&
                     getenv("SGN_GRAPH") && atoi(getenv("SGN_GRAPH")) == 1;
  if (ctx->nranks == 1 && ctx->persist_grid) {
    bool fresh = true;
    // persistent rounds: one launch runs up to kPersistRounds rounds (grid barriers inside);
    // a launch ends early at a held round edge (a pool grows here, then the rounds go on)
    while (ctx->h_ctrl->active && enq < max_rounds && ctx->persist_grid) {
      const uint32_t n = (uint32_t)std::min<uint64_t>(kPersistRounds, max_rounds - enq);
      // (no per-launch memsets: the launch resets its round buffers before its census)
      time_begin(ctx, K_EXECUTE);
      launch_k_rounds(ctx, n);
      time_end(ctx);
      ctx->kt[K_EXECUTE].total++;
      SGN_HIP(ctx, hipGetLastError());
      if ((rc = sync_ctrl_persist(ctx, ctx->res_epoch))) return rc;
      if (census_verdict(ctx, ctx->res_epoch) != 1) {
        // the grid was not resident (the occupancy model was wrong, or another context holds
        // part of the GPU): nothing ran; continue with one launch per round
        ctx->persist_grid = 0;
        ctx->persist_fallbacks++;
        ctx->persist_off = true;
        break;
      }
      if (ctx->h_ctrl->hold || ctx->h_ctrl->spill_n) fresh = false;  // (the host grows a pool)
      if ((rc = resolve_hold(ctx))) return rc;
      enq = ctx->h_ctrl->rounds - r_start;
    }
    if (!ctx->persist_grid) {
      uint64_t more = 0;
      rc = sgn_run(ctx, max_rounds - enq, &more);
      if (rounds_done) *rounds_done = ctx->h_ctrl->rounds - r_start;
      return rc;
    }
    if (rounds_done) *rounds_done = ctx->h_ctrl->rounds - r_start;
    ctx->ctrl_fresh = fresh;
    return 0;
  }
  // multi-shard, one shard per GPU: persistent rounds with the peers' inboxes mapped into this
  // process (k_rounds_x; mapped at the first run, a collective over RCCL), unless refused — then
  // per-round launches with the RCCL send/recv for the rest
  if (ctx->nranks > 1 && ctx->comm && xpersist_possible(ctx)) {
    if (!ctx->x_mapped && (rc = comm_xpeer_map(ctx))) return rc;
    if (ctx->x_mapped) {
      uint64_t k = 0;
      if ((rc = run_xpersist({ctx}, true, max_rounds, &k))) return rc;
      if (!ctx->x_off || k >= max_rounds || !ctx->h_ctrl->active) {
        if (rounds_done) *rounds_done = ctx->h_ctrl->rounds - r_start;
        return 0;
      }
    }
  }
  // rounds are counted as they complete: a multi-shard round held for a full-slot exchange
  // (comm_complete_spill) turns the rest of its batch into no-ops, which are not rounds
  uint64_t done = ctx->h_ctrl->rounds - r_start;
  static const bool dbg = getenv("SGN_DEBUG_RUN") != nullptr;
  while (ctx->h_ctrl->active && done < max_rounds) {
    const uint64_t n = std::min<uint64_t>(batch, max_rounds - done);
    if (dbg)
      fprintf(stderr, "[sgn r%u] batch n=%llu done=%llu graph=%d gexec=%d gsz=%u xsz=%u spills=%llu\n", ctx->rank,
              (unsigned long long)n, (unsigned long long)done, (int)graph, ctx->gexec != nullptr, ctx->gsz,
              ctx->xsz_cur, (unsigned long long)ctx->x_spills);
    if (graph && n == batch) {
      if (ctx->gexec && ctx->gsz != ctx->xsz_cur) drop_graph(ctx);  // the send size changed
      if (!ctx->gexec) {
        ctx->ev_pending.clear();
        ctx->ev_next = 0;
        ctx->capturing = true;
        hipError_t e = hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal);
        for (uint64_t i = 0; i < n && rc == 0 && e == hipSuccess; i++) rc = launch_round(ctx);
        hipGraph_t g = nullptr;
        hipError_t e2 = hipStreamEndCapture(ctx->stream, &g);
        ctx->capturing = false;
        if (rc) return rc;
        if (e != hipSuccess) return hip_fail(ctx, e, "hipStreamBeginCapture");
        if (e2 != hipSuccess) return hip_fail(ctx, e2, "hipStreamEndCapture");
        ctx->graph = g;
        if ((rc = add_timing_nodes(ctx, g))) return rc;
        SGN_HIP(ctx, hipGraphInstantiate(&ctx->gexec, g, nullptr, nullptr, 0));
        ctx->gbatch = batch;
        ctx->gsz = ctx->xsz_cur;
      }
      SGN_HIP(ctx, hipGraphLaunch(ctx->gexec, ctx->stream));
      ctx->kt[K_EXECUTE].total += n;
      if (ctx->nranks > 1) ctx->kt[K_IMPORT].total += n;
      ctx->graph_pending = !ctx->graph_timed.empty();
      ctx->x_bytes += n * comm_round_bytes(ctx);
    } else {
      for (uint64_t i = 0; i < n; i++)
        if ((rc = launch_round(ctx))) return rc;
    }
    if ((rc = sync_ctrl(ctx))) return rc;
    if (dbg)
      fprintf(stderr, "[sgn r%u] synced rounds=%llu spill=%u hwm=%llu\n", ctx->rank,
              (unsigned long long)(ctx->h_ctrl->rounds - r_start), ctx->h_ctrl->xspill,
              (unsigned long long)ctx->h_ctrl->xhwm);
    if (ctx->h_ctrl->xspill && (rc = comm_complete_spill(ctx))) return rc;
    if ((rc = resolve_hold(ctx))) return rc;
    if (dbg && ctx->h_ctrl->xspill == 0) fprintf(stderr, "[sgn r%u] after: rounds=%llu\n", ctx->rank,
                                                 (unsigned long long)(ctx->h_ctrl->rounds - r_start));
    done = ctx->h_ctrl->rounds - r_start;
  }
  if (rounds_done) *rounds_done = ctx->h_ctrl->rounds - r_start;
  return 0;
}

namespace {
// the records of owned hosts [off, off + n) (device -> host)
int read_recs(sgn_ctx* ctx, uint32_t off, uint32_t n, std::vector<HostRec>* out) {
  out->resize(n);
  if (n) SGN_HIP(ctx, hipMemcpy(out->data(), (const void*)(ctx->S.hrec + off), (size_t)n * sizeof(HostRec),
                                hipMemcpyDeviceToHost));
  if (n && ctx->S.htile) {  // the hot lines from their tiles
    const uint32_t t0 = off >> 6, t1 = (off + n + 63) >> 6;
    std::vector<uint64_t> tile((size_t)(t1 - t0) * 8 * 64 * 2);
    SGN_HIP(ctx, hipMemcpy(tile.data(), (const void*)(ctx->S.htile + (size_t)t0 * 8 * 64 * 2), tile.size() * 8,
                           hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; i++)
      for (uint32_t c = 0; c < 8; c++)
        std::memcpy((char*)&(*out)[i] + 16 * c, &tile[2 * (hot_idx(off + i, c) - (size_t)t0 * 8 * 64)], 16);
  }
  return 0;
}
// the per-host totals of owned slots [off, off + n): N_CNT rows, then the CoDel maxima
int read_counts(sgn_ctx* ctx, uint32_t off, uint32_t n, std::vector<uint64_t>* cnt, std::vector<uint32_t>* mq) {
  const size_t nH = ctx->S.nH;
  cnt->assign((size_t)N_CNT * n, 0);
  if (mq) mq->assign(n, 0);
  if (!n) return 0;
  if (ctx->S.tkind != SGN_TRAFFIC_PERIODIC) {  // (these kinds keep them in the cold lines)
    std::vector<HostRec> recs;
    if (int e = read_recs(ctx, off, n, &recs)) return e;
    for (uint32_t i = 0; i < n; i++) {
      (*cnt)[(size_t)N_SENT * n + i] = recs[i].n_sent;
      (*cnt)[(size_t)N_POPPED * n + i] = recs[i].n_popped;
      (*cnt)[(size_t)N_DELIVERED * n + i] = recs[i].n_delivered;
      if (mq) (*mq)[i] = recs[i].max_codel;
    }
    return 0;
  }
  for (int k = 0; k < N_CNT; k++)
    SGN_HIP(ctx, hipMemcpy(cnt->data() + (size_t)k * n, (const void*)(ctx->S.n_cnt + k * nH + off), (size_t)n * 8,
                           hipMemcpyDeviceToHost));
  if (mq) SGN_HIP(ctx, hipMemcpy(mq->data(), (const void*)(ctx->S.maxq + off), (size_t)n * 4, hipMemcpyDeviceToHost));
  return 0;
}
// the cold lines hold the host's queue state (else it is an idle host's: empty queues)
inline bool cold_valid(const sgn_ctx* ctx, const HostRec& r) {
  return ctx->S.tkind != SGN_TRAFFIC_PERIODIC || (r.flags & F_COLD);
}
}  // namespace

int sgn_stats_get(sgn_ctx* ctx, sgn_stats* out) {
  if (!ctx || !out) return SGN_EINVAL;
  if (!ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "no simulation");
  int rc = sync_ctrl(ctx);
  const uint32_t nH = ctx->S.nH;
  std::vector<HostRec> recs;
  std::vector<uint64_t> cnt;
  std::vector<uint32_t> mq;
  if (int e = read_recs(ctx, 0, nH, &recs)) return e;
  if (int e = read_counts(ctx, 0, nH, &cnt, &mq)) return e;
  sgn_stats s{};
  uint64_t mc = 0;
  for (uint32_t h = 0; h < nH; h++) {
    const HostRec& r = recs[h];
    s.packets_sent += cnt[(size_t)N_SENT * nH + h];
    s.packets_unknown_dst += r.n_unknown;
    s.packet_events_popped += cnt[(size_t)N_POPPED * nH + h];
    s.codel_dropped += r.n_codel;
    s.delivered += cnt[(size_t)N_DELIVERED * nH + h];
    s.local_delivered += r.n_local_deliv;
    s.app_blocked += r.n_blocked;
    mc = std::max<uint64_t>(mc, mq[h]);
  }
  s.rounds = ctx->h_ctrl->rounds;
  s.min_used_latency_ns = ctx->h_ctrl->min_used;
  s.max_codel_len = mc;

  {
    const size_t G = ctx->S.G;
    std::vector<uint64_t> wc(W_N * G);
    SGN_HIP(ctx, hipMemcpy(wc.data(), (const void*)ctx->S.w_cnt, wc.size() * 8, hipMemcpyDeviceToHost));
    uint64_t acc[W_N] = {};
    for (int k = 0; k < W_N; k++)
      for (size_t g = 0; g < G; g++)
        acc[k] = k == W_MAXFILL ? std::max(acc[k], wc[k * G + g]) : acc[k] + wc[k * G + g];
    s.max_pending_events = acc[W_MAXFILL];
    s.host_executions = acc[W_EXEC];
    s.event_runs = acc[W_RUNS];
    s.sched_sorted_segments = acc[W_SORTED];
    s.packets_loss_dropped = acc[W_LOSS];
    s.local_events = acc[W_LOCAL_EV];
    s.bytes_delivered = acc[W_BYTES];
  }
  s.sched_heavy_hosts = 0;
  *out = s;
  return rc;
}

int sgn_host_digests(sgn_ctx* ctx, uint32_t lo, uint32_t hi, sgn_host_digest* out) {
  if (!ctx || !out) return SGN_EINVAL;
  if (!ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "no simulation");
  if (lo < ctx->lo || hi > ctx->hi || lo > hi) return set_error(ctx, SGN_EINVAL, "range outside the owned shard");
  if (int e = rng_release(ctx)) return e;
  int rc = sync_ctrl(ctx);
  const uint32_t n = hi - lo;
  // the range's hosts sit in permuted slots: read the slots they span
  uint32_t smin = ctx->hi, smax = ctx->lo;
  for (uint32_t i = lo; i < hi; i++) {
    smin = std::min(smin, ctx->sid_of[i]);
    smax = std::max(smax, ctx->sid_of[i]);
  }
  std::vector<HostRec> recs;
  std::vector<uint64_t> cnt;
  const uint32_t ns = n ? smax - smin + 1 : 0;
  if (n) {
    if (int e = read_recs(ctx, smin - ctx->lo, ns, &recs)) return e;
    if (int e = read_counts(ctx, smin - ctx->lo, ns, &cnt, nullptr)) return e;
  }
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t j = ctx->sid_of[lo + i] - smin;
    const HostRec& r = recs[j];
    sgn_host_digest& o = out[i];
    o.tx = r.dig[0];
    o.rx = r.dig[1];
    o.app = r.dig[2];
    for (int k = 0; k < 4; k++) o.rng[k] = r.rng[k];
    o.next_event_id = r.eid;
    o.n_sent = cnt[(size_t)N_SENT * ns + j];
    o.n_popped = cnt[(size_t)N_POPPED * ns + j];
    o.n_delivered = cnt[(size_t)N_DELIVERED * ns + j];
    o.n_codel_dropped = r.n_codel;
  }
  return rc;
}

namespace {
// Host::next_event_time for owned HostIds [lo, hi): two small kernels, one copy.
int next_event_times(sgn_ctx* ctx, uint32_t lo, uint32_t hi, uint64_t* out) {
  if (!ctx || (!out && hi > lo)) return SGN_EINVAL;
  if (!ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "no simulation");
  if (lo < ctx->lo || hi > ctx->hi || lo > hi) return set_error(ctx, SGN_EINVAL, "host range not owned by this shard");
  int rc = sync_ctrl(ctx);
  if (rc) return rc;
  const uint32_t n = hi - lo;
  if (n == 0) return 0;
  const DevSim& S = ctx->S;
  SGN_HIP(ctx, hipSetDevice(ctx->device));
  uint64_t* d = nullptr;
  SGN_HIP(ctx, hipMalloc(&d, (size_t)n * 8));
  // the groups holding the range's slots: one host's group, or all of them
  uint32_t g0 = 0, ng = S.G;
  if (n == 1) {
    g0 = (ctx->sid_of[lo] - ctx->lo) >> S.gsh;
    ng = 1;
  }
  hipLaunchKernelGGL(k_next_local, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, (const DevSim*)ctx->d_S, lo, n, d);
  hipLaunchKernelGGL(k_next_packet, dim3(S.NB * ng), dim3(64), 0, ctx->stream, (const DevSim*)ctx->d_S, lo, n, g0,
                     ng, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  hipFree(d);
  if (e != hipSuccess) return hip_fail(ctx, e, "next event times");
  return 0;
}
}  // namespace

int sgn_host_next_event_time(sgn_ctx* ctx, uint32_t host, uint64_t* t) {
  if (!ctx || !t) return SGN_EINVAL;
  return next_event_times(ctx, host, host + 1, t);
}

int sgn_hosts_next_event_time(sgn_ctx* ctx, uint32_t host_lo, uint32_t host_hi, uint64_t* out) {
  return next_event_times(ctx, host_lo, host_hi, out);
}

int sgn_trace_read(sgn_ctx* ctx, sgn_trace_rec* out, uint64_t cap, uint64_t* n_total) {
  if (!ctx) return SGN_EINVAL;
  if (!ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "no simulation");
  int rc = sync_ctrl(ctx);
  const uint64_t n = std::min<uint64_t>(ctx->h_ctrl->trace_n, ctx->S.trace_cap);
  if (n_total) *n_total = ctx->h_ctrl->trace_n;
  const uint64_t k = std::min(n, cap);
  if (k && out) SGN_HIP(ctx, hipMemcpy(out, ctx->S.trace, k * sizeof(sgn_trace_rec), hipMemcpyDeviceToHost));
  return rc;
}

int sgn_engine_info_get(sgn_ctx* ctx, sgn_engine_info* out) {
  if (!ctx || !out) return SGN_EINVAL;
  if (!ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "no simulation");
  const DevSim& S = ctx->S;
  out->calendar_buckets = S.NB;
  out->bucket_width_ns = S.BW;
  out->host_groups = S.G;
  out->slab_capacity = S.CAP;
  out->hosts_per_wave = 1u << S.gsh;
  out->persistent_grid = ctx->persist_grid;
  out->persistent_fallbacks = ctx->persist_fallbacks;
  out->device_bytes = ctx->sim_bytes;
  out->exchange_slot_runs = ctx->nranks > 1 ? ctx->xslot : 0;
  out->exchange_send_runs = ctx->xsz_cur;
  out->exchange_hwm_runs = ctx->h_ctrl ? ctx->h_ctrl->xhwm : 0;
  out->exchange_spills = ctx->x_spills;
  out->exchange_bytes = ctx->x_bytes;
  out->codel_pages = ctx->S.cq_pages;
  // the control block as is (an overflow is reported by the calls that run rounds, not here)
  SGN_HIP(ctx, hipStreamSynchronize(ctx->stream));
  SGN_HIP(ctx, hipMemcpy(ctx->h_ctrl, (const void*)ctx->S.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost));
  const Ctrl& c = *ctx->h_ctrl;
  out->codel_page_allocs = ctx->codel_allocs_before + c.pg_alloc;
  out->codel_pages_free = c.pg_tail >= c.pg_alloc ? c.pg_tail - c.pg_alloc : 0;
  std::vector<HostRec> recs;
  if (int e = read_recs(ctx, 0, ctx->S.nH, &recs)) return e;
  uint64_t chained = 0;
  for (const HostRec& r : recs) {
    const uint32_t nr = cold_valid(ctx, r) ? r.cq_nr : 0;
    chained += nr == 0 ? 1 : ((r.cq_head & (CQ_PAGE - 1)) + nr + CQ_PAGE - 1) / CQ_PAGE;
  }
  out->codel_pages_chained = chained;
  int ncu = 0;
  SGN_HIP(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
  out->compute_units = (uint64_t)ncu;
  out->bucket_min_lds = ctx->S.agg_bmin;
  out->lds_per_cu = ctx->lds_per_cu;
  out->codel_pool_grows = ctx->codel_grows;
  out->calendar_grows = ctx->cal_grows;
  out->calendar_spill_runs = ctx->cal_spill_runs;
  out->exchange_slot_grows = ctx->xslot_grows;
  out->rounds_held = ctx->rounds_held;
  out->slab_extensions = ctx->ext_slabs;
  out->slab_extension_runs = ctx->S.ext_total;
  {
    const size_t G = ctx->S.G;
    std::vector<uint64_t> wb(G);
    SGN_HIP(ctx, hipMemcpy(wb.data(), (const void*)(ctx->S.w_cnt + W_BIG * G), G * 8, hipMemcpyDeviceToHost));
    uint64_t t = 0;
    for (uint64_t v : wb) t += v;
    out->big_slab_pieces = t;
  }
  out->spill_area_runs = ctx->S.spill_cap;
  out->spill_area_grows = ctx->spill_grows;
  out->exchange_mode = ctx->nranks > 1 ? ctx->x_mode : 0;
  out->inbox_slot_runs = ctx->nranks > 1 ? ctx->S.xislot : 0;
  out->inbox_grows = ctx->x_grows;
  out->inbox_overflow_rounds = ctx->x_over_rounds;
  out->inbox_moved_runs = ctx->x_moved;
  out->persistent_x_launches = ctx->x_launches;
  out->persistent_x_grid = ctx->x_grid;
  return 0;
}

int sgn_kernel_times_get(sgn_ctx* ctx, sgn_kernel_times* out) {
  if (!ctx || !out) return SGN_EINVAL;
  if (ctx->sim_ready) {
    int rc = sync_ctrl(ctx);
    if (rc) return rc;
  }
  std::memset(out, 0, sizeof(*out));
  out->n_kernels = K_NUM;
  for (int i = 0; i < K_NUM; i++) {
    out->launches[i] = ctx->kt[i].launches;
    out->launches_total[i] = ctx->kt[i].total;
    out->ms[i] = ctx->kt[i].ms;
    out->name[i] = kKernelNames[i];
  }
  // the round kernel's slot: persistent launches (many rounds each) when enabled
  if (ctx->persist_grid) out->name[K_EXECUTE] = "k_rounds";
  if (ctx->x_mode == 2) out->name[K_EXECUTE] = "k_rounds_x";
  return 0;
}

// Diagnostics: per-wave {cycles, events, max lane events, busy lanes} of the last k_execute
// (allocated when SGN_STAMPS=1 is set in the environment at sgn_sim_init).
// Diagnostics of the last persistent launch (SGN_STAMPS=2): per round {earliest start, latest
// arrival, round edge done} (100 MHz clock), 128 rounds; resets the buffer for the next launch.
int sgn_debug_rounds(sgn_ctx* ctx, uint64_t* out) {
  if (!ctx || !ctx->sim_ready || !ctx->S.rdbg) return SGN_EINVAL;
  SGN_HIP(ctx, hipStreamSynchronize(ctx->stream));
  SGN_HIP(ctx, hipMemcpy(out, (const void*)ctx->S.rdbg, 3 * 128 * 8, hipMemcpyDeviceToHost));
  std::vector<uint64_t> init(3 * 128, 0);
  for (int r = 0; r < 128; r++) init[3 * r] = ~0ULL;
  SGN_HIP(ctx, hipMemcpy((void*)ctx->S.rdbg, init.data(), init.size() * 8, hipMemcpyHostToDevice));
  return 0;
}

// The same for k_rounds_x: per round 8 words (see the kernel's stamps), 128 rounds; resets.
int sgn_debug_rounds_x(sgn_ctx* ctx, uint64_t* out) {
  if (!ctx || !ctx->sim_ready || !ctx->S.rdbg) return SGN_EINVAL;
  SGN_HIP(ctx, hipDeviceSynchronize());
  SGN_HIP(ctx, hipMemcpy(out, (const void*)ctx->S.rdbg, 8 * 128 * 8, hipMemcpyDeviceToHost));
  std::vector<uint64_t> init(8 * 128, 0);
  for (int r = 0; r < 128; r++) init[8 * r] = ~0ULL;
  SGN_HIP(ctx, hipMemcpy((void*)ctx->S.rdbg, init.data(), init.size() * 8, hipMemcpyHostToDevice));
  return 0;
}

// k_rounds_x with SGN_STAMPS=3: every workgroup's stamps, [128 rounds][2048 workgroups][8]
// (this shard's workgroup index; unwritten: 0); resets.
int sgn_debug_rounds_xw(sgn_ctx* ctx, uint64_t* out) {
  if (!ctx || !ctx->sim_ready || !ctx->S.rdbg || !ctx->S.rdbg_wg) return SGN_EINVAL;
  const size_t n = (size_t)8 * 128 * 2048;
  SGN_HIP(ctx, hipDeviceSynchronize());
  SGN_HIP(ctx, hipMemcpy(out, (const void*)ctx->S.rdbg, n * 8, hipMemcpyDeviceToHost));
  SGN_HIP(ctx, hipMemset((void*)ctx->S.rdbg, 0, n * 8));
  return 0;
}

int sgn_debug_stamps(sgn_ctx* ctx, uint64_t* out, uint64_t cap, uint64_t* n) {
  if (!ctx || !ctx->sim_ready) return SGN_EINVAL;
  const uint64_t waves = ctx->S.G;
  if (n) *n = ctx->S.stamps ? waves : 0;
  if (!ctx->S.stamps || !out) return 0;
  SGN_HIP(ctx, hipStreamSynchronize(ctx->stream));
  SGN_HIP(ctx, hipMemcpy(out, ctx->S.stamps, std::min(cap, waves) * SGN_STAMP_WORDS * 8, hipMemcpyDeviceToHost));
  return 0;
}

// ---- CPU-resident applications (SGN_TRAFFIC_EXTERNAL) ----
int sgn_drain_enable(sgn_ctx* ctx, uint64_t capacity) {
  if (!ctx) return SGN_EINVAL;
  if (ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "sgn_drain_enable must precede sgn_sim_init");
  if (capacity == 0) return set_error(ctx, SGN_EINVAL, "drain capacity must be >= 1");
  ctx->drain_cap = capacity;
  return 0;
}

int sgn_submit(sgn_ctx* ctx, const sgn_pkt_soa* b) {
  if (ctx) ctx->ctrl_fresh = false;  // (it may change the device control block)
  if (!ctx || !b) return SGN_EINVAL;
  if (!ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "no simulation");
  const DevSim& S = ctx->S;
  if (S.tkind != SGN_TRAFFIC_EXTERNAL)
    return set_error(ctx, SGN_ESTATE, "sgn_submit needs SGN_TRAFFIC_EXTERNAL traffic");
  if (b->n == 0) return 0;
  if (!b->src_host || !b->dst_ip || !b->payload_len || !b->send_time)
    return set_error(ctx, SGN_EINVAL, "sgn_submit: missing array");
  int rc = sync_ctrl(ctx);
  if (rc) return rc;
  const uint64_t ws = ctx->h_ctrl->ws;
  // the calendar holds NB buckets of BW ns; the gather walks forward from the window
  const uint64_t horizon = ws + (uint64_t)(S.NB - 2) * S.BW;
  if (ctx->handles.size() + b->n > SGN_TAG_SLOT_MASK)
    return set_error(ctx, SGN_ERANGE, "more than 2^29 submissions on one shard");
  std::vector<EvRec> recs(b->n);
  std::vector<uint32_t> seq_add;
  std::vector<uint32_t> seq = ctx->submit_seq;  // committed only on success
  for (uint64_t i = 0; i < b->n; i++) {
    const uint32_t src = b->src_host[i];
    const uint64_t t = b->send_time[i];
    const uint32_t pay = b->payload_len[i];
    if (src < ctx->lo || src >= ctx->hi)
      return set_error(ctx, SGN_EINVAL, "sgn_submit: source host " + std::to_string(src) + " not owned by this shard");
    if (t < ws || t >= S.end_time)
      return set_error(ctx, SGN_EINVAL, "sgn_submit: send_time outside [window start, stop time)");
    if (t >= horizon)
      return set_error(ctx, SGN_EINVAL, "sgn_submit: send_time beyond the event calendar's horizon; submit it closer to its window");
    if (pay > 0xFFFFu) return set_error(ctx, SGN_EINVAL, "sgn_submit: payload_len > 65535");
    uint32_t hdr = 0;
    if (b->wire_len && b->wire_len[i] != 0) {
      const uint32_t w = b->wire_len[i];
      if (w == pay + SGN_UDP_HEADER_BYTES) hdr = 0;
      else if (w == pay + SGN_TCP_HEADER_BYTES) hdr = SGN_TAG_HDR_TCP;
      else if (w == pay + SGN_TCP_WS_HEADER_BYTES) hdr = SGN_TAG_HDR_TCPWS;
      else
        return set_error(ctx, SGN_EINVAL,
                         "sgn_submit: wire_len must be payload_len + 28 (UDP/IPv4), + 40 or + 44 (TCP/IPv4)");
    }
    uint32_t& q = seq[src - ctx->lo];
    if (q == 0xFFFFFFFFu) return set_error(ctx, SGN_ERANGE, "sgn_submit: 2^32 submissions from one host");
    EvRec& r = recs[i];
    r.time = t;
    r.eid = ((uint64_t)q++ << 32) | b->dst_ip[i];  // submission order, then the address
    r.src = src;
    r.dst = ctx->sid_of[src];  // filed in the source's own slot
    r.pc = pay | (1u << 16);
    r.tag = SGN_TAG_EXT | hdr | (uint32_t)(ctx->handles.size() + i);
  }
  SGN_HIP(ctx, hipSetDevice(ctx->device));
  if (ctx->stage_cap < b->n) {
    if (ctx->d_stage) hipFree(ctx->d_stage);
    ctx->d_stage = nullptr;
    ctx->stage_cap = 0;
    SGN_HIP(ctx, hipMalloc(&ctx->d_stage, b->n * sizeof(EvRec)));
    ctx->stage_cap = b->n;
  }
  SGN_HIP(ctx, hipMemcpyAsync(ctx->d_stage, recs.data(), b->n * sizeof(EvRec), hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_inject, dim3((uint32_t)((b->n + 255) / 256)), dim3(256), 0, ctx->stream,
                     (const DevSim*)ctx->d_S, (const EvRec*)ctx->d_stage, (uint32_t)b->n);
  SGN_HIP(ctx, hipGetLastError());
  // the runs are in the device calendar from here: a failure past this point leaves them there
  // with no handle, so the context is marked unusable (a retry would file them twice)
  rc = sync_ctrl(ctx);
  if (!rc && ctx->h_ctrl->spill_n) rc = relayout_calendar(ctx);
  if (rc) {
    ctx->failed = std::string("sgn_submit failed after filing its runs: ") + sgn_last_error(ctx);
    return rc;
  }
  for (uint64_t i = 0; i < b->n; i++) ctx->handles.push_back(b->handle ? b->handle[i] : 0);
  ctx->submit_seq.swap(seq);
  return 0;
}

// ---- per-thread staging: stages are plain host buffers; one flush submits all
int sgn_stage_create(sgn_ctx* ctx, sgn_stage** out) {
  if (!ctx || !out) return SGN_EINVAL;
  sgn_stage* st = new sgn_stage();
  st->ctx = ctx;
  std::lock_guard<std::mutex> g(ctx->stage_mu);
  ctx->stages.push_back(st);
  *out = st;
  return 0;
}

void sgn_stage_destroy(sgn_stage* st) {
  if (!st) return;
  if (st->ctx) {
    std::lock_guard<std::mutex> g(st->ctx->stage_mu);
    auto& v = st->ctx->stages;
    v.erase(std::remove(v.begin(), v.end(), st), v.end());
  }
  delete st;
}

int sgn_stage_push(sgn_stage* st, const sgn_pkt_soa* b) {
  if (!st || !b) return SGN_EINVAL;
  if (b->n == 0) return 0;
  if (!b->src_host || !b->dst_ip || !b->payload_len || !b->send_time) return SGN_EINVAL;
  for (uint64_t i = 0; i < b->n; i++) {
    if (b->payload_len[i] > 0xFFFFu) return SGN_EINVAL;
    if (b->wire_len && b->wire_len[i] != 0) {
      const uint32_t w = b->wire_len[i], p = b->payload_len[i];
      if (w != p + SGN_UDP_HEADER_BYTES && w != p + SGN_TCP_HEADER_BYTES && w != p + SGN_TCP_WS_HEADER_BYTES)
        return SGN_EINVAL;
    }
  }
  std::lock_guard<std::mutex> g(st->mu);  // (uncontended except against a concurrent flush)
  st->src.insert(st->src.end(), b->src_host, b->src_host + b->n);
  st->dst.insert(st->dst.end(), b->dst_ip, b->dst_ip + b->n);
  st->pay.insert(st->pay.end(), b->payload_len, b->payload_len + b->n);
  st->time.insert(st->time.end(), b->send_time, b->send_time + b->n);
  for (uint64_t i = 0; i < b->n; i++) st->handle.push_back(b->handle ? b->handle[i] : 0);
  for (uint64_t i = 0; i < b->n; i++) st->wire.push_back(b->wire_len ? b->wire_len[i] : 0);
  return 0;
}

uint64_t sgn_stage_pending(const sgn_stage* st) {
  if (!st) return 0;
  std::lock_guard<std::mutex> g(st->mu);
  return st->src.size();
}

int sgn_stage_flush(sgn_ctx* ctx) {
  if (ctx) ctx->ctrl_fresh = false;  // (it may change the device control block)
  if (!ctx) return SGN_EINVAL;
  std::vector<uint32_t> src, dst, pay, wire;
  std::vector<uint64_t> time, handle;
  // each stage's size at copy time: only that prefix is cleared after the submit, so a push
  // that lands while the flush runs stays staged for the next flush
  std::vector<std::pair<sgn_stage*, size_t>> taken;
  {
    std::lock_guard<std::mutex> g(ctx->stage_mu);
    for (sgn_stage* st : ctx->stages) {
      std::lock_guard<std::mutex> sg(st->mu);
      taken.push_back({st, st->src.size()});
      wire.insert(wire.end(), st->wire.begin(), st->wire.end());
      src.insert(src.end(), st->src.begin(), st->src.end());
      dst.insert(dst.end(), st->dst.begin(), st->dst.end());
      pay.insert(pay.end(), st->pay.begin(), st->pay.end());
      time.insert(time.end(), st->time.begin(), st->time.end());
      handle.insert(handle.end(), st->handle.begin(), st->handle.end());
    }
  }
  if (src.empty()) return 0;
  sgn_pkt_soa b{src.size(), src.data(), dst.data(), pay.data(), wire.data(), time.data(), handle.data()};
  if (int rc = sgn_submit(ctx, &b)) return rc;
  std::lock_guard<std::mutex> g(ctx->stage_mu);
  for (auto& t : taken) {
    sgn_stage* st = t.first;
    if (std::find(ctx->stages.begin(), ctx->stages.end(), st) == ctx->stages.end()) continue;  // destroyed meanwhile
    std::lock_guard<std::mutex> sg(st->mu);
    const size_t k = t.second;
    st->src.erase(st->src.begin(), st->src.begin() + k);
    st->dst.erase(st->dst.begin(), st->dst.begin() + k);
    st->pay.erase(st->pay.begin(), st->pay.begin() + k);
    st->time.erase(st->time.begin(), st->time.begin() + k);
    st->handle.erase(st->handle.begin(), st->handle.begin() + k);
    st->wire.erase(st->wire.begin(), st->wire.begin() + k);
  }
  return 0;
}

int sgn_drain(sgn_ctx* ctx, uint32_t lo, uint32_t hi, sgn_drain_rec* out, uint64_t cap, uint64_t* n_out) {
  if (ctx) ctx->ctrl_fresh = false;  // (it may change the device control block)
  if (!ctx || (!out && cap)) return SGN_EINVAL;
  if (!ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "no simulation");
  if (ctx->S.tkind != SGN_TRAFFIC_EXTERNAL)
    return set_error(ctx, SGN_ESTATE, "sgn_drain needs SGN_TRAFFIC_EXTERNAL traffic");
  int rc = sync_ctrl(ctx);
  if (rc) return rc;
  const uint64_t n = ctx->h_ctrl->drain_n;
  if (n) {
    const size_t old = ctx->drain_held.size();
    ctx->drain_held.resize(old + n);
    SGN_HIP(ctx, hipMemcpy(ctx->drain_held.data() + old, (const void*)ctx->S.drain, n * sizeof(sgn_drain_rec),
                           hipMemcpyDeviceToHost));
    const uint64_t zero = 0;
    SGN_HIP(ctx, hipMemcpy((char*)ctx->S.ctrl + offsetof(Ctrl, drain_n), &zero, 8, hipMemcpyHostToDevice));
    ctx->h_ctrl->drain_n = 0;
    for (size_t i = old; i < ctx->drain_held.size(); i++) {
      sgn_drain_rec& r = ctx->drain_held[i];
      const uint32_t slot = r.tag & SGN_TAG_SLOT_MASK;
      // a slot is this shard's when the datagram's source is one of its hosts
      r.handle = ((r.tag & SGN_TAG_EXT) && r.src_host >= ctx->lo && r.src_host < ctx->hi &&
                  slot < ctx->handles.size()) ? ctx->handles[slot] : 0;
    }
  }
  std::vector<sgn_drain_rec> sel, keep;
  for (const sgn_drain_rec& r : ctx->drain_held) (r.host >= lo && r.host < hi ? sel : keep).push_back(r);
  auto key = [](const sgn_drain_rec& r) {
    return std::make_tuple(r.host, r.time, r.src_host, r.src_eid, r.tag, r.status);
  };
  std::sort(sel.begin(), sel.end(), [&](const sgn_drain_rec& a, const sgn_drain_rec& b) { return key(a) < key(b); });
  const uint64_t k = std::min<uint64_t>(cap, sel.size());
  if (k) std::memcpy(out, sel.data(), k * sizeof(sgn_drain_rec));
  keep.insert(keep.end(), sel.begin() + k, sel.end());
  ctx->drain_held.swap(keep);
  if (n_out) *n_out = k;
  return 0;
}

int sgn_set_window(sgn_ctx* ctx, uint64_t start, uint64_t end) {
  if (ctx) ctx->ctrl_fresh = false;  // (it may change the device control block)
  if (!ctx) return SGN_EINVAL;
  if (!ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "no simulation");
  int rc = sync_ctrl(ctx);
  if (rc) return rc;
  Ctrl& c = *ctx->h_ctrl;
  if (start < c.prev_we) return set_error(ctx, SGN_EINVAL, "sgn_set_window: start before the previous window's end");
  if (start > c.ws) return set_error(ctx, SGN_EINVAL, "sgn_set_window: start after the device's next event time");
  if (end <= start) return set_error(ctx, SGN_EINVAL, "sgn_set_window: empty window");
  if (end - start > ctx->S.BW)
    return set_error(ctx, SGN_EINVAL, "sgn_set_window: window longer than the runahead the calendar was sized for");
  end = std::min(end, ctx->S.end_time);
  if (end <= start) return set_error(ctx, SGN_EINVAL, "sgn_set_window: window at or past the stop time");
  c.ws = start;
  c.we = end;
  c.active = 1;
  SGN_HIP(ctx, hipMemcpy((void*)ctx->S.ctrl, &c, offsetof(Ctrl, overflow), hipMemcpyHostToDevice));
  // the CoDel guard for the window as set (the last round edge evaluated the one it computed)
  const uint64_t need = codel_need_host(ctx), have = c.pg_avail > c.pg_alloc ? c.pg_avail - c.pg_alloc : 0;
  if (have < need) return grow_codel(ctx, need - have);
  return 0;
}


namespace {
// rand_xoshiro 0.7.0 Xoshiro256PlusPlus::next_u64 on the CPU (a CPU-held host state)
inline uint64_t host_xoshiro_next(uint64_t* s) {
  auto rotl = [](uint64_t x, int k) { return (x << k) | (x >> (64 - k)); };
  const uint64_t r = rotl(s[0] + s[3], 23) + s[0], t = s[1] << 17;
  s[2] ^= s[0];
  s[3] ^= s[1];
  s[1] ^= s[2];
  s[0] ^= s[3];
  s[2] ^= t;
  s[3] = rotl(s[3], 45);
  return r;
}
// n single draws of one owned host on the CPU: the first draw after a device operation reads
// the state (one 32-byte copy); later ones are a few nanoseconds each
int rng_cpu_draws(sgn_ctx* ctx, uint32_t host, uint64_t n, uint64_t* out) {
  if (!ctx) return SGN_EINVAL;
  if (!ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "no simulation");
  if (host < ctx->lo || host >= ctx->hi) return set_error(ctx, SGN_EINVAL, "host not owned by this shard");
  const uint32_t slot = ctx->sid_of[host] - ctx->lo;
  auto it = ctx->rng_held.find(slot);
  if (it == ctx->rng_held.end()) {
    sgn_ctx::RngHeld h{};
    SGN_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->S.htile) {
      SGN_HIP(ctx, hipMemcpy(h.s, (const void*)(ctx->S.htile + 2 * hot_idx(slot, 0)), 16, hipMemcpyDeviceToHost));
      SGN_HIP(ctx, hipMemcpy(h.s + 2, (const void*)(ctx->S.htile + 2 * hot_idx(slot, 1)), 16, hipMemcpyDeviceToHost));
    } else {
      SGN_HIP(ctx, hipMemcpy(h.s, (const void*)(ctx->S.hrec + slot), 32, hipMemcpyDeviceToHost));
    }
    it = ctx->rng_held.emplace(slot, h).first;
  }
  for (uint64_t i = 0; i < n; i++) out[i] = host_xoshiro_next(it->second.s);
  it->second.draws += n;
  return 0;
}
// counts[i] draws from each of n distinct owned hosts, concatenated in order into out
int rng_draws(sgn_ctx* ctx, const uint32_t* hosts, const uint32_t* counts, uint32_t n, uint64_t* out) {
  if (!ctx || (n && (!hosts || !counts))) return SGN_EINVAL;
  if (!ctx->sim_ready) return set_error(ctx, SGN_ESTATE, "no simulation");
  std::vector<uint32_t> loc(n);
  std::vector<uint64_t> off(n);
  uint64_t total = 0;
  std::vector<uint32_t> seen;
  for (uint32_t i = 0; i < n; i++) {
    if (hosts[i] < ctx->lo || hosts[i] >= ctx->hi) return set_error(ctx, SGN_EINVAL, "host not owned by this shard");
    loc[i] = ctx->sid_of[hosts[i]] - ctx->lo;  // the host's slot
    off[i] = total;
    total += counts[i];
    seen.push_back(hosts[i]);
  }
  std::sort(seen.begin(), seen.end());
  if (std::adjacent_find(seen.begin(), seen.end()) != seen.end())
    return set_error(ctx, SGN_EINVAL, "sgn_rng_next_u64_batch: hosts must be distinct");
  if (total && !out) return SGN_EINVAL;
  if (n == 0) return 0;
  if (int rc = rng_release(ctx)) return rc;
  SGN_HIP(ctx, hipSetDevice(ctx->device));
  char* d = nullptr;
  const size_t bytes = (size_t)n * (4 + 4 + 8) + total * 8 + 16;
  SGN_HIP(ctx, hipMalloc(&d, bytes));
  uint32_t* dh = (uint32_t*)d;
  uint32_t* dc = dh + n;
  uint64_t* doff = (uint64_t*)(d + ((size_t)n * 8 + 7) / 8 * 8);
  uint64_t* dout = doff + n;
  hipError_t e = hipMemcpyAsync(dh, loc.data(), (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dc, counts, (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(doff, off.data(), (size_t)n * 8, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_rng, dim3((n + 63) / 64), dim3(64), 0, ctx->stream, (const DevSim*)ctx->d_S, dh, dc,
                       doff, n, dout);
    e = hipGetLastError();
  }
  if (e == hipSuccess && total) e = hipMemcpyAsync(out, dout, total * 8, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  hipFree(d);
  if (e != hipSuccess) return hip_fail(ctx, e, "host rng draws");
  return 0;
}
int rng_draw(sgn_ctx* ctx, uint32_t host, uint32_t n, uint64_t* out) {
  return rng_cpu_draws(ctx, host, n, out);
}
}  // namespace

int sgn_rng_next_u64_batch(sgn_ctx* ctx, const uint32_t* hosts, const uint32_t* counts, uint32_t n,
                           uint64_t* out) {
  if (ctx) ctx->ctrl_fresh = false;  // (it may change the device control block)
  return rng_draws(ctx, hosts, counts, n, out);
}

int sgn_rng_next_u64(sgn_ctx* ctx, uint32_t host, uint64_t* out) {
  if (ctx) ctx->ctrl_fresh = false;  // (it may change the device control block)
  return rng_draw(ctx, host, 1, out);
}

int sgn_rng_double(sgn_ctx* ctx, uint32_t host, double* out) {
  if (ctx) ctx->ctrl_fresh = false;  // (it may change the device control block)
  if (!out) return SGN_EINVAL;
  uint64_t x = 0;
  int rc = rng_draw(ctx, host, 1, &x);
  if (rc == 0) *out = (double)(x >> 11) * 0x1.0p-53;
  return rc;
}

int sgn_rng_fill_bytes(sgn_ctx* ctx, uint32_t host, uint8_t* buf, size_t len) {
  if (ctx) ctx->ctrl_fresh = false;  // (it may change the device control block)
  if (!buf && len) return SGN_EINVAL;
  if (len / 8 + 1 > 0xFFFFFFFFull) return set_error(ctx, SGN_ERANGE, "sgn_rng_fill_bytes: len too large");
  const size_t full = len / 8, rem = len % 8;
  std::vector<uint64_t> v(full + (rem ? 1 : 0));
  int rc = rng_draw(ctx, host, (uint32_t)v.size(), v.data());
  if (rc) return rc;
  for (size_t i = 0; i < full; i++)
    for (int k = 0; k < 8; k++) buf[8 * i + k] = (uint8_t)(v[i] >> (8 * k));
  if (rem) {
    // fill_bytes_via_next: 5..7 bytes from next_u64, 1..4 from next_u32 = next_u64 >> 32
    const uint64_t w = rem > 4 ? v[full] : (v[full] >> 32);
    for (size_t k = 0; k < rem; k++) buf[8 * full + k] = (uint8_t)(w >> (8 * k));
  }
  return 0;
}

// Test hook: device CoDel control-law increments for count in [0, n).
int sgn_selftest_codel_law(sgn_ctx* ctx, uint64_t n, uint64_t* out) {
  if (ctx) ctx->ctrl_fresh = false;  // (it may change the device control block)
  if (!ctx || !out) return SGN_EINVAL;
  SGN_HIP(ctx, hipSetDevice(ctx->device));
  uint64_t* d = nullptr;
  SGN_HIP(ctx, hipMalloc(&d, n * 8));
  hipLaunchKernelGGL(k_codel_law_test, dim3(1024), dim3(256), 0, ctx->stream, n, d);
  hipError_t e = hipMemcpyAsync(out, d, n * 8, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  hipFree(d);
  if (e != hipSuccess) return hip_fail(ctx, e, "codel law selftest");
  return 0;
}

}  // extern "C"

// hooks used by comm.cpp
namespace sgn {
// The CPU-held states go back before anything on the device uses a host RNG (rounds, batch
// draws, digests): one small upload and one kernel, stream-ordered (no host wait).
int rng_release(sgn_ctx* ctx) {
  if (ctx->rng_held.empty() || !ctx->sim_ready) {
    ctx->rng_held.clear();
    return 0;
  }
  std::vector<uint64_t> st;
  st.reserve(ctx->rng_held.size() * 6);
  for (auto& kv : ctx->rng_held) {
    if (!kv.second.draws) continue;
    st.push_back(kv.first);
    for (int k = 0; k < 4; k++) st.push_back(kv.second.s[k]);
    st.push_back(kv.second.draws);
  }
  ctx->rng_held.clear();
  const uint32_t n = (uint32_t)(st.size() / 6);
  if (!n) return 0;
  SGN_HIP(ctx, hipSetDevice(ctx->device));
  if (ctx->rng_stage_cap < st.size()) {
    if (ctx->d_rng_stage) hipFree(ctx->d_rng_stage);
    ctx->d_rng_stage = nullptr;
    ctx->rng_stage_cap = 0;
    SGN_HIP(ctx, hipMalloc(&ctx->d_rng_stage, st.size() * 8));
    ctx->rng_stage_cap = st.size();
  }
  SGN_HIP(ctx, hipMemcpyAsync(ctx->d_rng_stage, st.data(), st.size() * 8, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_rng_set, dim3((n + 63) / 64), dim3(64), 0, ctx->stream, (const DevSim*)ctx->d_S,
                     (const uint64_t*)ctx->d_rng_stage, n);
  SGN_HIP(ctx, hipGetLastError());
  SGN_HIP(ctx, hipStreamSynchronize(ctx->stream));  // (the staging vector goes out of scope)
  return 0;
}

void launch_execute(sgn_ctx* ctx) { launch_k_execute(ctx, ctx->stream); }
// k_import files the received runs and its last block advances the window
void launch_import(sgn_ctx* ctx) {
  hipLaunchKernelGGL(k_import, dim3(kImportBlocks), dim3(256), 0, ctx->stream, ctx->S);
  if (!ctx->capturing) ctx->kt[K_IMPORT].total++;
}
}  // namespace sgn

uint64_t sgn::layout_sig_engine() { return kLayoutSig; }
