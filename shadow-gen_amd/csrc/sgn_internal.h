// sgn_internal.h — device-state layout and host-side context of libsgn (gfx950 only).
//
// Layout in HBM (one shard = a contiguous HostId range [lo, lo + nH)):
//   * per-host state is structure-of-arrays indexed by the local host index, so a wave of
//     64 consecutive hosts loads each field with one coalesced access;
//   * in-flight packet events live in a calendar of NB time buckets of width BW ns; each
//     bucket is a fixed slab of BC 32-byte event records in one pool (plus one spare slab
//     that receives the partially consumed bucket's survivors each round);
//   * the events due in a window are counting-sorted by destination host into per-host
//     segments, which the execute kernel orders by (time, src host, src event id).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "sgn.h"

namespace sgn {

// Device pointers in DevSim carry the global address space in device code, so loads and
// stores through them are global_* (not flat_*) even though DevSim is read from memory.
#ifdef __HIP_DEVICE_COMPILE__
#define SGN_GLB __attribute__((address_space(1)))
#else
#define SGN_GLB
#endif
// Read-only for a kernel's lifetime (the constant address space): loads through it are
// invariant, so uniform ones are scalar loads (k_rounds_x's per-shard DevSim: read through a
// plain pointer from the launch descriptor, every field access was a vector flat load)
#ifdef __HIP_DEVICE_COMPILE__
#define SGN_CONST __attribute__((address_space(4)))
#else
#define SGN_CONST
#endif

constexpr uint64_t SIM_START = SGN_SIMULATION_START;
constexpr uint64_t EMU_MAX = SGN_EMUTIME_MAX;
constexpr uint64_t INVALID = SGN_EMUTIME_INVALID;

// A run of in-flight packet events (core/work/event.rs:20-31 + the packet fields the core
// needs): `count` packets from one source to one destination with the same delivery time,
// payload and tag and CONSECUTIVE source event ids eid, eid+1, ... Shadow queues each of
// them as its own Event; a run is only a compact encoding of events that are adjacent in
// Shadow's order anyway (same time and source, consecutive ids: nothing sorts between
// them), so popping a run = popping its packets one by one. A single packet is a run of 1.
struct __attribute__((aligned(16))) EvRec {
  uint64_t time;     // delivery time (EmulatedTime)
  uint64_t eid;      // source host's event id of the first packet
  uint32_t src;      // source HostId
  uint32_t dst;      // destination HostId
  uint32_t pc;       // UDP payload bytes (low 16; wire = payload + 28) | packets (high 16, >= 1)
  uint32_t tag;      // opaque app tag
};
static_assert(sizeof(EvRec) == 32, "EvRec is two 16-byte halves");
__host__ __device__ __forceinline__ uint32_t ev_payload(const EvRec& e) { return e.pc & 0xFFFFu; }
__host__ __device__ __forceinline__ uint32_t ev_count(const EvRec& e) { return e.pc >> 16; }
constexpr uint32_t RUN_MAX = 0xFFFFu;  // packets per event run

// A run of entries of the inbound CoDel queue (router/codel_queue.rs:51-54): `count`
// packets enqueued at the same time from one source with consecutive event ids and the
// same payload and tag (the same encoding as EvRec; CoDel still handles them one by one).
struct __attribute__((aligned(16))) CodelEnt {
  uint64_t enqueue_ts;
  uint64_t eid;      // first packet's source event id
  uint32_t src;
  uint32_t payload;
  uint32_t tag;
  uint32_t count;    // packets in the run (>= 1)
};
static_assert(sizeof(CodelEnt) == 32, "");

// One entry of the synthetic socket send queue (a train of `count` datagrams). The peer is
// resolved to its HostId when the datagram is queued: Dns::addr_to_host_id
// (network/dns.rs:174) is a pure function of the address and host addresses are unique
// (dns.rs:97-131), so resolving at enqueue gives Worker::send_packet the same HostId.
constexpr uint32_t NO_HOST = 0xFFFFFFFFu;  // address not in the simulation (InetDropped)
struct __attribute__((aligned(16))) FifoEnt {
  uint32_t dst;    // destination HostId, or NO_HOST
  uint32_t pay;    // payload (low 16) | last payload (high 16)
  uint32_t count;
  uint32_t tag;
};
static_assert(sizeof(FifoEnt) == 16, "");

// A route entry as the packet path reads it (WorkerShared::latency / reliability,
// worker.rs:523-537): the latency and the integer loss threshold T = reliability * 2^53
// (reliability = (f64)(1.0f - loss); the drop test is (x >> 11) >= T, see send_batch) — one
// 16-byte load instead of a latency line and a loss line.
struct __attribute__((aligned(16))) RouteEnt {
  uint64_t lat;
  uint64_t T;
};
static_assert(sizeof(RouteEnt) == 16, "");

// Round control block, device resident. The window advances on the device.
struct Ctrl {
  uint64_t ws, we;        // current window [ws, we)
  uint32_t active;        // 0 once the controller returned None
  uint32_t overflow;      // bit flags (OVF_*); first offender in overflow_info
  uint64_t overflow_info;
  uint64_t round_min;     // atomicMin: next local event over owned hosts
  uint64_t min_used;      // Runahead::min_used_latency (atomicMin), INVALID = None
  uint32_t keep_slab;     // spare slab: receives the window's last bucket this round
  uint32_t imp_done;      // multi-shard: k_import blocks finished this round (the last one advances)
  uint64_t keep_min;      // min time placed in the spare slab this round
  uint64_t last_min_next; // min_next_event_time of the last finished round
  uint64_t rounds;
  uint64_t max_bucket;    // high-water mark of any (bucket, host group) slab fill
  uint64_t trace_n;       // trace records produced
  uint64_t spill_imp;     // multi-shard: spill-area entries written by the last k_import (read by
                          // the next round's gathers: runs imported past their slab, lossless)
  uint64_t epoch;         // persistent rounds: round edges published (grid barrier)
  uint64_t prev_we;       // end of the last executed window (sgn_set_window's lower bound)
  uint64_t drain_n;       // drain records produced since the last sgn_drain
  // persistent launch residency census. Never reset: res_arrive counts every workgroup of every
  // persistent launch since sim_init (the host passes the count before a launch, sgn_ctx::res_base,
  // and the census compares against it), and res_verdict carries the launch's epoch (epoch << 2 |
  // verdict: 1 = whole grid resident, 2 = not, 3 = a peer shard not resident — every workgroup
  // left before touching simulation state; the host falls back to per-round launches). A memset
  // of either word breaks the census arithmetic.
  uint32_t res_arrive, res_verdict;
  // multi-shard exchange sizing: runs per peer the round's RCCL send/recv moves (set by the
  // host per batch; a slot holds up to xslot), 1 while a round is held because some shard
  // had more runs for a peer than that (the host completes it with a full-slot exchange),
  // and the largest per-peer run count any shard produced in a round so far
  uint32_t xsz, xspill;
  uint64_t xhwm;
  // CoDel page pool: allocations so far (index into the free ring), free-ring entries
  // written so far, entries allocations may use this round (the ring as of the last round
  // edge: a page freed in a round is reused from the next one), pages freed this round
  // (per-round launches; the persistent kernel counts in DevSim::rb_free)
  uint64_t pg_alloc, pg_tail, pg_avail, pg_freed;
  // Pools that grow instead of refusing a scenario (the reference's queues are unbounded):
  // runs in the event calendar (appended - gathered; the CoDel guard's bound), runs placed in
  // the calendar's spill area this batch (their slab was full), and the hold flags (HOLD_*)
  // that stop the rounds at a round edge — nothing of the next round has run — until the host
  // has grown the pool; hold_need = the CoDel pages the held round may take
  uint64_t cal_occ;
  uint64_t spill_n;
  uint32_t hold;
  // one shard per GPU (k_rounds_x): the peers' census combined by this shard's deciding
  // workgroup (epoch << 2 | verdict, as res_verdict); the shard's other workgroups read only this
  uint32_t res_xverdict;
  uint64_t hold_need;
  uint64_t rnd_alloc, rnd_spill;  // per-round launches: the Outbox counters' target (unread)
};

static_assert(offsetof(Ctrl, min_used) == offsetof(Ctrl, round_min) + 8,
              "comm.cpp all-reduces {round_min, min_used} as one u64[2]");

// hold flags (Ctrl::hold): why the rounds stopped at a round edge
enum : uint32_t {
  HOLD_CODEL = 1u,  // the next round could take more CoDel pages than the pool has free
  HOLD_SPILL = 2u,  // runs went to the calendar's spill area: the calendar is re-laid out
  HOLD_XSLOT = 4u,  // persistent multi-shard: some shard sent a peer more runs than its inbox slot
                    // holds (the rest wait in the sender's spill area: the host moves them)
  HOLD_XGROW = 8u,  // persistent multi-shard: a round used more than half an inbox slot (grow)
};

enum : uint32_t {
  OVF_BUCKET = 1u,
  OVF_CODEL = 2u,
  OVF_FIFO = 4u,
  OVF_SEG = 8u,
  OVF_EXCHANGE = 16u,
  OVF_TRACE = 32u,
  OVF_TIMEOUT = 64u,  // a persistent grid barrier gave up (grid not resident)
  OVF_DRAIN = 128u,   // drain buffer full (raise sgn_drain_enable's capacity)
  OVF_HORIZON = 256u, // a delivery beyond the event calendar's horizon
};

// One host's state record (array of records, one per owned host, 512 B, 128-B aligned).
// A round touches only the hosts with something due (~1 in 8 at config C, every host at D).
// Line 0 is the HOT line: what Host::execute reads and writes every time a host runs (RNG,
// event-id counter, the app's timer, token buckets, digests, app counter, flags, CoDel page).
// Lines 1-3 are COLD: the relays' pending tasks and cached packets, the CoDel and send queues'
// bookkeeping, the route cache, CoDel's drop state, rare counters. PERIODIC hosts (configs B, D)
// end nearly every round with both queues empty and both relays idle: their store() leaves the
// cold lines alone (F_COLD clear: the cold state is the default of an idle host, whatever the
// lines hold) and load() reads them only when F_COLD is set. TGEN / EXTERNAL hosts always use
// them. The per-host totals are no-return atomic adds into dense arrays (DevSim::n_cnt, maxq)
// and the constants (HostId, address, node, refill increments) a dense array of their own, so
// an idle PERIODIC host-round moves one line each way plus 32 read bytes.
constexpr uint32_t CQ_PAGE = 16;  // CoDel runs per pool page (cq_head = page * CQ_PAGE + offset)

struct __attribute__((aligned(128))) HostRec {
  // ---- line 0: hot ----
  uint64_t rng[4];           // Xoshiro256++ state (host/host.rs:234)
  uint64_t eid;              // next event id (host.rs:259,662-666)
  uint64_t st2, se2;         // the app's local event slot: time, event id
  uint64_t tb_bal[2];        // token buckets (0 = inet_out, 1 = inet_in): balance ...
  uint64_t tb_last[2];       // ... last refill
  uint64_t dig[3];           // digests tx, rx, app
  uint64_t app_k;            // synthetic app counter
  uint32_t flags, cq_head;   // flag bits; CoDel head run (pool index; an empty queue keeps its page)
  // ---- lines 1-3: cold ----
  // (first: the queue fields that the next loads depend on — the CoDel head run and the send
  // queue's head entry are loaded from them in load(); from the third line they cost config C
  // 1 % per launch, same-box A/B of this order against the previous one, round 4)
  uint32_t cq_nr, cq_len, cq_tp;             // CoDel runs / packets / chain's tail page
  uint32_t fq_head, fq_len;                  // send queue (an empty queue's head is 0)
  uint32_t rc_dst, rc_sid, pad_c;            // route cache peer (NO_HOST: none) and its slot id
  uint64_t st0, se0, st1, se1;  // local event slots: relay out, relay in (time, event id)
  uint64_t ri_eid;           // relay_inet_in cached packet: src event id
  uint64_t cq_bytes;         // CoDel queued bytes
  uint64_t rc_lat, rc_T;     // route cache: latency, integer loss threshold (TGEN, EXTERNAL)
  uint64_t cq_ie, cq_dn, cq_cur, cq_prev;    // CoDel interval end / drop next / counts
  uint32_t ro_dst, ro_pay, ro_tag;           // relay_inet_out cached packet
  uint32_t ri_src, ri_pay, ri_tag;           // relay_inet_in cached packet
  // TGEN / EXTERNAL (their cold lines are read and written with the hot one anyway): the
  // constants and the per-host totals here, in the lines they already move (PERIODIC: the
  // dense HostConst array and no-return adds into DevSim::n_cnt / maxq)
  uint64_t k_tbinc[2];                       // = HostConst::tb_inc
  uint32_t k_gid, k_ip, k_unode, max_codel;  // = HostConst; the largest CoDel queue length
  uint64_t n_sent, n_popped, n_delivered;
  // rare paths only (never loaded with the state: traced runs, sgn_rng_*, no-return atomics)
  uint64_t tseq;                            // trace sequence
  uint64_t rng_pos;                         // RNG draws so far (kept while tracing, and by sgn_rng_*)
  uint64_t n_codel, n_unknown, n_local_deliv, n_blocked;
  uint64_t pad[16];
};
static_assert(sizeof(HostRec) == 512, "HostRec is 4 cache lines");
// PERIODIC simulations (configs B and D): the hot line lives in per-64-host tiles, field-major —
// its 16-byte chunk c of host slot h at DevSim::htile[hot_idx(h, c)], so a wave's load of one
// chunk is one contiguous 1 KB access instead of 64 lines (HostRec's line 0 is then unused on
// the device; engine.hip kSoa)
__host__ __device__ inline size_t hot_idx(uint32_t h, uint32_t c) { return ((size_t)(h >> 6) * 8 + c) * 64 + (h & 63); }
static_assert(offsetof(HostRec, cq_nr) == 128, "line 0: the hot line");
// the constants of a host's slot, read with the hot line (32 B)
struct __attribute__((aligned(32))) HostConst {
  uint32_t gid, ip, unode, pad;  // HostId, address, used-node index
  uint64_t tb_inc[2];            // token-bucket refill increments (capacity = increment + MTU)
};
static_assert(sizeof(HostConst) == 32, "");
enum { N_SENT = 0, N_POPPED, N_DELIVERED, N_CNT };  // DevSim::n_cnt rows

// per-wave counters (DevSim::w_cnt rows of G)
enum { W_EXEC = 0, W_RUNS, W_SORTED, W_LOSS, W_LOCAL_EV, W_BYTES, W_MAXFILL, W_BIG, W_N };  // W_MAXFILL: max, not sum
                                                                                            // W_BIG: big-slab pieces

// host flag bits
enum : uint32_t {
  F_RO_STATE = 0x3u,         // relay_inet_out state (Idle/Pending/Forwarding)
  F_RI_STATE_SHIFT = 2,      // relay_inet_in state << 2
  F_RO_NEXT = 0x10u,         // relay_inet_out cached packet
  F_RI_NEXT = 0x20u,         // relay_inet_in cached packet
  F_SERVER = 0x40u,          // TGEN server
  F_CODEL_DROP = 0x80u,      // CoDel mode Drop
  F_CODEL_IE = 0x100u,       // CoDel interval_end is Some
  F_CODEL_DN = 0x200u,       // CoDel drop_next is Some
  F_HAS_APP = 0x400u,        // host runs a synthetic app timer
  F_RO_CONT = 0x800u,        // inside relay_inet_out's forwarding task (never stored)
  F_FH_DIRTY = 0x1000u,      // the send queue's head exists only in LDS (never stored)
  F_COLD = 0x2000u,          // the record's cold lines hold the host's state (else: idle defaults)
};

enum { SLOT_RO = 0, SLOT_RI = 1, SLOT_APP = 2, NSLOT = 3 };

// Division by a run-time invariant u64 d > 0 as a multiply-high and shifts (the libdivide
// "round up / add indicator" scheme): exact for every u64 x. GPU u64 division is a long
// software routine; the round kernel divides every event time by the bucket width.
struct UDiv64 {
  uint64_t m;      // magic multiplier (0: d is a power of two)
  uint32_t shift;
  uint32_t add;    // 1: use the add-indicator form
  __host__ void init(uint64_t d) {
    const uint32_t l = 63u - (uint32_t)__builtin_clzll(d);
    if ((d & (d - 1)) == 0) {
      m = 0;
      shift = l;
      add = 0;
      return;
    }
    const unsigned __int128 num = (unsigned __int128)1 << (64 + l);
    uint64_t pm = (uint64_t)(num / d);
    const uint64_t rem = (uint64_t)(num % d);
    const uint64_t e = d - rem;
    if (e < (1ULL << l)) {
      add = 0;
    } else {
      pm += pm;
      const uint64_t r2 = rem + rem;
      if (r2 >= d || r2 < rem) pm += 1;
      add = 1;
    }
    m = pm + 1;
    shift = l;
  }
  __host__ __device__ __forceinline__ uint64_t div(uint64_t x) const {
    if (m == 0) return x >> shift;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint64_t q = __umul64hi(m, x);
#else
    const uint64_t q = (uint64_t)(((unsigned __int128)m * x) >> 64);
#endif
    if (add) return (((x - q) >> 1) + q) >> shift;
    return q >> shift;
  }
};

// Everything the round kernels need, passed by value as a kernel argument.
struct DevSim {
  // shard and config
  uint32_t n_all, lo, nH, U;
  uint64_t end_time, boot_end, runahead_cfg;
  uint64_t min_possible;
  uint64_t max_lat;   // largest route latency (the persistent kernel's calendar-alias check)
  int32_t dynamic;
  uint32_t fifo_cap;
  uint32_t cq_pages;  // CoDel page pool: pages of CQ_PAGE runs (every host owns >= 1)
  uint32_t qdisc_rr;  // interface_qdisc == SGN_QDISC_ROUND_ROBIN
  uint32_t pad_q;
  uint32_t trace_on;
  // traffic
  uint32_t tkind, payload_len, unknown_permille, req_payload;
  uint32_t n_servers;
  uint32_t diag_mode;  // diagnostic build only (SGN_DIAG_MODE): 1 = light waves skip
  uint64_t flow_seed, period, period_jitter;
  uint64_t file_bytes[3];
  SGN_GLB const uint32_t* servers;
  // routing (replicated on every shard)
  SGN_GLB const uint64_t* rlat;
  SGN_GLB const float* rloss;
  SGN_GLB const uint32_t* unode;  // [n_all] used-node index of every host
  SGN_GLB const uint32_t* ip;     // [n_all]
  // Hosts live in SLOTS: a shard's HostId range [lo, hi) is permuted so that hosts of the
  // same kind (server / client, bandwidth class) share waves (their event loops converge).
  // A slot id (sid) is lo + slot; event records carry the destination's sid.
  SGN_GLB const uint32_t* sid_of;   // [n_all] HostId -> sid (every shard's permutation)
  SGN_GLB const uint64_t* peer;     // [n_all] HostId -> sid | used-node index << 32 (one load per peer)
  SGN_GLB const uint32_t* peer32;   // the same packed in 4 bytes (sid | node << peer_sb) when it fits, else null
  uint32_t peer_sb;                 // sid bits of peer32
  SGN_GLB const RouteEnt* route;    // [U x U] {latency, loss threshold} (routing table, packet-path form)
  SGN_GLB const uint32_t* host_of;  // [nH] slot -> HostId of this shard
  SGN_GLB const uint32_t* dns_key;
  SGN_GLB const uint32_t* dns_val;
  uint32_t dns_mask;
  uint32_t pad1;
  // host state: one record per owned host, and each host's next local event time (read
  // for all hosts at the start of a round: a dense array keeps that read coalesced)
  SGN_GLB HostRec* hrec;        // [nH]
  SGN_GLB const HostConst* hconst;  // [nH]
  SGN_GLB uint64_t* n_cnt;      // [N_CNT * nH] per-host totals (sent, popped, delivered)
  SGN_GLB uint32_t* maxq;       // [nH] per-host largest CoDel queue length
  SGN_GLB uint64_t* nextloc;    // [nH]
  // PERIODIC traffic: the peer (HostId, NO_HOST for an unknown address) of each host's next
  // datagram, a hash of its app counter written when the host's record is stored, so the next
  // round loads the peer's slot and node beside the host record instead of after it
  SGN_GLB uint32_t* npeer;      // [nH] (null for other traffic kinds)
  // CoDel queues (Router's inbound CoDelQueue, unbounded in the reference) as chains of
  // pages from ONE pool sized by total occupancy, not per host: a host's queue is its runs
  // in order over a chain head page -> ... -> tail page (cq_next links them). Pages leave
  // the chain from the head and go back through the free ring.
  SGN_GLB CodelEnt* codel;      // [cq_pages * CQ_PAGE] page pool
  SGN_GLB uint32_t* cq_next;    // [cq_pages] next page of the chain
  SGN_GLB uint32_t* cq_free;    // [cq_pages] free ring (Ctrl::pg_alloc / pg_tail index it mod cq_pages)
  SGN_GLB uint64_t* rb_free;    // [3] persistent rounds: pages freed in the round (by round % 3)
  SGN_GLB FifoEnt* fifo;        // [nH * fifo_cap] send queue per host
  SGN_GLB uint32_t* fifo_addr;  // [nH * fifo_cap] traced runs: an unknown entry's address
  // calendar: NB time buckets of width BW; every bucket is a set of slabs, one per host
  // group (2^gsh consecutive hosts = one wave of k_execute), of CAP event runs each. Slab
  // ids are indirect (bucket_slab) so the partially consumed last bucket of a window can
  // swap with the spare slab set (Ctrl::keep_slab) instead of being copied.
  SGN_GLB EvRec* pool;            // [(NB + 1) * G * CAP]
  SGN_GLB uint32_t* slab_n;       // [(NB + 1) * G] fill of slab (s, g)
  SGN_GLB uint32_t* bucket_slab;  // [NB] slab id of bucket b
  SGN_GLB uint64_t* bucket_min;   // [NB] earliest event in bucket b (INVALID = empty)
  // spill area: a run whose slab is full goes here with its slab index (lossless); the round
  // edge then holds and the host re-lays the calendar out with larger slabs before any spilled
  // run can be due (appends only ever target buckets after the running window)
  SGN_GLB EvRec* spill;           // [spill_cap]
  SGN_GLB uint32_t* spill_idx;    // [spill_cap] (slab set, group) index of each spilled run
  uint64_t spill_cap;
  // slab extensions (a hot slab: thousands of sources sending to one host group in one bucket
  // width): runs past a slab's CAP continue in its extension, ext[slab] = offset into ext_pool
  // | capacity << 40 (0: none), laid out by the host at a held round edge (relayout_calendar).
  // A slab with more runs than the LDS holds is ordered in pieces (exec_group's big-slab path).
  SGN_GLB const uint64_t* ext;    // [(NB + 1) * G] or null (no slab has an extension)
  SGN_GLB EvRec* ext_pool;
  uint64_t ext_total;             // runs in all extensions (the CoDel guard's due-run bound)
  uint32_t NB, G;         // NB: a power of two (bucket index = (t / BW) & (NB - 1))
  uint32_t CAP;
  uint32_t gsh;           // log2(hosts per group); a group is served by one 64-lane wave
  // per-wave cumulative counters (one row slot per wave, no-return adds: no same-address
  // atomics across thousands of waves): {host executions, due runs, sorted segments, ...}
  SGN_GLB uint64_t* w_cnt;        // [W_N * G]
  SGN_GLB uint32_t* fin_cnt;      // [ceil(G / 64) + 1] arrival counters (chunks, then chunks done)
  SGN_GLB uint64_t* fin_keep;     // [ceil(G / 64)] per-chunk minima (atomicMin) of w_keep / w_next
  SGN_GLB uint64_t* fin_next;
  SGN_GLB uint64_t* fin_occ;      // [ceil(G / 64)] per-chunk calendar occupancy change (two's complement sums)
  // persistent rounds (k_rounds): per round % 3, chunk minima {kept, next} and the minimum of
  // new runs for the window's last bucket, and the arrival counters (chunks, then chunks done)
  SGN_GLB uint64_t* rb_min;       // [3][64][2]
  SGN_GLB uint64_t* rb_keep;      // [3]
  SGN_GLB uint32_t* rb_cnt;       // [3][65], then one monotone counter: the gap barrier (k_rounds)
  SGN_GLB uint64_t* rb_occ;       // [3][64] per-chunk calendar occupancy change of the round,
                                  // then rb_alloc [3] (pages allocated) and rb_spill [3] (runs spilled)
  uint32_t gspec;         // slab slots a gather loads before the fill is known (sim_init)
  uint32_t fuse_finalize; // single shard: k_execute's last wave runs the round edge
  uint32_t agg_bmin;      // the round kernels fold bucket minima in an LDS table (see engine.hip)
  uint64_t BW;
  UDiv64 bw_div;          // division by BW
  UDiv64 div_n, div_1000, div_ns;  // by n_all, 1000, n_servers (the synthetic apps' hashes, exact)
  SGN_GLB uint64_t* stamps;     // diagnostics (nullptr unless SGN_STAMPS is set)
  SGN_GLB uint64_t* rdbg;       // ... per-round timeline of the persistent kernel
  uint32_t n_ranks;
  SGN_GLB Ctrl* ctrl;
  // trace
  SGN_GLB sgn_trace_rec* trace;
  uint64_t trace_cap;
  // EXTERNAL traffic: interface deliveries and drops for the CPU-side applications
  SGN_GLB sgn_drain_rec* drain;
  uint64_t drain_cap;
  // multi-GPU exchange: xout block r (1 + xslot records) goes to rank r, xin block r came
  // from it. Record 0 of a block is the round-edge message, 4 u64: {runs sent to that peer,
  // the sender's min next event (incl. the runs it exported this round), its min used
  // latency, its largest per-peer run count}; runs follow from record 1. This shard's own
  // message is record 0 of its own xin block.
  SGN_GLB EvRec* xout;
  SGN_GLB uint32_t* xout_n;  // [n_ranks] runs appended per peer this round
  SGN_GLB EvRec* xin;
  SGN_GLB uint32_t* xin_n;   // (unused)
  uint32_t xslot;    // run capacity per peer block
  uint32_t rank;
  SGN_GLB const uint32_t* rank_lo;  // [n_ranks + 1] host ranges
  // persistent multi-shard rounds (k_rounds_x): this shard's view of every shard's inbox (xp[q],
  // q = this shard: its own), its own inbox (headers [2][n_ranks][XH_WORDS], runs [2][n_ranks]
  // [xslot], census words [n_ranks]), and the second barrier's counters (after the imports)
  SGN_GLB const struct XPeer* xp;
  SGN_GLB uint64_t* xin_hdr;
  SGN_GLB EvRec* xin_runs;
  SGN_GLB uint64_t* xin_cen;
  SGN_GLB uint32_t* rb2_cnt;  // [3][RB_CB_MAX]
  uint32_t xislot;            // inbox runs per sender and round parity
  uint32_t xsys;              // 1: the inboxes are other GPUs' (uncached, system-scope accesses);
                              // 0: one GPU's (a local group: device-scope accesses, L2-served)
  uint32_t xown;              // a round's imports up to this many runs: filed by their own
                              // workgroups at the next round's start (else shared + a barrier)
  uint32_t xbk;               // inbox bins: runs per (round parity, sender, receiving host group)
  // inbox bins (k_rounds_x): [2][n_ranks][G][xbk] runs sent to this shard, binned by the
  // receiving host group, which reads its own bins during its next gather (empty entries: pc 0,
  // the reader zeroes what it took); the senders' position counters per (parity, receiver,
  // receiving group), [2][n_ranks][xgx]
  SGN_GLB EvRec* xin_bins;
  SGN_GLB uint32_t* xbin_n;
  uint32_t xgx;               // the largest shard's host groups (the counters' row length)
  uint32_t rdbg_wg;           // diagnostics: rdbg holds every workgroup's stamps (SGN_STAMPS=3)
  // the control block's host-visible copy (pinned host memory): the persistent kernel's last
  // workgroup writes it at the launch's end, then the launch's census epoch in the word after it
  // (the host reads it after the stream synchronises, instead of a device-to-host copy)
  SGN_GLB uint64_t* ctrl_mirror;
  SGN_GLB uint64_t* htile;    // PERIODIC: the hot lines, tiled (hot_idx; null: in HostRec)
};

// Persistent multi-shard rounds (k_rounds_x): every shard owns an INBOX — per sender shard and
// round parity a message (the round edge's, below) and a slot of xislot runs — that the senders
// write directly (peer-mapped memory
// across GPUs, ordinary device memory when the shards are workgroup ranges of one launch).
// XPeer is one sender's view of one receiver's inbox: where its runs and its message go in each
// round parity, and its census word. runs[2] is the RCCL transport's send block (per-round path).
// bins[k]: this sender's bins in the receiver's inbox for round parity k ([G_receiver][xbk]).
struct XPeer {
  SGN_GLB EvRec* runs[3];
  SGN_GLB uint64_t* hdr[2];
  SGN_GLB uint64_t* cen;
  SGN_GLB EvRec* bins[2];
};
// A message is 16 GRANULES of 16 bytes: granule k holds message word k as two TAGGED 8-byte
// words {lo32 | tag32 << 32, hi32 | tag32 << 32} (xh_pack / xh_unpack), tag32 the low 32 bits
// of the global round number + 1. Every 8-byte word carries the tag, so the receiver never
// trusts more than one naturally aligned 8-byte store to arrive whole: across GPUs (xGMI) each
// word is written by its own 8-byte system-scope atomic store, within one GPU a granule by one
// 16-byte store. The receiver polls them and has the values in the same round trip: 256 bytes,
// XH_WORDS u64.
constexpr uint32_t XH_WORDS = 32;
__host__ __device__ inline uint32_t xh_tag32(uint64_t tag) { return (uint32_t)tag; }
__host__ __device__ inline uint64_t xh_lo(uint64_t v, uint64_t tag) { return (v & 0xFFFFFFFFull) | ((uint64_t)xh_tag32(tag) << 32); }
__host__ __device__ inline uint64_t xh_hi(uint64_t v, uint64_t tag) { return (v >> 32) | ((uint64_t)xh_tag32(tag) << 32); }
__host__ __device__ inline bool xh_ok(uint64_t lo, uint64_t hi, uint64_t tag) {
  return (uint32_t)(lo >> 32) == xh_tag32(tag) && (uint32_t)(hi >> 32) == xh_tag32(tag);
}
__host__ __device__ inline uint64_t xh_val(uint64_t lo, uint64_t hi) { return (lo & 0xFFFFFFFFull) | (hi << 32); }
enum : uint32_t {  // granule k holds message word k (its tag: the global round number + 1)
  XH_CNT = 0,    // runs the sender put in this receiver's slot this round (may exceed the slot)
  XH_MIN,        // the sender's min next event time, the runs it exported included (EMU_MAX: none)
  XH_MU,         // the sender's min used latency (dynamic runahead; INVALID: none)
  XH_XMAX,       // the sender's largest per-peer run count this round
  XH_SPILL,      // the sender's spill area holds runs (the calendar must be re-laid out)
  XH_PFREE,      // the sender's free CoDel pages for the next round
  XH_OCC,        // the sender's calendar occupancy (before this round's imports)
  XH_XSUM,       // runs the sender exported this round (a bound on what any shard receives)
  XH_CAPB,       // the sender's slab runs per bucket (extensions included)
  XH_NH,         // the sender's hosts
  // the sender's own round edge, read by its own workgroups (the message to itself): the spare
  // slab's new minimum, the calendar occupancy change, CoDel pages allocated and freed
  XH_NB1,
  XH_OCCD,
  XH_NALLOC,
  XH_NFREE,
  XH_TOT,        // runs the sender sent this receiver this round: its bins and its slot
  XH_N
};
// k_rounds_x launch descriptor (device memory): the shards this launch runs, each on a
// contiguous range of workgroups (all shards of a local group on one GPU, or this GPU's one)
constexpr uint32_t XL_MAX = 16;
struct XLaunch {
  uint32_t n_local;              // shards in this launch
  uint32_t peers_census;         // 1: one shard per GPU: the census is exchanged with the peers
  uint64_t epoch;                // launch number (census tags)
  uint32_t res_base;             // the first shard's census arrival count before this launch
  uint32_t refuse;               // one shard per GPU: this GPU cannot hold a resident grid; the
                                 // launch (one workgroup) only tells the peers "not resident"
  uint32_t base[XL_MAX + 1];     // workgroup range of local shard i: [base[i], base[i + 1])
  const SGN_CONST struct DevSim* S[XL_MAX];
};

constexpr uint32_t SPILL_PEER = 0x80000000u;  // spill area tag: a run for that peer shard's exchange slot
constexpr uint32_t SPILL_DEAD = 0xFFFFFFFFu;  // spill area tag: a run a gather already took (multi-shard)
constexpr uint64_t EXT_OFF_MASK = (1ULL << 40) - 1;  // DevSim::ext: offset bits (capacity above)
constexpr uint32_t XHDR = 2;  // multi-shard: message records (64 B) at the head of a peer's block
constexpr uint32_t GROUP_MAX = 64;  // hosts per group <= lanes of one k_execute wave
// event runs per (bucket, group) slab: one bucket's due runs of a group are ordered in LDS
// (k_execute's dynamic LDS = CAP * 36 B), so CAP also sets k_execute's occupancy
constexpr uint32_t CAP_MIN = 64, CAP_MAX = 1024;
constexpr uint32_t LDS_BSLAB = 256;  // calendars with up to this many buckets keep their
                                     // bucket -> slab table in k_execute's LDS

}  // namespace sgn

struct sgn_ctx;
// A CPU worker thread's staging buffer for sgn_submit (sgn_stage_*).
struct sgn_stage {
  sgn_ctx* ctx = nullptr;
  mutable std::mutex mu;  // the worker thread's pushes against a concurrent sgn_stage_flush
  std::vector<uint32_t> src, dst, pay, wire;
  std::vector<uint64_t> time, handle;
};

// Host-side context.
struct sgn_ctx {
  int device = 0;
  uint32_t rank = 0, nranks = 1;
  uint32_t flags = 0;
  std::string err;
  hipStream_t stream = nullptr;

  // routing
  bool routes_ready = false;
  uint32_t U = 0;
  std::vector<uint32_t> used_ids;
  std::vector<uint64_t> h_lat;  // host copy of the table (CPU-side consumers)
  std::vector<float> h_loss;
  uint64_t lat_min = 0, lat_max = 0;  // over the U x U table (Runahead seed, calendar size)
  bool h_routes = false;               // h_lat / h_loss hold the table (ensure_host_routes)
  uint64_t* d_lat = nullptr;
  float* d_loss = nullptr;
  sgn_routes_timing rt_timing{};

  // hosts (all, HostId order)
  bool hosts_ready = false;
  uint32_t n_all = 0;
  std::vector<uint32_t> ip, node_id, unode;
  std::vector<uint64_t> bw_up, bw_down, seed;
  std::vector<uint32_t> dns_key, dns_val;
  uint32_t dns_mask = 0;
  uint32_t lo = 0, hi = 0;
  std::vector<uint32_t> sid_of;   // HostId -> slot id (sim_init; every shard's permutation)
  std::vector<uint32_t> host_of;  // this shard's slot -> HostId

  // simulation
  bool sim_ready = false;
  sgn::DevSim S{};
  void* d_S = nullptr;  // device copy of S (the execute kernel reads it through a pointer)
  std::vector<void*> allocs;
  uint64_t sim_bytes = 0;  // device bytes in allocs
  sgn::Ctrl* h_ctrl = nullptr;  // pinned mirror for reads
  uint64_t* h_mirror = nullptr; // the persistent kernel's copy of the control block (DevSim::ctrl_mirror)
  bool ctrl_fresh = false;      // h_ctrl is the device's control block (set by sgn_run; cleared by
                                // every call that may change it)
  uint64_t trace_cap = 0;
  uint64_t drain_cap = 0;                 // sgn_drain_enable (EXTERNAL traffic)
  std::vector<uint64_t> handles;          // sgn_submit handles by slot (tag & ~SGN_TAG_EXT)
  std::vector<uint32_t> submit_seq;       // per owned host: submissions so far
  std::vector<sgn_drain_rec> drain_held;  // drained from the device, not yet returned
  void* d_stage = nullptr;                // sgn_submit staging (device)
  std::vector<sgn_stage*> stages;         // sgn_stage_create order
  // CPU-side draws of host RNGs (sgn_rng_next_u64 / _double / _fill_bytes) between rounds: a
  // host's state is read once, stepped on the CPU, and written back (with its stream position)
  // before the next device operation that uses it (sgn::rng_release)
  struct RngHeld {
    uint64_t s[4];
    uint64_t draws;  // since it was read
  };
  std::unordered_map<uint32_t, RngHeld> rng_held;  // by slot
  void* d_rng_stage = nullptr;
  uint64_t rng_stage_cap = 0;
  std::mutex stage_mu;
  uint64_t stage_cap = 0;
  uint64_t rounds_enqueued = 0;

  // multi-GPU
  void* comm = nullptr;  // ncclComm_t
  bool comm_local = false;           // local shard group (sgn_comm_init_local)
  std::vector<sgn_ctx*> group;       // ... its contexts, shard order
  uint64_t xslot = 0;
  uint32_t xsz_cur = 0;    // runs per peer the current rounds' send/recv move (<= xslot)
  uint64_t x_spills = 0;   // rounds completed by a full-slot exchange
  uint64_t x_bytes = 0;    // bytes sent to peers by the round exchange (runs + messages)

  // kernel timing
  struct KT {
    const char* name;
    uint64_t launches = 0;   // timed (a sample of per-round launches)
    double ms = 0;
    uint64_t total = 0;      // every launch
  };
  KT kt[16];
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  std::vector<std::pair<int, size_t>> ev_pending;  // (kernel, pool index)
  size_t ev_next = 0;
  uint64_t t_seq = 0;  // per-round launches so far (a sample of them is timed)

  // a batch of rounds captured once as a hipGraph and replayed (single shard)
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  uint64_t gbatch = 0;
  uint32_t gsz = 0;        // multi-shard: the exchange size the captured batch sends
  std::vector<std::pair<int, size_t>> graph_timed;
  bool graph_pending = false;
  bool use_graph = true;
  uint32_t persist_grid = 0;  // persistent-rounds grid size (0: per-round launches)
  uint32_t persist_fallbacks = 0;  // persistent launches refused by the residency census
  uint32_t res_epoch = 0, res_base = 0;  // persistent launches so far / census arrivals so far
  bool persist_off = false;        // ... since sim_init: per-round launches from then on
  uint32_t lds_per_cu = 0;         // LDS bytes per CU (device attribute; the residency model)
  // pool growth (a held round, then a larger pool): counts for sgn_engine_info
  uint64_t codel_grows = 0, cal_grows = 0, cal_spill_runs = 0, xslot_grows = 0, rounds_held = 0;
  uint64_t ext_slabs = 0, spill_grows = 0;  // slabs with an extension; spill-area growths
  std::vector<uint64_t> h_ext;              // host mirror of DevSim::ext (empty: none)
  std::string failed;  // sticky: an operation left the device state unusable (every call fails)
  uint64_t codel_allocs_before = 0;  // page allocations before the last pool growth (its ring restarts)
  bool capturing = false;
  // persistent multi-shard rounds (k_rounds_x): this shard's inbox (uncached device memory:
  // peers write it over xGMI), its XPeer table, peer inboxes opened from IPC handles (one shard
  // per GPU), the launch descriptor, and the mode the rounds run in
  void* xin_mem = nullptr;
  size_t xin_bytes = 0;
  void* d_xp = nullptr;
  void* d_xl = nullptr;
  std::vector<void*> x_opened;
  std::vector<char*> x_base;   // every shard's inbox as this process addresses it (by rank)
  void* x_hxl = nullptr;       // pinned host copy of the launch descriptor
  bool x_mapped = false;       // the XPeer table points at every shard's current inbox
  bool x_off = false;          // the persistent path was refused (mapping / residency): per-round
  uint32_t x_mode = 0;         // 0 one shard, 1 per-round launches + exchange, 2 persistent rounds
  uint32_t x_grid = 0;         // this shard's workgroups in the last k_rounds_x launch
  uint32_t x_share = 1;        // shards on this GPU (one shard per GPU: 1)
  uint64_t x_epoch = 0, x_grows = 0, x_over_rounds = 0, x_moved = 0, x_launches = 0;
  std::vector<uint32_t> x_G;   // every shard's host groups (its bins' rows), by rank

  ~sgn_ctx();
};

namespace sgn {
int set_error(sgn_ctx* ctx, int code, const std::string& msg);
int hip_fail(sgn_ctx* ctx, hipError_t e, const char* what);
void* dev_alloc(sgn_ctx* ctx, size_t bytes, bool zero = true);
void dev_free(sgn_ctx* ctx, void* p, size_t bytes);
void free_sim(sgn_ctx* ctx);
void drop_graph(sgn_ctx* ctx);  // the captured batch of rounds, if any
// multi-shard exchange (comm.cpp): runs per peer the first RCCL rounds move; bytes one
// round sends to peers; completion of a held round with a full-slot exchange
constexpr uint32_t kXszInit = 512;
uint64_t comm_round_bytes(const sgn_ctx* ctx);
int comm_complete_spill(sgn_ctx* ctx);
int ensure_host_routes(sgn_ctx* ctx);
int rng_release(sgn_ctx* ctx);  // CPU-held host RNG states back to the device (stream-ordered)
// timing helpers around a launch
void time_begin(sgn_ctx* ctx, int kernel);
void time_end(sgn_ctx* ctx);
void time_collect(sgn_ctx* ctx);
// comm.cpp
void comm_destroy(sgn_ctx* ctx);
int comm_round_exchange(sgn_ctx* ctx);
int comm_bcast_blocks(sgn_ctx* ctx, void* base, size_t unit_bytes, const std::vector<uint64_t>& off);
int comm_allreduce_minmax(sgn_ctx* ctx, uint64_t* p, size_t n_min, size_t n_max);
int comm_allreduce_max_u32(sgn_ctx* ctx, uint32_t* p, size_t n);
// persistent multi-shard rounds (engine.hip: the launches; comm.cpp: the IPC mapping over RCCL)
struct XLay {
  size_t hdr, cen, runs, bins, bytes;
};
XLay xlay(uint32_t R, uint64_t xislot, uint32_t G, uint32_t xbk);
int xinbox_alloc(sgn_ctx* ctx, uint64_t xislot);
void xinbox_release(sgn_ctx* ctx);
int xpeer_upload(sgn_ctx* ctx);  // the XPeer table from ctx->x_base (and the RCCL send blocks)
bool xpersist_possible(sgn_ctx* ctx);
int run_xpersist(const std::vector<sgn_ctx*>& sh, bool peers, uint64_t max_rounds, uint64_t* rounds_done);
int comm_xpeer_map(sgn_ctx* ctx);       // one shard per GPU: map every peer's inbox (collective)
int comm_xmove_spills(sgn_ctx* ctx, const std::vector<std::vector<EvRec>>& out,
                      std::vector<EvRec>* in);  // runs past an inbox slot, to their shards (collective)
int comm_allreduce_max_u64(sgn_ctx* ctx, uint64_t* host_v, size_t n);  // (host values, collective)
int inject_runs(sgn_ctx* ctx, const std::vector<EvRec>& runs);      // engine.hip: into the calendar
}  // namespace sgn

// Every object of libsgn is compiled against this header. A library linked from objects built
// against different versions of it (an experiment build linking stale objects: the round-5
// segfault of libsgn_exp_rbrel.so) would read every struct at the wrong offsets.
// Each translation unit reports the layout it was compiled with and sgn_create refuses a
// mismatch (SGN_ESTATE) instead of running.
constexpr uint64_t kLayoutSig = (uint64_t)sizeof(sgn_ctx) * 1000003ull ^ (uint64_t)sizeof(sgn::DevSim) * 7919ull ^
                                (uint64_t)sizeof(sgn::Ctrl) * 131ull ^ (uint64_t)sizeof(sgn::HostRec) ^
                                ((uint64_t)sizeof(sgn::XLaunch) << 40) ^ ((uint64_t)sizeof(sgn::XPeer) << 48);
namespace sgn {
uint64_t layout_sig_api();
uint64_t layout_sig_engine();
uint64_t layout_sig_routes();
uint64_t layout_sig_comm();
}  // namespace sgn

#define SGN_HIP(ctx, call)                                   \
  do {                                                       \
    hipError_t e_ = (call);                                  \
    if (e_ != hipSuccess) return sgn::hip_fail(ctx, e_, #call); \
  } while (0)
