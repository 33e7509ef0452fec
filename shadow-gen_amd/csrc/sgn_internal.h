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

#include <string>
#include <vector>

#include "sgn.h"

namespace sgn {

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

// One entry of the synthetic socket send queue (a train of `count` datagrams).
struct __attribute__((aligned(16))) FifoEnt {
  uint32_t dst_ip;
  uint32_t pay;    // payload (low 16) | last payload (high 16)
  uint32_t count;
  uint32_t tag;
};
static_assert(sizeof(FifoEnt) == 16, "");

// Round control block, device resident. The window advances on the device.
struct Ctrl {
  uint64_t ws, we;        // current window [ws, we)
  uint32_t active;        // 0 once the controller returned None
  uint32_t overflow;      // bit flags (OVF_*); first offender in overflow_info
  uint64_t overflow_info;
  uint64_t round_min;     // atomicMin: next local event over owned hosts
  uint64_t min_used;      // Runahead::min_used_latency (atomicMin), INVALID = None
  uint32_t keep_slab;     // spare slab: receives the window's last bucket this round
  uint32_t pad0;
  uint64_t keep_min;      // min time placed in the spare slab this round
  uint64_t last_min_next; // min_next_event_time of the last finished round
  uint64_t rounds;
  uint64_t max_bucket;    // high-water mark of any (bucket, host group) slab fill
  uint64_t trace_n;       // trace records produced
  uint64_t remote_min;    // multi-GPU: min over events exported this round
  uint64_t exec_hosts;    // cumulative host executions (hosts with due events per round)
  uint64_t tot_runs;      // cumulative due event runs (records) handled
  uint64_t tot_sorted;    // cumulative host segments that needed ordering (>= 2 runs)
};

static_assert(offsetof(Ctrl, min_used) == offsetof(Ctrl, round_min) + 8,
              "comm.cpp all-reduces {round_min, min_used} as one u64[2]");

enum : uint32_t {
  OVF_BUCKET = 1u,
  OVF_CODEL = 2u,
  OVF_FIFO = 4u,
  OVF_SEG = 8u,
  OVF_EXCHANGE = 16u,
  OVF_TRACE = 32u,
};

// per-host counters (index * nH + host)
enum {
  CNT_SENT = 0,
  CNT_LOSS,
  CNT_UNKNOWN,
  CNT_POPPED,
  CNT_CODEL,
  CNT_DELIV,
  CNT_LOCAL_DELIV,
  CNT_BLOCKED,
  CNT_LOCAL_EV,
  CNT_BYTES,
  CNT_MAX_CODEL,
  NCNT
};

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
};

enum { SLOT_RO = 0, SLOT_RI = 1, SLOT_APP = 2, NSLOT = 3 };

// Everything the round kernels need, passed by value as a kernel argument.
struct DevSim {
  // shard and config
  uint32_t n_all, lo, nH, U;
  uint64_t end_time, boot_end, runahead_cfg;
  uint64_t min_possible;
  int32_t dynamic;
  uint32_t fifo_cap, codel_cap;
  uint32_t trace_on;
  // traffic
  uint32_t tkind, payload_len, unknown_permille, req_payload;
  uint32_t n_servers;
  uint32_t diag_mode;  // diagnostic build only (SGN_DIAG_MODE): 1 = light waves skip
  uint64_t flow_seed, period, period_jitter;
  uint64_t file_bytes[3];
  const uint32_t* servers;
  // routing (replicated on every shard)
  const uint64_t* rlat;
  const float* rloss;
  const uint32_t* unode;  // [n_all] used-node index of every host
  const uint32_t* ip;     // [n_all]
  const uint32_t* dns_key;
  const uint32_t* dns_val;
  uint32_t dns_mask;
  uint32_t pad1;
  // host state, SoA [nH] (slots/buckets: [k * nH + h])
  uint64_t *rng0, *rng1, *rng2, *rng3;
  uint64_t* eid;
  uint64_t* app_k;
  uint64_t* slot_t;
  uint64_t* slot_e;
  uint32_t* flags;
  uint32_t *ro_dst, *ro_pay, *ro_tag;
  uint32_t *ri_src, *ri_pay, *ri_tag;
  uint64_t* ri_eid;
  uint64_t *tb_bal, *tb_last, *tb_cap, *tb_inc;  // [2 * nH]: 0 = inet_out, 1 = inet_in
  CodelEnt* codel;       // [nH * codel_cap] run ring per host
  uint32_t *cq_head, *cq_nr, *cq_len;  // head run slot, runs, packets
  uint64_t *cq_bytes, *cq_ie, *cq_dn, *cq_cur, *cq_prev;
  FifoEnt* fifo;
  uint32_t *fq_head, *fq_len;
  uint64_t *d_tx, *d_rx, *d_app;
  uint64_t* cnt;
  uint64_t* trace_seq;
  // calendar: NB time buckets of width BW; every bucket is a set of slabs, one per host
  // group (GROUP consecutive hosts = one wave of k_execute), of CAP event runs each. Slab
  // ids are indirect (bucket_slab) so the partially consumed last bucket of a window can
  // swap with the spare slab set (Ctrl::keep_slab) instead of being copied.
  EvRec* pool;            // [(NB + 1) * G * CAP]
  uint32_t* slab_n;       // [(NB + 1) * G] fill of slab (s, g)
  uint32_t* bucket_slab;  // [NB] slab id of bucket b
  uint64_t* bucket_min;   // [NB] earliest event in bucket b (INVALID = empty)
  uint32_t NB, G;
  uint32_t CAP;
  uint32_t pad2;
  uint64_t BW;
  uint64_t* stamps;     // diagnostics (nullptr unless SGN_STAMPS is set)
  uint32_t n_ranks;
  Ctrl* ctrl;
  // trace
  sgn_trace_rec* trace;
  uint64_t trace_cap;
  // multi-GPU exchange: out slot r holds events for rank r
  EvRec* xout;
  uint32_t* xout_n;  // [n_ranks]
  EvRec* xin;
  uint32_t* xin_n;   // [n_ranks] (received counts)
  uint32_t xslot;    // events per slot
  uint32_t rank;
  const uint32_t* rank_lo;  // [n_ranks + 1] host ranges
};

constexpr uint32_t GROUP = 64;      // hosts per group = lanes of one k_execute wave
constexpr uint32_t CAP_MAX = 1024;  // event runs per (bucket, group) slab
constexpr uint32_t LDS_CAP = CAP_MAX;  // one bucket's runs of one group are ordered in LDS

}  // namespace sgn

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

  // simulation
  bool sim_ready = false;
  sgn::DevSim S{};
  std::vector<void*> allocs;
  sgn::Ctrl* h_ctrl = nullptr;  // pinned mirror for reads
  uint64_t trace_cap = 0;
  uint64_t rounds_enqueued = 0;

  // multi-GPU
  void* comm = nullptr;  // ncclComm_t
  uint64_t xslot = 0;

  // kernel timing
  struct KT {
    const char* name;
    uint64_t launches = 0;
    double ms = 0;
  };
  KT kt[16];
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  std::vector<std::pair<int, size_t>> ev_pending;  // (kernel, pool index)
  size_t ev_next = 0;

  // a batch of rounds captured once as a hipGraph and replayed (single shard)
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  uint64_t gbatch = 0;
  std::vector<std::pair<int, size_t>> graph_timed;
  bool graph_pending = false;
  bool use_graph = true;
  bool capturing = false;

  ~sgn_ctx();
};

namespace sgn {
int set_error(sgn_ctx* ctx, int code, const std::string& msg);
int hip_fail(sgn_ctx* ctx, hipError_t e, const char* what);
void* dev_alloc(sgn_ctx* ctx, size_t bytes, bool zero = true);
void free_sim(sgn_ctx* ctx);
// timing helpers around a launch
void time_begin(sgn_ctx* ctx, int kernel);
void time_end(sgn_ctx* ctx);
void time_collect(sgn_ctx* ctx);
// comm.cpp
void comm_destroy(sgn_ctx* ctx);
int comm_round_exchange(sgn_ctx* ctx);
}  // namespace sgn

#define SGN_HIP(ctx, call)                                   \
  do {                                                       \
    hipError_t e_ = (call);                                  \
    if (e_ != hipSuccess) return sgn::hip_fail(ctx, e_, #call); \
  } while (0)
