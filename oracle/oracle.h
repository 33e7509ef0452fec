/*
 * oracle.h — CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load the
 * oracle, and only as the checker (or the timed CPU baseline). libsgn never links it.
 *
 * Each function restates reference code (iiins0mn1a/shadow-gen, paths relative to src/):
 * see the file:line citations in oracle.cpp. Parity pinning:
 *   - APSP latencies, token bucket, CoDel, units, IP assignment: pinned by the reference's
 *     own unit tests (tests/golden/reference_unit_vectors.json);
 *   - Xoshiro256++/SplitMix64: pinned by rand_xoshiro 0.7.0's published test vectors;
 *     SipHash: pinned by the SipHash-2-4 reference vectors (same code path, c=2,d=4);
 *   - loss-fold values, host seeds, event order: parity unpinned (no reference-produced
 *     values exist; restated from the cited code).
 */
#ifndef SGN_ORACLE_H
#define SGN_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "sgn.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- RNG / hashing (rand_xoshiro 0.7.0, rand 0.9.2, core::hash::sip) ---- */
uint64_t ora_siphash(int c_rounds, int d_rounds, uint64_t k0, uint64_t k1, const uint8_t* msg,
                     size_t len);
void ora_xoshiro_seed_from_u64(uint64_t seed, uint64_t state_out[4]);
uint64_t ora_xoshiro_next_u64(uint64_t state[4]);
double ora_xoshiro_next_f64(uint64_t state[4]);
uint64_t ora_splitmix_next(uint64_t* state);
void ora_host_seeds(uint32_t sim_seed, const char* const* names, uint32_t n, uint64_t* out);

/* ---- units (utility/units.rs:406-440) ---- */
int ora_units_parse(int kind, const char* text, uint64_t* value_base);

/* ---- token bucket (network/relay/token_bucket.rs) and CoDel (router/codel_queue.rs)
 *      scripted for the reference's own unit tests ---- */
typedef struct ora_tb {
  uint64_t capacity, balance, refill_increment, refill_interval, last_refill;
} ora_tb;
int ora_tb_new(uint64_t capacity, uint64_t refill_increment, uint64_t refill_interval_ns,
               uint64_t last_refill, ora_tb* out);
/* returns 1 ok (balance_or_dur = new balance) or 0 err (balance_or_dur = conforming dur) */
int ora_tb_remove(ora_tb* tb, uint64_t decrement, uint64_t now, uint64_t* balance_or_dur);
uint64_t ora_codel_control_law(uint64_t time, uint64_t count);
typedef struct ora_codel ora_codel;
ora_codel* ora_codel_new(void);
void ora_codel_free(ora_codel* q);
void ora_codel_push(ora_codel* q, uint32_t wire_len, uint64_t now);
/* returns 1 and *wire_len if a packet is returned */
int ora_codel_pop(ora_codel* q, uint64_t now, uint32_t* wire_len);
int ora_codel_process_standing_delay(ora_codel* q, uint64_t now, uint64_t standing_delay);
typedef struct ora_codel_state {
  uint64_t len, total_bytes, mode, has_interval_end, interval_end, has_drop_next, drop_next,
      current_drop_count, previous_drop_count, dropped_total;
} ora_codel_state;
void ora_codel_get(const ora_codel* q, ora_codel_state* out);
void ora_codel_set_mode(ora_codel* q, int drop_mode);
int ora_codel_was_dropping_recently(const ora_codel* q, uint64_t now);
int ora_codel_should_drop(const ora_codel* q, uint64_t now);

/* ---- IP assignment (network/graph/mod.rs:348-418, core/sim_config.rs:386-407) ---- */
/* explicit[i] != 0 means host i has a configured address ips_inout[i]; others are
 * assigned sequentially. Returns 0 or SGN_EINVAL on a duplicate explicit address. */
int ora_assign_ips(uint32_t n, const uint8_t* explicit_flags, uint32_t* ips_inout);

/* ---- GML (lib/gml-parser, network/graph/mod.rs:28-179) ---- */
typedef struct ora_gml ora_gml;
int ora_gml_parse(const char* text, size_t len, ora_gml** out, char* err, size_t err_len);
void ora_gml_free(ora_gml* g);
int ora_gml_graph(const ora_gml* g, sgn_graph* out);
int ora_gml_node_bandwidth(const ora_gml* g, uint32_t node_index, uint64_t* up, int32_t* has_up,
                           uint64_t* down, int32_t* has_down);

/* ---- routing (network/graph/mod.rs:181-250,291-334,472) ---- */
int ora_routes(const sgn_graph* g, const uint32_t* used_node_ids, uint32_t n_used,
               int use_shortest_path, uint64_t* lat_out, float* loss_out, char* err,
               size_t err_len);

/* The same with the reference's data structures (faithful != 0: hash-map scores, the O(U)
 * contains filter, hashed U^2 output and re-collect) or dense arrays (0), on `threads` worker
 * threads (rayon over sources). Identical results. */
int ora_routes_mode(const sgn_graph* g, const uint32_t* used_node_ids, uint32_t n_used,
                    int use_shortest_path, int faithful, int threads, uint64_t* lat_out,
                    float* loss_out, char* err, size_t err_len);

/* ---- the round loop (core/manager.rs:541-656 and everything it calls) ---- */
typedef struct ora_sim ora_sim;
/* route table as produced by ora_routes for used_node_ids (U x U) */
int ora_sim_create(const uint32_t* used_node_ids, uint32_t n_used, const uint64_t* lat,
                   const float* loss, const sgn_hosts* hosts, const sgn_sim_config* cfg,
                   const sgn_traffic* traffic, int trace, ora_sim** out, char* err,
                   size_t err_len);
void ora_sim_free(ora_sim* s);
/* Worker threads of the round loop (a persistent pool, one rendezvous per round). */
int ora_sim_set_threads(ora_sim* s, int n);
/* Reference-faithful per-packet data structures (1) or the CPU-optimised ones (0). */
int ora_sim_set_faithful(ora_sim* s, int on);
int ora_sim_window(const ora_sim* s, uint64_t* start, uint64_t* end, int32_t* active);
int ora_sim_round(ora_sim* s, uint64_t* min_next);
int ora_sim_run(ora_sim* s, uint64_t max_rounds, uint64_t* rounds_done);
int ora_sim_stats(const ora_sim* s, sgn_stats* out);
int ora_sim_host_digests(const ora_sim* s, uint32_t lo, uint32_t hi, sgn_host_digest* out);
uint64_t ora_sim_trace_count(const ora_sim* s);
uint64_t ora_sim_trace_read(const ora_sim* s, sgn_trace_rec* out, uint64_t cap);
int ora_sim_host_next_event_time(const ora_sim* s, uint32_t host, uint64_t* t);
/* CPU-resident applications (SGN_TRAFFIC_EXTERNAL): same contract as libsgn's sgn_submit,
 * sgn_drain (handles resolved from this oracle's own submissions) and sgn_set_window. */
int ora_sim_submit(ora_sim* s, const sgn_pkt_soa* batch);
int ora_sim_drain(ora_sim* s, uint32_t lo, uint32_t hi, sgn_drain_rec* out, uint64_t cap,
                  uint64_t* n_out);
int ora_sim_set_window(ora_sim* s, uint64_t start, uint64_t end);
/* The host RNG (host/host.rs:1324-1336); same contract as sgn_rng_*. */
int ora_sim_rng_next_u64(ora_sim* s, uint32_t host, uint64_t* out);
int ora_sim_rng_double(ora_sim* s, uint32_t host, double* out);
int ora_sim_rng_fill_bytes(ora_sim* s, uint32_t host, uint8_t* buf, size_t len);
/* Sharded mode (round-edge protocol rehearsal, tests only): restrict execution to
 * [lo,hi); packet events for other hosts are exported instead of queued. */
int ora_sim_set_shard(ora_sim* s, uint32_t lo, uint32_t hi);
/* Executes the round's hosts only (no window advance). Returns exported event count. */
int ora_sim_shard_execute(ora_sim* s, uint64_t* n_exported);
/* Exported records since the last execute: 6 u64 per event
 * (dst, time, src, eid, payload, tag). */
uint64_t ora_sim_shard_take_exports(ora_sim* s, uint64_t* out, uint64_t cap);
int ora_sim_shard_import(ora_sim* s, const uint64_t* recs, uint64_t n);
/* Local min over owned queue heads and local min used latency (or INVALID). */
int ora_sim_shard_local_min(const ora_sim* s, uint64_t* min_next, uint64_t* min_used_lat);
/* Advances the window from the global minimum (Controller, controller.rs:88-112). */
int ora_sim_shard_advance(ora_sim* s, uint64_t global_min_next, uint64_t global_min_used_lat);

#ifdef __cplusplus
}
#endif
#endif
