/*
 * sgn_workload.h — the synthetic workload and digest definitions shared by every
 * implementation of the packet core (the HIP engine and the parity oracle).
 *
 * These are NOT reference semantics: they define the synthetic applications that stand
 * in for Shadow's managed processes (which stay on the CPU per the north star) and the
 * order-sensitive digests used to compare runs. Reference semantics (routing, RNG draws,
 * event order, relays, token buckets, CoDel, runahead) are implemented separately by each
 * side. Pure functions of integers; no state.
 */
#ifndef SGN_WORKLOAD_H
#define SGN_WORKLOAD_H

#include <stdint.h>

#if defined(__HIPCC__)
#define SGN_HD __host__ __device__ __forceinline__
#else
#define SGN_HD static inline
#endif

/* SplitMix64 finalizer (also the SplitMix64 output function). */
SGN_HD uint64_t sgn_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

/* Workload hash H(seed, a, b): independent streams per (host, counter). */
SGN_HD uint64_t sgn_flow_hash(uint64_t seed, uint64_t a, uint64_t b) {
  return sgn_mix64(sgn_mix64(seed ^ (0x9e3779b97f4a7c15ULL * (a + 1))) ^
                   (0xd1b54a32d192ed03ULL * (b + 1)));
}

#define SGN_SALT_START 0xFFFFFFFF00000001ULL
#define SGN_SALT_THINK 0xFFFFFFFF00000002ULL

/* Address space for sends to destinations outside the simulation (never assigned:
 * automatic IPs start at 11.0.0.1, graph/mod.rs:359-417; the library rejects explicit
 * host addresses inside 10.255.0.0/16). */
#define SGN_UNKNOWN_IP_BASE 0x0AFF0000u /* 10.255.0.0 */

/* First app event of host i. */
SGN_HD uint64_t sgn_app_start_rel(uint64_t flow_seed, uint32_t host, uint64_t start_ns,
                                  uint64_t jitter_ns) {
  uint64_t j = jitter_ns ? sgn_flow_hash(flow_seed, host, SGN_SALT_START) % (jitter_ns + 1) : 0;
  return start_ns + j;
}

/* PERIODIC: destination of the k-th datagram of host i.
 * Returns 1 and *peer_host when addressed to a host, 0 and *unknown_ip otherwise. */
SGN_HD int sgn_periodic_dst(uint64_t flow_seed, uint32_t host, uint64_t k, uint32_t n_hosts,
                            uint32_t unknown_permille, uint32_t* peer_host,
                            uint32_t* unknown_ip) {
  uint64_t r = sgn_flow_hash(flow_seed, host, k);
  if ((uint32_t)(r % 1000u) < unknown_permille) {
    *unknown_ip = SGN_UNKNOWN_IP_BASE + (uint32_t)((r >> 32) & 0xFFFFu);
    return 0;
  }
  *peer_host = (uint32_t)((r >> 16) % (uint64_t)n_hosts);
  return 1;
}

/* TGEN: the k-th fetch of client i: server index into server_hosts and file size class. */
SGN_HD void sgn_tgen_fetch(uint64_t flow_seed, uint32_t host, uint64_t k, uint32_t n_servers,
                           uint32_t* server_idx, uint32_t* size_class) {
  uint64_t r = sgn_flow_hash(flow_seed, host, k);
  *server_idx = (uint32_t)((r >> 8) % (uint64_t)n_servers);
  *size_class = (uint32_t)((r >> 40) % 3u);
}

/* TGEN: think time after the k-th fetch of client i. */
SGN_HD uint64_t sgn_tgen_think(uint64_t flow_seed, uint32_t host, uint64_t k, uint64_t think_ns,
                               uint64_t jitter_ns) {
  uint64_t j = jitter_ns ? sgn_flow_hash(flow_seed ^ SGN_SALT_THINK, host, k) % (jitter_ns + 1)
                         : 0;
  return think_ns + j;
}

/* UDP payload per full datagram of a TGEN response train (1500 B on the wire). */
#define SGN_TGEN_MSS 1472u /* 1500 - 20 (IPv4) - 8 (UDP) */

/* Packet tags (carried opaque through the core; the synthetic apps interpret them). */
#define SGN_TAG_DATA 0u        /* PERIODIC datagram */
#define SGN_TAG_REQ 0x10000u   /* TGEN request | size class */
#define SGN_TAG_RESP 0x20000u  /* TGEN response datagram */
#define SGN_TAG_EXT 0x80000000u /* EXTERNAL datagram: low 29 bits = sgn_submit slot */
#define SGN_TAG_SLOT_MASK 0x1FFFFFFFu
/* Header kind of a packet (tag bits 29-30): its wire length is payload + this many bytes
 * (network/packet.rs:388-396: IPv4 20 + UDP 8, or + TCP 20 / 24 with window scale). */
#define SGN_TAG_HDR_SHIFT 29
#define SGN_TAG_HDR_TCP (1u << SGN_TAG_HDR_SHIFT)
#define SGN_TAG_HDR_TCPWS (2u << SGN_TAG_HDR_SHIFT)
SGN_HD uint32_t sgn_header_bytes(uint32_t tag) {
  const uint32_t k = (tag >> SGN_TAG_HDR_SHIFT) & 3u;
  return k == 0 ? 28u : (k == 1 ? 40u : 44u);
}

/* Order-sensitive per-host digest step: each word is xored in and followed by a
 * bijective multiply / xorshift, so any change of value or order changes the result
 * (with overwhelming probability). Three multiplies: cheap on the per-event hot path. */
SGN_HD uint64_t sgn_digest3(uint64_t h, uint64_t a, uint64_t b, uint64_t c) {
  h = (h ^ a) * 0x9e3779b97f4a7c15ULL;
  h = (h ^ (h >> 32) ^ b) * 0xd1b54a32d192ed03ULL;
  h = (h ^ (h >> 29) ^ c) * 0xbf58476d1ce4e5b9ULL;
  return h ^ (h >> 32);
}

/* Run-encoded digests. Each digest is taken over the host's records in order, but a maximal
 * run of records that differ only by a counter is folded in as ONE step (a bijective
 * re-encoding of the same sequence: any change of a value, of the order or of a run length
 * still changes the digest w.h.p.), so a train of n packets costs O(1) digest work:
 *  tx : per send_packet call past the is_completed check, record (now, dst_host |
 *       outcome << 32, deliver_time_or_0); outcome 0 sent / 1 loss-dropped / 2 unknown
 *       destination (dst_host = 0xFFFFFFFF). A run = n identical records:
 *       digest3(h, now, dst | outcome << 32 | n << 34, deliver_or_0).
 *  rx : per packet event popped, (event_time, src_host, src_event_id). A run = n records
 *       with the same time and source and consecutive ids e0, e0+1, ...:
 *       digest3(h, time, src | n << 32, e0).
 *  app: per interface delivery (now, src_host, src_event_id) and per CoDel drop
 *       (now, src_host | 1<<63, src_event_id), runs as for rx (n in bits 32..61); a local
 *       (loopback) delivery is a run of its own: digest3(h, now, src | 1<<62 | 1<<32,
 *       payload).
 * Runs never span two values of `now`; every implementation flushes its pending runs at
 * least whenever `now` changes and at the end of each Host::execute.                     */
typedef struct sgn_drun {
  uint64_t a, b, c; /* run key (a, b) and c = next id (seq runs) or the common value */
  uint32_t n;       /* records in the pending run (0 = none) */
} sgn_drun;

SGN_HD void sgn_drun_flush_seq(uint64_t* h, sgn_drun* r) {
  if (r->n) *h = sgn_digest3(*h, r->a, r->b | ((uint64_t)r->n << 32), r->c - r->n);
  r->n = 0;
}
SGN_HD void sgn_drun_flush_same(uint64_t* h, sgn_drun* r) {
  if (r->n) *h = sgn_digest3(*h, r->a, r->b | ((uint64_t)r->n << 34), r->c);
  r->n = 0;
}
/* n records (a, b, c0), (a, b, c0+1), ... (rx, app) */
SGN_HD void sgn_drun_add_seq(uint64_t* h, sgn_drun* r, uint64_t a, uint64_t b, uint64_t c0,
                             uint32_t n) {
  if (r->n && r->a == a && r->b == b && r->c == c0) {
    r->n += n;
    r->c += n;
    return;
  }
  sgn_drun_flush_seq(h, r);
  r->a = a;
  r->b = b;
  r->c = c0 + n;
  r->n = n;
}
/* n identical records (a, b, c) (tx) */
SGN_HD void sgn_drun_add_same(uint64_t* h, sgn_drun* r, uint64_t a, uint64_t b, uint64_t c,
                              uint32_t n) {
  if (r->n && r->a == a && r->b == b && r->c == c) {
    r->n += n;
    return;
  }
  sgn_drun_flush_same(h, r);
  r->a = a;
  r->b = b;
  r->c = c;
  r->n = n;
}
#define SGN_DIGEST_SEED 0x5eed5eed5eed5eedULL

#endif /* SGN_WORKLOAD_H */
