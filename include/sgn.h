/*
 * sgn.h — C ABI of libsgn, the MI355X-native packet-level network core for Shadow.
 *
 * libsgn replaces the data-parallel half of Shadow's simulation round (reference:
 * iiins0mn1a/shadow-gen, a Shadow 3.3.0 fork). Every entry point below names the
 * reference interface it replaces (file:line relative to the reference's src/main/ unless
 * stated). Conventions:
 *   - plain C types only, no torch/HIP types; caller owns every input array for the
 *     duration of the call, the library owns all device buffers;
 *   - every function returns int status: 0 = ok, negative = errno-style failure, with a
 *     message in sgn_last_error(ctx). Nothing unwinds or aborts across the ABI;
 *   - times are EmulatedTime nanoseconds (since the Unix epoch) unless a field says
 *     "_rel"/"_ns" (SimulationTime, nanoseconds since SIMULATION_START)
 *     (lib/shadow-shim-helper-rs/src/emulated_time.rs:25-50);
 *   - HostId is the u32 index of the host in hostname-sorted order (core/manager.rs:377-382).
 */
#ifndef SGN_H
#define SGN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGN_ABI_VERSION 10

/* emulated_time.rs:27-40 */
#define SGN_SIMULATION_START 946684800000000000ULL
#define SGN_EMUTIME_INVALID 0xFFFFFFFFFFFFFFFFULL
#define SGN_EMUTIME_MAX 0xFFFFFFFFFFFFFFFEULL

/* core/definitions.h:124 */
#define SGN_CONFIG_MTU 1500u
/* IPv4 header (network/packet.rs:477-484) + UDP header (network/packet.rs:737-740) */
#define SGN_UDP_HEADER_BYTES 28u
/* IPv4 + TCP header: 20 B, plus the 3-B window-scale option padded to 4 (packet.rs:617-635) */
#define SGN_TCP_HEADER_BYTES 40u
#define SGN_TCP_WS_HEADER_BYTES 44u

/* status codes */
#define SGN_OK 0
#define SGN_EINVAL (-22)
#define SGN_ENOMEM (-12)
#define SGN_ENOENT (-2)
#define SGN_ERANGE (-34)
#define SGN_EDEVICE (-5)    /* HIP runtime failure */
#define SGN_ESTATE (-71)    /* call out of order (e.g. round before sim_init) */
#define SGN_EOVERFLOW (-75) /* a device capacity was exceeded; message names which */

typedef struct sgn_ctx sgn_ctx;

/* ------------------------------------------------------------------------------------ */
/* Context                                                                              */
/* ------------------------------------------------------------------------------------ */

typedef struct sgn_create_opts {
  int32_t device;      /* HIP device ordinal */
  uint32_t shard_rank; /* this process's shard (0 for a single GPU) */
  uint32_t shard_count;/* number of shards (1 for a single GPU) */
  uint32_t flags;      /* SGN_CREATE_* */
} sgn_create_opts;

#define SGN_CREATE_TIME_KERNELS 1u /* HIP events around the engine's launches (a sample: sgn_kernel_times) */
#define SGN_CREATE_TIME_EXECUTE 2u /* ... around the per-host execute kernel only */

/* Creates a context bound to one GPU. Replaces WorkerShared construction
 * (core/manager.rs:447-470) for the data-parallel state. */
int sgn_create(sgn_ctx** out, const sgn_create_opts* opts);
void sgn_destroy(sgn_ctx* ctx);
/* Last error message for ctx (or for a failed sgn_create when ctx == NULL). */
const char* sgn_last_error(const sgn_ctx* ctx);
/* ABI version compiled into the library. */
int sgn_abi_version(void);

/* ------------------------------------------------------------------------------------ */
/* Routing (network/graph/mod.rs:181-250, core/sim_config.rs:411-448)                   */
/* ------------------------------------------------------------------------------------ */

/* A parsed network graph: what NetworkGraph::parse (network/graph/mod.rs:132-179) produces.
 * Node i (0-based) is petgraph NodeIndex i; edges keep GML order. Self-loops are edges. */
typedef struct sgn_graph {
  uint32_t n_nodes;
  const uint32_t* node_id;          /* [n_nodes] GML ids */
  uint32_t n_edges;
  const uint32_t* edge_src;         /* [n_edges] GML ids */
  const uint32_t* edge_dst;         /* [n_edges] GML ids */
  const uint64_t* edge_latency_ns;  /* [n_edges] > 0 (graph/mod.rs:103) */
  const float* edge_loss;           /* [n_edges] in [0,1] (graph/mod.rs:99) */
  int32_t directed;
} sgn_graph;

/* Builds the U x U routing table {latency u64 ns, packet_loss f32} between the used nodes.
 * Replaces generate_routing_info (core/sim_config.rs:411) ->
 * NetworkGraph::compute_shortest_paths (graph/mod.rs:181) when use_shortest_path != 0, or
 * get_direct_paths (graph/mod.rs:228) otherwise. Entry (i,j) is the path from
 * used_node_ids[i] to used_node_ids[j]; (i,i) is the node's single self-loop edge
 * (graph/mod.rs:209-215). Errors (not aborts): unknown node, missing/duplicate self-loop,
 * disconnected used pair, missing/duplicate direct edge. */
int sgn_routes_build(sgn_ctx* ctx, const sgn_graph* graph, const uint32_t* used_node_ids,
                     uint32_t n_used, int32_t use_shortest_path);
/* RoutingInfo::path (graph/mod.rs:442) by GML node ids. SGN_ENOENT if not a used pair. */
int sgn_route_get(sgn_ctx* ctx, uint32_t src_node_id, uint32_t dst_node_id,
                  uint64_t* latency_ns, float* packet_loss);
/* Copies the whole table (row-major, used-node order) to host arrays of n_used^2 entries. */
int sgn_routes_copy(sgn_ctx* ctx, uint64_t* latency_ns, float* packet_loss);
/* RoutingInfo::get_smallest_latency_ns (graph/mod.rs:472): min over all U^2 entries. */
int sgn_min_latency(sgn_ctx* ctx, uint64_t* latency_ns);
/* Device time of the last sgn_routes_build (ms), split into its phases. */
typedef struct sgn_routes_timing {
  double total_ms;      /* whole build incl. upload/extract, device-timed */
  double latency_ms;    /* blocked min-plus (Floyd-Warshall) phase */
  double loss_ms;       /* tight-edge loss fold phase */
  uint32_t loss_iters;  /* sweeps to the fixed point */
  uint32_t tile;        /* min-plus tile edge T */
  uint64_t n_tight_edges;
  uint32_t latency_passes; /* min-plus squaring passes (u32 form), k-blocks (u64 Floyd-Warshall),
                              or relaxation sweeps (latency_bf) */
  uint32_t latency_u64;    /* 1: the u64 Floyd-Warshall form ran (an edge or path >= 2^32 - 1 ns) */
  uint32_t loss_multi;     /* sources per tight-arc sweep (u32 form, non-sparse graphs); 0: the
                              one-source loss pass */
  uint32_t latency_bf;     /* 1: sparse graph, latencies by per-source relaxation (u64, exact);
                              latency_passes = its most sweeps */
  uint32_t shards;         /* blocks the build was split into: the shard count when a
                              communicator is set (sgn_comm_init before the build; every shard
                              computes its block of used sources and the blocks are exchanged
                              over RCCL, so every shard ends with the whole table), else 1 */
  uint32_t shard_sources;  /* used sources whose rows this process computed */
  uint32_t loss_dense;     /* ABI 10: 1 when the sweep ran in its dense form (at least half of all
                              arcs, no parallel arcs: a (tail, head) matrix of arcs, loss_multi
                              sources per workgroup); 0: the CSR / arc-list sweep or none */
  uint32_t loss_fused;     /* ABI 10: 1 when the dense sweep ran fused with the first squaring pass
                              and found the direct arcs already closed (complete graphs whose arcs
                              are their own shortest paths): the tight arcs were found inside the
                              latency phase (latency_ms), and loss_ms is the fold alone */
} sgn_routes_timing;
int sgn_routes_timing_get(sgn_ctx* ctx, sgn_routes_timing* out);

/* ------------------------------------------------------------------------------------ */
/* Hosts (core/sim_config.rs:47-164,211-291; host/host.rs:234,283-295)                  */
/* ------------------------------------------------------------------------------------ */

typedef struct sgn_hosts {
  uint32_t n_hosts;            /* hosts in HostId order */
  const uint32_t* ip;          /* [n] IPv4 address, host byte order */
  const uint32_t* node_id;     /* [n] GML node id (must be a used node of the route table) */
  const uint64_t* bw_up_bits;  /* [n] HostInfo::bandwidth_up_bits (note sim_config.rs:252-254) */
  const uint64_t* bw_down_bits;/* [n] HostInfo::bandwidth_down_bits */
  const uint64_t* seed;        /* [n] HostInfo::seed = r ^ SipHash13(name) (sim_config.rs:242) */
} sgn_hosts;

/* Registers every host of the simulation (all shards pass the full list; each shard
 * keeps the contiguous HostId range it owns). Replaces DNS registration
 * (network/dns.rs:97-131: unspecified/loopback/broadcast/multicast and duplicate
 * addresses are errors) and Host::new's RNG/relay construction. */
int sgn_hosts_set(sgn_ctx* ctx, const sgn_hosts* hosts);

/* Derives per-host seeds exactly as SimConfig::new + build_host do
 * (core/sim_config.rs:50-54,220-242): G = Xoshiro256++::seed_from_u64(sim_seed);
 * r = G.next_u64(); seed[i] = r ^ SipHash13_{k0=k1=0}(names[i] || 0xFF). Host-side only. */
int sgn_derive_host_seeds(uint32_t sim_seed, const char* const* names, uint32_t n,
                          uint64_t* seeds_out);

/* ------------------------------------------------------------------------------------ */
/* Simulation rounds (core/manager.rs:541-656, host/host.rs:762-834, core/worker.rs:330-403)*/
/* ------------------------------------------------------------------------------------ */

typedef struct sgn_sim_config {
  uint64_t stop_time_ns;        /* general.stop_time (controller.rs:29-31) */
  uint64_t bootstrap_end_ns;    /* general.bootstrap_end_time (manager.rs:353-355) */
  uint64_t runahead_ns;         /* experimental.runahead; 0 = None (runahead.rs:55) */
  int32_t use_dynamic_runahead; /* experimental.use_dynamic_runahead (runahead.rs:61-67) */
  uint32_t out_fifo_cap;        /* synthetic socket send-queue entries per host (>= 1) */
  uint32_t codel_cap;           /* device CoDel run slots per host ON AVERAGE (reference:
                                   unlimited): the queues are chains of 16-run pages from one
                                   pool of max(hosts + 64, hosts * codel_cap / 16) pages, so any
                                   host may hold far more; exhausting the pool is
                                   SGN_EOVERFLOW, never a silent drop */
  uint32_t hosts_per_wave;      /* hosts served by one 64-lane execute wave: a power of two
                                   in [1, 64]; 0 = default (64). Performance only. */
  uint64_t event_capacity;      /* in-flight packet-event slots per shard (0 = auto) */
  uint32_t interface_qdisc;     /* experimental.interface_qdisc (configuration.rs:448,568,972):
                                   SGN_QDISC_FIFO (default) or SGN_QDISC_ROUND_ROBIN */
  uint32_t reserved;
} sgn_sim_config;

/* The interface's send queue of sockets (host/network/interface.rs:94-106,216-256,
 * queuing.rs:57-180). Every synthetic send-queue entry (a datagram, or a train written to its
 * own socket) is one socket. FIFO: sockets by the priority of their next packet = packets in
 * the order the applications wrote them. ROUND_ROBIN: the interface takes one packet from the
 * socket at the front and re-queues that socket at the back while it has more. */
#define SGN_QDISC_FIFO 0u
#define SGN_QDISC_ROUND_ROBIN 1u

/* Synthetic traffic (stands in for the managed processes, which stay on the CPU in
 * Shadow). Hosts talk UDP through the reference's own relay/router path. Workload
 * functions are defined once in sgn_workload.h. */
#define SGN_TRAFFIC_PERIODIC 1u /* configs B/D: every host sends one datagram per period */
#define SGN_TRAFFIC_TGEN 2u     /* config C: clients fetch files from servers as MTU trains */
#define SGN_TRAFFIC_EXTERNAL 3u /* no synthetic app: every host's application lives on the CPU;
                                   its datagrams enter with sgn_submit and its deliveries and
                                   drops leave with sgn_drain (the mixed real-app mode) */

typedef struct sgn_traffic {
  uint32_t kind;
  uint32_t payload_len;          /* PERIODIC datagram payload bytes */
  uint64_t flow_seed;
  uint64_t start_ns;             /* first app event (sim time) */
  uint64_t start_jitter_ns;      /* + H(i) % (jitter + 1) */
  uint64_t period_ns;            /* PERIODIC send period / TGEN think time */
  uint64_t period_jitter_ns;     /* TGEN: think time + H % (jitter + 1) */
  uint32_t unknown_dst_permille; /* PERIODIC: sends to an address outside the simulation */
  uint32_t req_payload;          /* TGEN request datagram payload */
  uint32_t n_servers;            /* TGEN */
  uint32_t reserved0;
  const uint32_t* server_hosts;  /* TGEN [n_servers] HostIds of servers (ascending) */
  uint64_t file_bytes[3];        /* TGEN file sizes (e.g. 50 KiB, 1 MiB, 5 MiB) */
} sgn_traffic;

/* Uploads state and schedules each host's first app event. Must follow routes_build and
 * hosts_set. Host RNGs are Xoshiro256++::seed_from_u64(seed) (host/host.rs:234). */
int sgn_sim_init(sgn_ctx* ctx, const sgn_sim_config* cfg, const sgn_traffic* traffic);

/* The current window [start, end) (EmulatedTime). The first is
 * [SIMULATION_START, SIMULATION_START + 1 ns) (manager.rs:506-509). active = 0 once
 * Controller::manager_finished_current_round returned None (controller.rs:88-112). */
int sgn_window(sgn_ctx* ctx, uint64_t* start, uint64_t* end, int32_t* active);

/* Runs one round on the current window: every owned host executes its events with
 * time < end (Host::execute, host.rs:762-830), packets are routed (Worker::send_packet,
 * worker.rs:330-403), events are queued at their destinations (push_packet_to_host,
 * worker.rs:603-613), then min_next_event = min over all queue heads (manager.rs:580-628)
 * and the next window is computed on the device. Synchronous. */
int sgn_round(sgn_ctx* ctx, uint64_t* min_next_event);

/* Runs up to max_rounds rounds without a host synchronisation per round (rounds are
 * enqueued in batches; the window lives on the device). Stops early when the simulation
 * ends. rounds_done may be NULL. */
int sgn_run(sgn_ctx* ctx, uint64_t max_rounds, uint64_t* rounds_done);

/* Whole-simulation counters (summed over owned hosts). */
typedef struct sgn_stats {
  uint64_t rounds;
  uint64_t packets_sent;       /* send_packet executions that passed the DNS check */
  uint64_t packets_loss_dropped;/* ... of which dropped by path reliability (worker.rs:371) */
  uint64_t packets_unknown_dst;/* InetDropped: destination not in the simulation (:347) */
  uint64_t packet_events_popped;/* packet events executed at destinations (host.rs:797) */
  uint64_t codel_dropped;      /* RouterDropped by CoDel (codel_queue.rs:319) */
  uint64_t delivered;          /* inbound packets handed to the host interface */
  uint64_t local_delivered;    /* packets to the host's own address (relay is_local) */
  uint64_t app_blocked;        /* synthetic sends refused by a full send queue */
  uint64_t local_events;       /* local (task) events executed */
  uint64_t bytes_delivered;    /* payload bytes handed to the interface */
  uint64_t min_used_latency_ns;/* Runahead::min_used_latency, SGN_EMUTIME_INVALID if none */
  uint64_t max_codel_len;      /* high-water mark of any CoDel ring (capacity planning) */
  uint64_t max_pending_events; /* high-water mark of in-flight packet events */
  uint64_t host_executions;    /* sum over rounds of hosts that had an event due */
  uint64_t sched_heavy_hosts;  /* sum over rounds of hosts run on a wave of their own */
  uint64_t sched_sorted_segments; /* sum over rounds of per-host segments that needed sorting */
  uint64_t event_runs;         /* due event runs (records) processed; <= packet_events_popped */
} sgn_stats;
int sgn_stats_get(sgn_ctx* ctx, sgn_stats* out);

/* Per-host order-sensitive digests (sgn_workload.h: SGN_DIGEST_*), counters and final RNG
 * state for the owned range [host_lo, host_hi). Arrays hold (host_hi - host_lo) entries;
 * any pointer may be NULL. Used by parity tests at full sizes. */
typedef struct sgn_host_digest {
  uint64_t tx;        /* every send_packet outcome, in order */
  uint64_t rx;        /* every packet event popped, in order (event order proof) */
  uint64_t app;       /* every interface delivery / CoDel drop, in order */
  uint64_t rng[4];    /* Xoshiro256++ state */
  uint64_t next_event_id;
  uint64_t n_sent, n_popped, n_delivered, n_codel_dropped;
} sgn_host_digest;
int sgn_host_digests(sgn_ctx* ctx, uint32_t host_lo, uint32_t host_hi, sgn_host_digest* out);

/* Host::next_event_time (host.rs:832): backs worker_maxEventRunaheadTime (worker.rs:774).
 * SGN_EMUTIME_INVALID when the queue is empty. Only valid between rounds. */
int sgn_host_next_event_time(sgn_ctx* ctx, uint32_t host, uint64_t* t);
/* The same for every owned host in [host_lo, host_hi) at once (out[host - host_lo]): one
 * device pass over the host records and the calendar, one copy. A CPU controller reads its
 * hosts' worker_maxEventRunaheadTime inputs with one call per round, not one per host. */
int sgn_hosts_next_event_time(sgn_ctx* ctx, uint32_t host_lo, uint32_t host_hi, uint64_t* out);

/* Per-packet trace (for bit-exact comparison at small sizes). Enable before sim_init.
 * The record kinds follow a packet through the path:
 *   IF_POP   the interface hands a packet to relay_inet_out (NetworkInterface::pop,
 *            interface.rs:216-256 - the pcap capture point of a sent packet, interface.rs:192-215)
 *   SEND     Worker::send_packet's outcome (worker.rs:330-403)
 *   POP      the packet event runs at its destination (host.rs:762-830)
 *   DELIVER  the interface receives it (NetworkInterface::push - the receive capture point)
 *   LOCAL    a packet to the host's own address, pushed back into the interface (relay/mod.rs:84-87)
 *   CODEL_DROP the router's CoDel queue drops it (codel_queue.rs:319-321)
 * b of IF_POP / DELIVER / LOCAL = payload | tag << 32 (the header kind rides in the tag). */
#define SGN_TRACE_SEND 1u   /* a = now, b = deliver time (0 if dropped/unknown), c = event id */
#define SGN_TRACE_POP 2u    /* a = event time, b = 0, c = src event id */
#define SGN_TRACE_DELIVER 3u/* a = now, b = payload|tag<<32, c = src event id */
#define SGN_TRACE_CODEL_DROP 4u
#define SGN_TRACE_IF_POP 5u /* a = now, b = payload|tag<<32, c = dst address when peer is unknown */
#define SGN_TRACE_LOCAL 6u  /* a = now, b = payload|tag<<32 */
typedef struct sgn_trace_rec {
  uint32_t kind;     /* SGN_TRACE_* */
  uint32_t host;     /* host where it happened */
  uint32_t peer;     /* SEND / IF_POP: dst HostId (0xFFFFFFFF unknown); LOCAL: itself; others: src HostId */
  uint32_t flags;    /* SEND: 0 sent, 1 loss-dropped, 2 unknown dst */
  uint64_t a, b, c;
  uint64_t seq;      /* per-host sequence number of this record */
  uint64_t rng_pos;  /* the host RNG's stream position: draws made so far, this record's
                        loss draw included (host.rs:234; worker.rs:366 draws one per
                        send_packet past the DNS check; sgn_rng_* draws count too) */
} sgn_trace_rec;
int sgn_trace_enable(sgn_ctx* ctx, uint64_t capacity);
/* Copies up to cap records (unordered; sort by (host, seq)). n_total = records produced. */
int sgn_trace_read(sgn_ctx* ctx, sgn_trace_rec* out, uint64_t cap, uint64_t* n_total);

/* ------------------------------------------------------------------------------------ */
/* CPU-resident applications (SGN_TRAFFIC_EXTERNAL)                                      */
/* ------------------------------------------------------------------------------------ */

/* Packet ingress: datagrams written by CPU-side applications (the socket send that ends in
 * Host::notify_socket_has_packets, host.rs:969-983, and then relay_inet_out + Router::push +
 * Worker::send_packet, worker.rs:330). Each datagram is queued on the device as an event of
 * its source host at send_time; when the host reaches it (ordered with the host's packet
 * events at that time by (source = itself, submission order)), it enters the host's socket
 * send queue and the relay path takes it from there exactly like a synthetic app's datagram
 * (token bucket, loss draw from the device-held host RNG, source event id, delivery time).
 * Rules: traffic kind SGN_TRAFFIC_EXTERNAL; src_host owned by this shard; send_time in
 * [current window start, stop time) and within the event calendar's horizon (the
 * longest route latency ahead of the window); payload_len <= 65535; wire_len 0 or
 * payload_len + 28 (UDP over IPv4, packet.rs:388-396,477-484,737-740), or payload_len + 40 /
 * + 44 (a TCP segment from the CPU TCP stack without / with the window-scale option,
 * packet.rs:617-635; the wire length feeds the token buckets and CoDel's byte count, and a
 * zero-payload segment is never loss-dropped, worker.rs:371). handle is opaque
 * (the payload stays on the CPU) and comes back in the packet's drain record. Call between
 * rounds; a failed call queues nothing. Replaces Worker::send_packet's CPU callers. */
typedef struct sgn_pkt_soa {
  uint64_t n;
  const uint32_t* src_host;    /* [n] HostId */
  const uint32_t* dst_ip;      /* [n] IPv4, host byte order (unknown: InetDropped) */
  const uint32_t* payload_len; /* [n] UDP payload bytes */
  const uint32_t* wire_len;    /* [n] or NULL */
  const uint64_t* send_time;   /* [n] EmulatedTime */
  const uint64_t* handle;      /* [n] opaque, returned by sgn_drain (may be NULL: 0) */
} sgn_pkt_soa;
int sgn_submit(sgn_ctx* ctx, const sgn_pkt_soa* batch);

/* Per-thread staging: Shadow calls Worker::send_packet from every worker thread
 * at once (router/mod.rs:70-73, worker.rs:330). Each CPU worker thread owns one stage and
 * appends to it with sgn_stage_push — safe concurrently on DISTINCT stages, no device work;
 * the controller thread then submits every stage with one sgn_stage_flush between rounds.
 * A flush is exactly one sgn_submit of the stages' datagrams concatenated in stage-creation
 * order (each stage in push order); on failure nothing is queued and the stages keep their
 * datagrams. A push that runs while a flush runs is either part of that flush or stays
 * staged for the next one (a flush clears only what it copied). Create and destroy stages
 * only while no flush runs. */
typedef struct sgn_stage sgn_stage;
int sgn_stage_create(sgn_ctx* ctx, sgn_stage** out);
void sgn_stage_destroy(sgn_stage* stage);
/* Copies the batch into the stage (checks array presence and payload/wire sizes only; the
 * window and horizon rules are checked at flush). */
int sgn_stage_push(sgn_stage* stage, const sgn_pkt_soa* batch);
/* Datagrams waiting in a stage. */
uint64_t sgn_stage_pending(const sgn_stage* stage);
int sgn_stage_flush(sgn_ctx* ctx);

/* Packet egress: one record per datagram that left the network core, on the host where it
 * happened. Every submitted datagram yields exactly one record (delivered or dropped) once
 * its fate is decided; datagrams sent to EXTERNAL hosts are all submitted ones. */
#define SGN_DRAIN_DELIVERED 0u /* handed to the destination's interface (relay_inet_in) */
#define SGN_DRAIN_LOCAL 1u     /* to the host's own address (loopback, relay is_local) */
#define SGN_DRAIN_LOSS 2u      /* dropped by path reliability at send (worker.rs:366-371) */
#define SGN_DRAIN_UNKNOWN 3u   /* destination not in the simulation (InetDropped, :347) */
#define SGN_DRAIN_CODEL 4u     /* dropped by the destination router's CoDel (:319-321) */
#define SGN_DRAIN_BLOCKED 5u   /* the source's socket send queue was full */
typedef struct sgn_drain_rec {
  uint64_t time;        /* when it happened (EmulatedTime) */
  uint64_t src_eid;     /* source event id (DELIVERED / CODEL; 0 otherwise) */
  uint64_t handle;      /* sgn_submit handle (0 if submitted on another shard) */
  uint32_t host;        /* HostId where it happened */
  uint32_t src_host;    /* sender HostId */
  uint32_t dst_host;    /* destination HostId (0xFFFFFFFF unknown / not resolved) */
  uint32_t status;      /* SGN_DRAIN_* */
  uint32_t payload_len;
  uint32_t tag;         /* SGN_TAG_EXT | header kind << 29 | submission slot (sgn_workload.h) */
} sgn_drain_rec;
/* Device buffer for drain records between two sgn_drain calls (before sgn_sim_init;
 * default 1<<20 for EXTERNAL traffic). Running out is SGN_EOVERFLOW at the round. */
int sgn_drain_enable(sgn_ctx* ctx, uint64_t capacity);
/* Moves the records of hosts [host_lo, host_hi) out, ordered by (host, time, src_host,
 * src_eid, tag, status); records of other hosts stay for a later call. At most cap are
 * returned (*n_out); the rest stay. Between rounds only. */
int sgn_drain(sgn_ctx* ctx, uint32_t host_lo, uint32_t host_hi, sgn_drain_rec* out, uint64_t cap,
              uint64_t* n_out);

/* The next window, decided by a caller that also runs hosts of its own (Controller with CPU
 * hosts, controller.rs:88-112): [start, end) with previous window end <= start <= the
 * device's minimum next event time (sgn_window's start), start < end, end - start <= the
 * runahead the calendar was sized for, end clamped to the stop time. */
int sgn_set_window(sgn_ctx* ctx, uint64_t start, uint64_t end);

/* The host RNG, held on the device (the one authoritative copy): CPU-side draws
 * of host_rngDouble / host_rngNextNBytes (host/host.rs:1324-1336) and raw next_u64. They
 * advance the same Xoshiro256++ stream the loss draws use. Between rounds only. */
int sgn_rng_next_u64(sgn_ctx* ctx, uint32_t host, uint64_t* out);
/* counts[i] draws from each of n DISTINCT owned hosts in one device pass, concatenated in
 * order into out (sum(counts) entries): the batched form of sgn_rng_next_u64. */
int sgn_rng_next_u64_batch(sgn_ctx* ctx, const uint32_t* hosts, const uint32_t* counts, uint32_t n,
                           uint64_t* out);
/* rand 0.9 StandardUniform f64: (next_u64 >> 11) * 2^-53 */
int sgn_rng_double(sgn_ctx* ctx, uint32_t host, double* out);
/* rand_core 0.9 fill_bytes_via_next: little-endian next_u64 per 8 bytes; a tail of 5..7
 * bytes takes the low bytes of one more next_u64, a tail of 1..4 those of next_u32 (the
 * upper half of next_u64, rand_xoshiro 0.7). */
int sgn_rng_fill_bytes(sgn_ctx* ctx, uint32_t host, uint8_t* buf, size_t len);

/* Engine layout and execution mode chosen by sgn_sim_init (capacity planning, tests). */
typedef struct sgn_engine_info {
  uint64_t calendar_buckets;    /* NB: time buckets of the event calendar (a power of two) */
  uint64_t bucket_width_ns;     /* BW = max(min route latency, configured runahead) */
  uint64_t host_groups;         /* G: groups of hosts_per_wave consecutive hosts */
  uint64_t slab_capacity;       /* event runs per (bucket, group) slab */
  uint64_t hosts_per_wave;
  uint64_t persistent_grid;     /* workgroups of the persistent round kernel (0: per-round) */
  uint64_t persistent_fallbacks;/* persistent launches refused by the residency census */
  uint64_t device_bytes;        /* device memory held by the simulation */
  /* multi-shard round exchange (0 on one shard): per-peer slot capacity, runs per peer the
   * current rounds' send/recv move (sized from the high-water mark; a round that needs more
   * is held and completed with a full-slot exchange), the largest per-peer run count of any
   * round so far, rounds completed that way, and bytes sent to peers since sim_init */
  uint64_t exchange_slot_runs;
  uint64_t exchange_send_runs;
  uint64_t exchange_hwm_runs;
  uint64_t exchange_spills;
  uint64_t exchange_bytes;
  /* CoDel queues: pages of 16 runs in the shared pool (codel_cap slots per host on average,
   * at least one page per host), and pages taken from its free ring so far */
  uint64_t codel_pages;
  uint64_t codel_page_allocs;
  uint64_t codel_pages_free;     /* pages in the free ring now */
  uint64_t codel_pages_chained;  /* pages in the hosts' queue chains now (read from the host
                                    records: free + chained == codel_pages, no page lost) */
  uint64_t compute_units;        /* of this context's GPU */
  uint64_t bucket_min_lds;       /* 1: round kernels fold bucket minima in LDS first */
  /* ABI 7: device pools grow instead of refusing a scenario (the reference's queues are
   * unbounded, codel_queue.rs:33,303-317, event_queue.rs:57-66). A round that could need more
   * than a pool holds is held at its start (nothing of it has run), the pool grows between
   * launches, and the round runs. */
  uint64_t lds_per_cu;           /* LDS bytes per CU the residency model used (device attribute) */
  uint64_t codel_pool_grows;     /* CoDel page pool enlargements */
  uint64_t calendar_grows;       /* calendar re-layouts with larger slabs */
  uint64_t calendar_spill_runs;  /* runs that went to the calendar's spill area (then re-filed) */
  uint64_t exchange_slot_grows;  /* multi-shard exchange slot enlargements */
  uint64_t rounds_held;          /* rounds held at their start for a pool to grow */
  /* ABI 8: hot slabs. A (bucket, host group) slab past its capacity continues in an extension
   * (laid out at a held round edge); a slab holding more runs than one workgroup's LDS orders
   * at once is ordered and executed in pieces in Shadow's key order (event.rs:84-155), so no
   * fan-in is refused (the reference's EventQueue is an unbounded BinaryHeap,
   * core/work/event_queue.rs:12,57-66). */
  uint64_t slab_extensions;      /* slabs with an extension now */
  uint64_t slab_extension_runs;  /* runs the extensions hold in total */
  uint64_t big_slab_pieces;      /* pieces run by the big-slab path since sim_init */
  uint64_t spill_area_runs;      /* the spill area's capacity */
  uint64_t spill_area_grows;     /* spill area enlargements */
  /* ABI 9: persistent multi-shard rounds. With N > 1 shards the rounds run in one persistent
   * launch per GPU (or, for a local group on one GPU, one launch whose workgroup ranges are the
   * shards): runs for another shard go straight into that shard's inbox (peer-mapped memory),
   * and every shard computes the next window from the N round-edge messages in its inbox
   * (core/manager.rs:568-628, core/controller.rs:88-112). */
  uint64_t exchange_mode;        /* 0: one shard; 1: per-round launches + RCCL send/recv (or the
                                    local group's copies); 2: persistent rounds, peer inboxes */
  uint64_t inbox_slot_runs;      /* runs per sender and round parity in each inbox */
  uint64_t inbox_grows;          /* inbox enlargements (a round used more than half a slot) */
  uint64_t inbox_overflow_rounds;/* rounds whose runs past a slot the host moved */
  uint64_t inbox_moved_runs;     /* ... runs moved that way (into this shard) */
  uint64_t persistent_x_launches;/* persistent multi-shard launches */
  uint64_t persistent_x_grid;    /* this shard's workgroups in the last one */
} sgn_engine_info;
int sgn_engine_info_get(sgn_ctx* ctx, sgn_engine_info* out);

/* Device timing of the engine's kernels since sim_init (needs SGN_CREATE_TIME_KERNELS or
 * SGN_CREATE_TIME_EXECUTE). Persistent launches (k_rounds, many rounds each) are all timed;
 * per-round launches are timed one in eight (an event pair around every launch cost ~20 % of
 * the rounds), so launches[k] / ms[k] cover that sample: the average duration is
 * ms[k] / launches[k], and launches_total[k] counts every launch (timed or not) to scale
 * it to the total. */
typedef struct sgn_kernel_times {
  uint64_t launches[16];         /* timed launches */
  double ms[16];                 /* their summed duration */
  const char* name[16];
  uint32_t n_kernels;
  uint64_t launches_total[16];   /* every launch since sim_init (ABI 7) */
} sgn_kernel_times;
int sgn_kernel_times_get(sgn_ctx* ctx, sgn_kernel_times* out);

/* ------------------------------------------------------------------------------------ */
/* Multi-GPU shard exchange (round edge). Hosts are partitioned into contiguous HostId   */
/* ranges; events for remote hosts leave through per-peer slots and the window minimum */
/* is reduced across shards. The library drives RCCL itself on its own stream.         */
/* ------------------------------------------------------------------------------------ */

/* Size of the opaque RCCL unique id blob (ncclUniqueId). */
#define SGN_COMM_ID_BYTES 128
/* Rank 0 produces the id; the caller broadcasts it (e.g. torch.distributed) to all ranks. */
int sgn_comm_get_unique_id(uint8_t id_out[SGN_COMM_ID_BYTES]);
/* Creates the communicator over shard_count ranks; this ctx is rank shard_rank.
 * exchange_slot_events = capacity (events) of each per-peer slot per round. */
int sgn_comm_init(sgn_ctx* ctx, const uint8_t id[SGN_COMM_ID_BYTES],
                  uint64_t exchange_slot_events);
/* Local shard group: ctxs[i] is shard i of n (sgn_create with shard_count n) in THIS
 * process, on any devices (several may share one GPU). The round edge runs with device
 * copies instead of RCCL (host-synchronous per round): a test transport that exercises the
 * same device-side multi-shard path. Call before sgn_sim_init on every context; drive the
 * rounds with sgn_run_local_group (not sgn_run). */
int sgn_comm_init_local(sgn_ctx* const* ctxs, uint32_t n, uint64_t exchange_slot_events);
int sgn_run_local_group(sgn_ctx* const* ctxs, uint32_t n, uint64_t max_rounds,
                        uint64_t* rounds_done);
/* Owned HostId range of a shard (same split on every rank). */
int sgn_shard_range(uint32_t n_hosts, uint32_t shard_rank, uint32_t shard_count,
                    uint32_t* host_lo, uint32_t* host_hi);

/* ------------------------------------------------------------------------------------ */
/* CPU-side consumers (core/worker.rs:657-690, host/host.rs:1325-1336)                  */
/* ------------------------------------------------------------------------------------ */

/* worker_getLatency (worker.rs:657-667): addresses in NETWORK byte order; returns
 * SimulationTime ns or SGN_EMUTIME_INVALID (= SIMTIME_INVALID) if either is unknown. */
uint64_t sgn_worker_get_latency(sgn_ctx* ctx, uint32_t src_be, uint32_t dst_be);
/* worker_isRoutable (worker.rs:684-690). */
int32_t sgn_worker_is_routable(sgn_ctx* ctx, uint32_t src_be, uint32_t dst_be);
/* worker_getBandwidth{Up,Down}Bytes (worker.rs:670-681): bits / 8; 0 if unknown. */
uint64_t sgn_worker_get_bandwidth_up_bytes(sgn_ctx* ctx, uint32_t ip_be);
uint64_t sgn_worker_get_bandwidth_down_bytes(sgn_ctx* ctx, uint32_t ip_be);
/* Dns::addr_to_host_id (network/dns.rs:174): 0 and *host set, or SGN_ENOENT. */
int sgn_addr_to_host_id(sgn_ctx* ctx, uint32_t ip, uint32_t* host);

/* ------------------------------------------------------------------------------------ */
/* Front end (drop-in graph ingest): GML text -> sgn_graph (lib/gml-parser, graph/mod.rs)*/
/* ------------------------------------------------------------------------------------ */

typedef struct sgn_gml sgn_gml;
/* Parses GML text as gml_parser::parse + NetworkGraph::parse do (lib/gml-parser/src/
 * parser.rs:66-230, network/graph/mod.rs:28-179, units.rs:406-440). On failure returns
 * SGN_EINVAL and, if err/err_len given, a message. */
int sgn_gml_parse(const char* text, size_t len, sgn_gml** out, char* err, size_t err_len);
void sgn_gml_free(sgn_gml* g);
/* Borrowed view valid until sgn_gml_free. */
int sgn_gml_graph(const sgn_gml* g, sgn_graph* out);
/* Node bandwidths from host_bandwidth_up/_down (bits/s); has_* = 0 when absent. */
int sgn_gml_node_bandwidth(const sgn_gml* g, uint32_t node_index, uint64_t* up_bits,
                           int32_t* has_up, uint64_t* down_bits, int32_t* has_down);

/* assign_ips (core/sim_config.rs:386-407) over IpAssignment (network/graph/mod.rs:355-417),
 * hosts in HostId (= hostname) order. Hosts with explicit_ip[i] != 0 keep ips[i] (host byte
 * order) and are registered first; a repeated configured address is SGN_EINVAL with
 * *bad_host = the later host. Every other host gets the next address after the last one
 * handed out (from 11.0.0.0), skipping x.x.x.0, x.x.x.255 and configured addresses;
 * SGN_ERANGE past 255.255.255.254. Host-side only. */
int sgn_assign_ips(uint32_t n, const uint8_t* explicit_ip, uint32_t* ips, uint32_t* bad_host);

/* units.rs:406-440 FromStr + convert(): parse "10 ms" / "81920 Kibit" / "1 GiB".
 * kind: 0 Time -> ns, 1 Bytes -> bytes, 2 BitsPerSec -> bits/s. */
int sgn_units_parse(int32_t kind, const char* text, uint64_t* value_base);

/* ------------------------------------------------------------------------------------ */
/* Packet capture (utility/pcap_writer.rs, network/packet.rs:800-934, interface.rs:192-215)  */
/* ------------------------------------------------------------------------------------ */

typedef struct sgn_pcap sgn_pcap;
/* PcapWriter::new: a file with the libpcap global header (magic 0xA1B2C3D4, v2.4, zone 0,
 * sigfigs 0, snaplen = capture_len, link type 101 raw IP), native byte order. */
int sgn_pcap_open(const char* path, uint32_t capture_len, sgn_pcap** out);
/* PcapWriter::write_packet: record header {ts_sec, ts_usec, min(len, capture_len), len}
 * and the first min(len, capture_len) bytes. */
int sgn_pcap_write_packet(sgn_pcap* p, uint32_t ts_sec, uint32_t ts_usec, const uint8_t* bytes,
                          uint32_t len);
int sgn_pcap_close(sgn_pcap* p);
/* Packet::display_bytes for the path's packets: the IPv4 header (0x45, DSCP 0, total length,
 * id 0, DF, TTL 64, protocol, checksum 0, addresses), then a UDP header (ports, length,
 * checksum 0) or, by the tag's header kind, a TCP header (20 B, or 24 B with the window
 * scale option 3,3,ws + padding), then the payload. The synthetic applications have no
 * sockets: ports, TCP sequence/ack/flags/window and the payload bytes are 0. Returns the
 * packet length (header + payload) and writes min(that, cap) bytes. */
uint32_t sgn_packet_bytes(uint32_t src_ip, uint32_t dst_ip, uint32_t payload_len, uint32_t tag,
                          uint8_t* out, uint32_t cap);
/* One host's interface capture from trace records (any order; the host's records are taken
 * in seq order): every IF_POP record (send side) and every DELIVER and LOCAL record
 * (receive side) is one captured packet, stamped with the record's time as
 * to_abs_simtime (seconds saturated to u32, microseconds). host_ip[HostId] gives addresses;
 * an unknown peer's address is the record's c. Returns the number of packets written. */
int64_t sgn_trace_pcap(const sgn_trace_rec* recs, uint64_t n, uint32_t host, const uint32_t* host_ip,
                       uint32_t n_hosts, const char* path, uint32_t capture_len);

/* ------------------------------------------------------------------------------------ */
/* Test hooks (not part of the reference interface)                                      */
/* ------------------------------------------------------------------------------------ */

/* Device CoDel control-law increments round(1e8 / sqrt(count)) for count in [0, n)
 * (router/codel_queue.rs:285-298), for checking device f64 rounding against the host. */
int sgn_selftest_codel_law(sgn_ctx* ctx, uint64_t n, uint64_t* out);

/* Diagnostics of the last execute launch, SGN_STAMP_WORDS u64 per wave: {shader cycles,
 * events handled, max events of one host, hosts with events, then (diagnostic build
 * libsgn_diag.so only) lane 0's per-event-kind cycles and counts}. Needs SGN_STAMPS=1 in
 * the environment at sgn_sim_init; n = number of waves (0 when disabled), cap in waves. */
#define SGN_STAMP_WORDS 96
int sgn_debug_stamps(sgn_ctx* ctx, uint64_t* out, uint64_t cap, uint64_t* n);
/* Per-round timeline of the last persistent launch (SGN_STAMPS=1): 128 x {earliest round
 * start, latest arrival at the round barrier, round edge done} on the 100 MHz clock. */
int sgn_debug_rounds(sgn_ctx* ctx, uint64_t* out);
/* the persistent multi-shard kernel's per-round timeline (SGN_STAMPS=2): 8 words per round for 128
 * rounds — earliest start, latest local arrival, local barrier seen, messages sent, latest "all
 * messages seen", latest imports filed, latest second barrier seen (100 MHz clock); resets */
int sgn_debug_rounds_x(sgn_ctx* ctx, uint64_t* out);
/* the same per workgroup (SGN_STAMPS=3: plain stores, no shared words): [128 rounds][2048
 * workgroups of this shard][8] u64, the same 8 stamps (0: not written); resets */
int sgn_debug_rounds_xw(sgn_ctx* ctx, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* SGN_H */
