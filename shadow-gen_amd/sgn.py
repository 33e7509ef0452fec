"""ctypes binding of libsgn (include/sgn.h) plus the synthetic-workload generators.

This module is host-side plumbing for tests and bench.py: every computation of the packet
core happens inside libsgn.so on the GPU. Loading fails loudly if the library is missing;
there is no CPU fallback anywhere in this package.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
# SGN_LIB overrides the library file (diagnostic builds such as libsgn_diag.so)
LIB_PATH = pathlib.Path(os.environ["SGN_LIB"]) if os.environ.get("SGN_LIB") else HERE / "libsgn.so"

SIMULATION_START = 946684800 * 1_000_000_000
EMUTIME_INVALID = 0xFFFFFFFFFFFFFFFF
EMUTIME_MAX = 0xFFFFFFFFFFFFFFFE
TRAFFIC_PERIODIC = 1
TRAFFIC_TGEN = 2
TRAFFIC_EXTERNAL = 3  # CPU-resident apps: sgn_submit / sgn_drain
QDISC_FIFO, QDISC_ROUND_ROBIN = 0, 1
TAG_EXT = 0x80000000
DRAIN_DELIVERED, DRAIN_LOCAL, DRAIN_LOSS, DRAIN_UNKNOWN, DRAIN_CODEL, DRAIN_BLOCKED = range(6)
STAMP_WORDS = 96  # include/sgn.h SGN_STAMP_WORDS
CREATE_TIME_KERNELS = 1

u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
f32p = C.POINTER(C.c_float)


class Graph(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint32),
        ("node_id", u32p),
        ("n_edges", C.c_uint32),
        ("edge_src", u32p),
        ("edge_dst", u32p),
        ("edge_latency_ns", u64p),
        ("edge_loss", f32p),
        ("directed", C.c_int32),
    ]


class Hosts(C.Structure):
    _fields_ = [
        ("n_hosts", C.c_uint32),
        ("ip", u32p),
        ("node_id", u32p),
        ("bw_up_bits", u64p),
        ("bw_down_bits", u64p),
        ("seed", u64p),
    ]


class SimConfig(C.Structure):
    _fields_ = [
        ("stop_time_ns", C.c_uint64),
        ("bootstrap_end_ns", C.c_uint64),
        ("runahead_ns", C.c_uint64),
        ("use_dynamic_runahead", C.c_int32),
        ("out_fifo_cap", C.c_uint32),
        ("codel_cap", C.c_uint32),
        ("hosts_per_wave", C.c_uint32),
        ("event_capacity", C.c_uint64),
        ("interface_qdisc", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class Traffic(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32),
        ("payload_len", C.c_uint32),
        ("flow_seed", C.c_uint64),
        ("start_ns", C.c_uint64),
        ("start_jitter_ns", C.c_uint64),
        ("period_ns", C.c_uint64),
        ("period_jitter_ns", C.c_uint64),
        ("unknown_dst_permille", C.c_uint32),
        ("req_payload", C.c_uint32),
        ("n_servers", C.c_uint32),
        ("reserved0", C.c_uint32),
        ("server_hosts", u32p),
        ("file_bytes", C.c_uint64 * 3),
    ]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "rounds", "packets_sent", "packets_loss_dropped", "packets_unknown_dst",
        "packet_events_popped", "codel_dropped", "delivered", "local_delivered",
        "app_blocked", "local_events", "bytes_delivered", "min_used_latency_ns",
        "max_codel_len", "max_pending_events", "host_executions",
        "sched_heavy_hosts", "sched_sorted_segments", "event_runs")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class HostDigest(C.Structure):
    _fields_ = [
        ("tx", C.c_uint64), ("rx", C.c_uint64), ("app", C.c_uint64),
        ("rng", C.c_uint64 * 4), ("next_event_id", C.c_uint64),
        ("n_sent", C.c_uint64), ("n_popped", C.c_uint64), ("n_delivered", C.c_uint64),
        ("n_codel_dropped", C.c_uint64),
    ]


class TraceRec(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32), ("host", C.c_uint32), ("peer", C.c_uint32), ("flags", C.c_uint32),
        ("a", C.c_uint64), ("b", C.c_uint64), ("c", C.c_uint64), ("seq", C.c_uint64),
        ("rng_pos", C.c_uint64),
    ]


TRACE_DTYPE = np.dtype([("kind", "<u4"), ("host", "<u4"), ("peer", "<u4"), ("flags", "<u4"),
                        ("a", "<u8"), ("b", "<u8"), ("c", "<u8"), ("seq", "<u8"), ("rng_pos", "<u8")])
TRACE_SEND, TRACE_POP, TRACE_DELIVER, TRACE_CODEL_DROP, TRACE_IF_POP, TRACE_LOCAL = 1, 2, 3, 4, 5, 6
DIGEST_DTYPE = np.dtype([("tx", "<u8"), ("rx", "<u8"), ("app", "<u8"), ("rng", "<u8", (4,)),
                         ("next_event_id", "<u8"), ("n_sent", "<u8"), ("n_popped", "<u8"),
                         ("n_delivered", "<u8"), ("n_codel_dropped", "<u8")])


class PktSoa(C.Structure):
    _fields_ = [("n", C.c_uint64), ("src_host", u32p), ("dst_ip", u32p), ("payload_len", u32p),
                ("wire_len", u32p), ("send_time", u64p), ("handle", u64p)]


class DrainRec(C.Structure):
    _fields_ = [("time", C.c_uint64), ("src_eid", C.c_uint64), ("handle", C.c_uint64),
                ("host", C.c_uint32), ("src_host", C.c_uint32), ("dst_host", C.c_uint32),
                ("status", C.c_uint32), ("payload_len", C.c_uint32), ("tag", C.c_uint32)]


DRAIN_DTYPE = np.dtype([("time", "<u8"), ("src_eid", "<u8"), ("handle", "<u8"), ("host", "<u4"),
                        ("src_host", "<u4"), ("dst_host", "<u4"), ("status", "<u4"),
                        ("payload_len", "<u4"), ("tag", "<u4")])
assert DRAIN_DTYPE.itemsize == C.sizeof(DrainRec)


def pkt_soa(src_host, dst_ip, payload_len, send_time, handle=None, wire_len=None):
    """(PktSoa, keep-alive arrays) for sgn_submit / ora_sim_submit."""
    a = [np.ascontiguousarray(src_host, dtype=np.uint32), np.ascontiguousarray(dst_ip, dtype=np.uint32),
         np.ascontiguousarray(payload_len, dtype=np.uint32), np.ascontiguousarray(send_time, dtype=np.uint64)]
    h = None if handle is None else np.ascontiguousarray(handle, dtype=np.uint64)
    w = None if wire_len is None else np.ascontiguousarray(wire_len, dtype=np.uint32)
    b = PktSoa(len(a[0]), ptr(a[0], C.c_uint32), ptr(a[1], C.c_uint32), ptr(a[2], C.c_uint32),
               ptr(w, C.c_uint32) if w is not None else None, ptr(a[3], C.c_uint64),
               ptr(h, C.c_uint64) if h is not None else None)
    return b, (a, h, w)
assert TRACE_DTYPE.itemsize == C.sizeof(TraceRec)
assert DIGEST_DTYPE.itemsize == C.sizeof(HostDigest)


class CreateOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("shard_rank", C.c_uint32),
                ("shard_count", C.c_uint32), ("flags", C.c_uint32)]


class RoutesTiming(C.Structure):
    _fields_ = [("total_ms", C.c_double), ("latency_ms", C.c_double), ("loss_ms", C.c_double),
                ("loss_iters", C.c_uint32), ("tile", C.c_uint32), ("n_tight_edges", C.c_uint64),
                ("latency_passes", C.c_uint32), ("latency_u64", C.c_uint32),
                ("loss_multi", C.c_uint32), ("latency_bf", C.c_uint32),
                ("shards", C.c_uint32), ("shard_sources", C.c_uint32),
                ("loss_dense", C.c_uint32), ("loss_fused", C.c_uint32)]


class EngineInfo(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "calendar_buckets", "bucket_width_ns", "host_groups", "slab_capacity", "hosts_per_wave",
        "persistent_grid", "persistent_fallbacks", "device_bytes", "exchange_slot_runs",
        "exchange_send_runs", "exchange_hwm_runs", "exchange_spills", "exchange_bytes", "codel_pages",
        "codel_page_allocs", "codel_pages_free", "codel_pages_chained",
        "compute_units", "bucket_min_lds", "lds_per_cu", "codel_pool_grows", "calendar_grows",
        "calendar_spill_runs", "exchange_slot_grows", "rounds_held", "slab_extensions",
        "slab_extension_runs", "big_slab_pieces", "spill_area_runs", "spill_area_grows",
        "exchange_mode", "inbox_slot_runs", "inbox_grows", "inbox_overflow_rounds", "inbox_moved_runs",
        "persistent_x_launches", "persistent_x_grid")]


class KernelTimes(C.Structure):
    _fields_ = [("launches", C.c_uint64 * 16), ("ms", C.c_double * 16),
                ("name", C.c_char_p * 16), ("n_kernels", C.c_uint32),
                ("launches_total", C.c_uint64 * 16)]


_lib = None


def build_id() -> str:
    """A fingerprint of the libsgn sources the shipped libsgn.so is built from (csrc/ and the
    public headers): measurements filed under profiles/ carry it, and bench.py quotes a
    measurement only for the build it was taken on."""
    import hashlib
    here = pathlib.Path(__file__).resolve().parent
    files = sorted(list((here / "csrc").glob("*.hip")) + list((here / "csrc").glob("*.cpp")) +
                   list((here / "csrc").glob("*.h")) + [here / "csrc" / "Makefile"] +
                   list((here.parent / "include").glob("*.h")))
    h = hashlib.sha256()
    for f in files:
        h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()[:16]


def load(path: str | os.PathLike | None = None) -> C.CDLL:
    """Load libsgn.so (raises if it was not built: the product has no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = pathlib.Path(path) if path else LIB_PATH
    if not p.exists():
        raise RuntimeError(f"libsgn not built: {p} missing (run __graft_entry__.build())")
    L = C.CDLL(str(p))
    vp = C.c_void_p
    sig = {
        "sgn_create": (C.c_int, [C.POINTER(vp), C.POINTER(CreateOpts)]),
        "sgn_destroy": (None, [vp]),
        "sgn_last_error": (C.c_char_p, [vp]),
        "sgn_abi_version": (C.c_int, []),
        "sgn_routes_build": (C.c_int, [vp, C.POINTER(Graph), u32p, C.c_uint32, C.c_int32]),
        "sgn_route_get": (C.c_int, [vp, C.c_uint32, C.c_uint32, u64p, f32p]),
        "sgn_routes_copy": (C.c_int, [vp, u64p, f32p]),
        "sgn_min_latency": (C.c_int, [vp, u64p]),
        "sgn_routes_timing_get": (C.c_int, [vp, C.POINTER(RoutesTiming)]),
        "sgn_hosts_set": (C.c_int, [vp, C.POINTER(Hosts)]),
        "sgn_derive_host_seeds": (C.c_int, [C.c_uint32, C.POINTER(C.c_char_p), C.c_uint32, u64p]),
        "sgn_sim_init": (C.c_int, [vp, C.POINTER(SimConfig), C.POINTER(Traffic)]),
        "sgn_window": (C.c_int, [vp, u64p, u64p, C.POINTER(C.c_int32)]),
        "sgn_round": (C.c_int, [vp, u64p]),
        "sgn_run": (C.c_int, [vp, C.c_uint64, u64p]),
        "sgn_stats_get": (C.c_int, [vp, C.POINTER(Stats)]),
        "sgn_host_digests": (C.c_int, [vp, C.c_uint32, C.c_uint32, C.POINTER(HostDigest)]),
        "sgn_host_next_event_time": (C.c_int, [vp, C.c_uint32, u64p]),
        "sgn_trace_enable": (C.c_int, [vp, C.c_uint64]),
        "sgn_trace_read": (C.c_int, [vp, C.POINTER(TraceRec), C.c_uint64, u64p]),
        "sgn_kernel_times_get": (C.c_int, [vp, C.POINTER(KernelTimes)]),
        "sgn_engine_info_get": (C.c_int, [vp, C.POINTER(EngineInfo)]),
        "sgn_comm_get_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
        "sgn_comm_init": (C.c_int, [vp, C.POINTER(C.c_uint8), C.c_uint64]),
        "sgn_shard_range": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, u32p, u32p]),
        "sgn_comm_init_local": (C.c_int, [C.POINTER(vp), C.c_uint32, C.c_uint64]),
        "sgn_run_local_group": (C.c_int, [C.POINTER(vp), C.c_uint32, C.c_uint64, u64p]),
        "sgn_worker_get_latency": (C.c_uint64, [vp, C.c_uint32, C.c_uint32]),
        "sgn_worker_is_routable": (C.c_int32, [vp, C.c_uint32, C.c_uint32]),
        "sgn_worker_get_bandwidth_up_bytes": (C.c_uint64, [vp, C.c_uint32]),
        "sgn_worker_get_bandwidth_down_bytes": (C.c_uint64, [vp, C.c_uint32]),
        "sgn_addr_to_host_id": (C.c_int, [vp, C.c_uint32, u32p]),
        "sgn_gml_parse": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(vp), C.c_char_p, C.c_size_t]),
        "sgn_gml_free": (None, [vp]),
        "sgn_gml_graph": (C.c_int, [vp, C.POINTER(Graph)]),
        "sgn_gml_node_bandwidth": (C.c_int, [vp, C.c_uint32, u64p, C.POINTER(C.c_int32), u64p,
                                             C.POINTER(C.c_int32)]),
        "sgn_units_parse": (C.c_int, [C.c_int32, C.c_char_p, u64p]),
        "sgn_assign_ips": (C.c_int, [C.c_uint32, C.POINTER(C.c_uint8), u32p, u32p]),
        "sgn_pcap_open": (C.c_int, [C.c_char_p, C.c_uint32, C.POINTER(vp)]),
        "sgn_pcap_write_packet": (C.c_int, [vp, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint8), C.c_uint32]),
        "sgn_pcap_close": (C.c_int, [vp]),
        "sgn_packet_bytes": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.POINTER(C.c_uint8), C.c_uint32]),
        "sgn_trace_pcap": (C.c_int64, [C.POINTER(TraceRec), C.c_uint64, C.c_uint32, u32p, C.c_uint32,
                                       C.c_char_p, C.c_uint32]),
        "sgn_selftest_codel_law": (C.c_int, [vp, C.c_uint64, u64p]),
        "sgn_debug_stamps": (C.c_int, [vp, u64p, C.c_uint64, u64p]),
        "sgn_debug_rounds": (C.c_int, [vp, u64p]),
        "sgn_debug_rounds_x": (C.c_int, [vp, u64p]),
        "sgn_debug_rounds_xw": (C.c_int, [vp, u64p]),
        "sgn_submit": (C.c_int, [vp, C.POINTER(PktSoa)]),
        "sgn_drain_enable": (C.c_int, [vp, C.c_uint64]),
        "sgn_drain": (C.c_int, [vp, C.c_uint32, C.c_uint32, C.POINTER(DrainRec), C.c_uint64, u64p]),
        "sgn_set_window": (C.c_int, [vp, C.c_uint64, C.c_uint64]),
        "sgn_rng_next_u64": (C.c_int, [vp, C.c_uint32, u64p]),
        "sgn_rng_double": (C.c_int, [vp, C.c_uint32, C.POINTER(C.c_double)]),
        "sgn_rng_fill_bytes": (C.c_int, [vp, C.c_uint32, C.POINTER(C.c_uint8), C.c_size_t]),
        "sgn_rng_next_u64_batch": (C.c_int, [vp, u32p, u32p, C.c_uint32, u64p]),
        "sgn_hosts_next_event_time": (C.c_int, [vp, C.c_uint32, C.c_uint32, u64p]),
        "sgn_stage_create": (C.c_int, [vp, C.POINTER(vp)]),
        "sgn_stage_destroy": (None, [vp]),
        "sgn_stage_push": (C.c_int, [vp, C.POINTER(PktSoa)]),
        "sgn_stage_pending": (C.c_uint64, [vp]),
        "sgn_stage_flush": (C.c_int, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = L
    return L


def ptr(a: np.ndarray, ct):
    return a.ctypes.data_as(C.POINTER(ct))


class SgnError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__(f"libsgn error {rc}: {msg}")
        self.rc = rc


class GraphArrays:
    """Keeps numpy arrays alive behind an sgn_graph struct."""

    def __init__(self, node_id, src, dst, lat, loss, directed):
        self.node_id = np.ascontiguousarray(node_id, dtype=np.uint32)
        self.src = np.ascontiguousarray(src, dtype=np.uint32)
        self.dst = np.ascontiguousarray(dst, dtype=np.uint32)
        self.lat = np.ascontiguousarray(lat, dtype=np.uint64)
        self.loss = np.ascontiguousarray(loss, dtype=np.float32)
        self.directed = int(directed)

    def struct(self) -> Graph:
        return Graph(len(self.node_id), ptr(self.node_id, C.c_uint32), len(self.src),
                     ptr(self.src, C.c_uint32), ptr(self.dst, C.c_uint32),
                     ptr(self.lat, C.c_uint64), ptr(self.loss, C.c_float), self.directed)


class HostArrays:
    def __init__(self, ip, node_id, bw_up, bw_down, seed):
        self.ip = np.ascontiguousarray(ip, dtype=np.uint32)
        self.node_id = np.ascontiguousarray(node_id, dtype=np.uint32)
        self.bw_up = np.ascontiguousarray(bw_up, dtype=np.uint64)
        self.bw_down = np.ascontiguousarray(bw_down, dtype=np.uint64)
        self.seed = np.ascontiguousarray(seed, dtype=np.uint64)

    @property
    def n(self):
        return len(self.ip)

    def struct(self) -> Hosts:
        return Hosts(len(self.ip), ptr(self.ip, C.c_uint32), ptr(self.node_id, C.c_uint32),
                     ptr(self.bw_up, C.c_uint64), ptr(self.bw_down, C.c_uint64),
                     ptr(self.seed, C.c_uint64))


def make_traffic(kind=TRAFFIC_PERIODIC, *, flow_seed=7, start_ns=0, start_jitter_ns=0,
                 period_ns=10_000_000, period_jitter_ns=0, payload_len=1024,
                 unknown_dst_permille=0, req_payload=64, servers=None,
                 file_bytes=(50 * 1024, 1024 * 1024, 5 * 1024 * 1024)):
    t = Traffic()
    t.kind = kind
    t.payload_len = payload_len
    t.flow_seed = flow_seed
    t.start_ns = start_ns
    t.start_jitter_ns = start_jitter_ns
    t.period_ns = period_ns
    t.period_jitter_ns = period_jitter_ns
    t.unknown_dst_permille = unknown_dst_permille
    t.req_payload = req_payload
    keep = None
    if servers is not None:
        keep = np.ascontiguousarray(servers, dtype=np.uint32)
        t.n_servers = len(keep)
        t.server_hosts = ptr(keep, C.c_uint32)
    for i in range(3):
        t.file_bytes[i] = int(file_bytes[i])
    t._keep = keep  # noqa: SLF001 keep the server array alive with the struct
    return t


def make_config(stop_time_ns, *, bootstrap_end_ns=0, runahead_ns=1_000_000, dynamic=False,
                out_fifo_cap=64, codel_cap=1024, event_capacity=0, qdisc=0):
    c = SimConfig()
    c.stop_time_ns = stop_time_ns
    c.bootstrap_end_ns = bootstrap_end_ns
    c.runahead_ns = runahead_ns
    c.use_dynamic_runahead = 1 if dynamic else 0
    c.out_fifo_cap = out_fifo_cap
    c.codel_cap = codel_cap
    c.event_capacity = event_capacity
    c.interface_qdisc = qdisc
    return c


class Context:
    """One libsgn context (one GPU / shard)."""

    def __init__(self, device=0, shard_rank=0, shard_count=1, flags=0, lib=None):
        self.L = lib or load()
        self.h = C.c_void_p()
        opts = CreateOpts(device, shard_rank, shard_count, flags)
        rc = self.L.sgn_create(C.byref(self.h), C.byref(opts))
        if rc != 0:
            raise SgnError(rc, self.L.sgn_last_error(None).decode())
        self._keep = []

    def check(self, rc):
        if rc != 0:
            raise SgnError(rc, self.L.sgn_last_error(self.h).decode())
        return rc

    def close(self):
        if self.h:
            self.L.sgn_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- routing ----
    def routes_build(self, g: GraphArrays, used_node_ids, shortest=True):
        used = np.ascontiguousarray(used_node_ids, dtype=np.uint32)
        gs = g.struct()
        self.check(self.L.sgn_routes_build(self.h, C.byref(gs), ptr(used, C.c_uint32),
                                           len(used), 1 if shortest else 0))
        self.U = len(used)

    def routes_copy(self):
        lat = np.zeros(self.U * self.U, dtype=np.uint64)
        loss = np.zeros(self.U * self.U, dtype=np.float32)
        self.check(self.L.sgn_routes_copy(self.h, ptr(lat, C.c_uint64), ptr(loss, C.c_float)))
        return lat.reshape(self.U, self.U), loss.reshape(self.U, self.U)

    def routes_timing(self):
        t = RoutesTiming()
        self.check(self.L.sgn_routes_timing_get(self.h, C.byref(t)))
        return {n: getattr(t, n) for n, _ in t._fields_}

    # ---- hosts / sim ----
    def hosts_set(self, hosts: HostArrays):
        self._hosts = hosts
        hs = hosts.struct()
        self.check(self.L.sgn_hosts_set(self.h, C.byref(hs)))

    def trace_enable(self, cap):
        self.check(self.L.sgn_trace_enable(self.h, cap))

    def sim_init(self, cfg: SimConfig, traffic: Traffic):
        self._traffic = traffic
        self.check(self.L.sgn_sim_init(self.h, C.byref(cfg), C.byref(traffic)))

    def window(self):
        s, e, a = C.c_uint64(), C.c_uint64(), C.c_int32()
        self.check(self.L.sgn_window(self.h, C.byref(s), C.byref(e), C.byref(a)))
        return s.value, e.value, bool(a.value)

    def round(self):
        m = C.c_uint64()
        self.check(self.L.sgn_round(self.h, C.byref(m)))
        return m.value

    def run(self, max_rounds=1 << 62):
        d = C.c_uint64()
        self.check(self.L.sgn_run(self.h, max_rounds, C.byref(d)))
        return d.value

    def stats(self):
        s = Stats()
        self.check(self.L.sgn_stats_get(self.h, C.byref(s)))
        return s.as_dict()

    def digests(self, lo, hi):
        out = np.zeros(hi - lo, dtype=DIGEST_DTYPE)
        self.check(self.L.sgn_host_digests(self.h, lo, hi, out.ctypes.data_as(C.POINTER(HostDigest))))
        return out

    def trace(self):
        n = C.c_uint64()
        self.check(self.L.sgn_trace_read(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, dtype=TRACE_DTYPE)
        self.check(self.L.sgn_trace_read(self.h, out.ctypes.data_as(C.POINTER(TraceRec)), n.value, C.byref(n)))
        return out

    # ---- CPU-resident applications (TRAFFIC_EXTERNAL) and the host RNG ----
    def drain_enable(self, cap):
        self.check(self.L.sgn_drain_enable(self.h, cap))

    def submit(self, src_host, dst_ip, payload_len, send_time, handle=None, wire_len=None):
        b, keep = pkt_soa(src_host, dst_ip, payload_len, send_time, handle, wire_len)
        self.check(self.L.sgn_submit(self.h, C.byref(b)))

    def drain(self, lo=0, hi=0xFFFFFFFF, cap=1 << 22):
        out = np.zeros(cap, dtype=DRAIN_DTYPE)
        n = C.c_uint64()
        self.check(self.L.sgn_drain(self.h, lo, hi, out.ctypes.data_as(C.POINTER(DrainRec)), cap, C.byref(n)))
        return out[: n.value]

    def set_window(self, start, end):
        self.check(self.L.sgn_set_window(self.h, start, end))

    def rng_next_u64(self, host):
        v = C.c_uint64()
        self.check(self.L.sgn_rng_next_u64(self.h, host, C.byref(v)))
        return v.value

    def rng_double(self, host):
        v = C.c_double()
        self.check(self.L.sgn_rng_double(self.h, host, C.byref(v)))
        return v.value

    def rng_fill_bytes(self, host, n):
        buf = (C.c_uint8 * max(1, n))()
        self.check(self.L.sgn_rng_fill_bytes(self.h, host, buf, n))
        return bytes(buf[:n])

    def engine_info(self):
        e = EngineInfo()
        self.check(self.L.sgn_engine_info_get(self.h, C.byref(e)))
        return {n: int(getattr(e, n)) for n, _ in e._fields_}

    def rng_next_u64_batch(self, hosts, counts):
        h = np.ascontiguousarray(hosts, dtype=np.uint32)
        k = np.ascontiguousarray(counts, dtype=np.uint32)
        out = np.zeros(max(1, int(k.sum())), dtype=np.uint64)
        self.check(self.L.sgn_rng_next_u64_batch(self.h, ptr(h, C.c_uint32), ptr(k, C.c_uint32), len(h),
                                                 ptr(out, C.c_uint64)))
        return out[: int(k.sum())]

    def next_event_time(self, host):
        t = C.c_uint64()
        self.check(self.L.sgn_host_next_event_time(self.h, host, C.byref(t)))
        return t.value

    def next_event_times(self, lo, hi):
        out = np.zeros(max(1, hi - lo), dtype=np.uint64)
        self.check(self.L.sgn_hosts_next_event_time(self.h, lo, hi, ptr(out, C.c_uint64)))
        return out[: hi - lo]

    # ---- per-thread staging (sgn_stage_*) ----
    def stage_create(self):
        st = C.c_void_p()
        self.check(self.L.sgn_stage_create(self.h, C.byref(st)))
        return st

    def stage_push(self, st, src_host, dst_ip, payload_len, send_time, handle=None, wire_len=None):
        b, keep = pkt_soa(src_host, dst_ip, payload_len, send_time, handle, wire_len)
        rc = self.L.sgn_stage_push(st, C.byref(b))
        if rc != 0:
            raise SgnError(rc, "sgn_stage_push: invalid batch")

    def stage_flush(self):
        self.check(self.L.sgn_stage_flush(self.h))

    def kernel_times(self):
        k = KernelTimes()
        self.check(self.L.sgn_kernel_times_get(self.h, C.byref(k)))
        return {k.name[i].decode(): (int(k.launches[i]), float(k.ms[i])) for i in range(k.n_kernels)}

    def kernel_launches_total(self):
        """Every launch of each engine kernel since sim_init (kernel_times() covers a sample)."""
        k = KernelTimes()
        self.check(self.L.sgn_kernel_times_get(self.h, C.byref(k)))
        return {k.name[i].decode(): int(k.launches_total[i]) for i in range(k.n_kernels)}


# ------------------------------------------------------------------------------------
# Workload helpers (host side of SimConfig::new: names, IPs, seeds, bandwidth)
# ------------------------------------------------------------------------------------

def host_names(n, prefix="h"):
    width = max(5, len(str(n - 1)))
    return [f"{prefix}{i:0{width}d}" for i in range(n)]


def assign_ips(n, explicit=None, lib=None):
    """assign_ips (core/sim_config.rs:386-407) through libsgn's sgn_assign_ips: hosts in HostId
    order; `explicit` maps host index -> configured IPv4 (int, host byte order); every other
    host gets the next free address from 11.0.0.1 on, skipping .0/.255 and configured ones
    (IpAssignment, network/graph/mod.rs:355-417)."""
    L = lib or load()
    ips = np.zeros(n, dtype=np.uint32)
    flags = np.zeros(n, dtype=np.uint8)
    for i, ip in (explicit or {}).items():
        ips[i] = ip
        flags[i] = 1
    bad = C.c_uint32(0)
    rc = L.sgn_assign_ips(n, ptr(flags, C.c_uint8), ptr(ips, C.c_uint32), C.byref(bad))
    if rc != 0:
        what = "IP address has already been assigned" if rc == -22 else "address space exhausted"
        raise SgnError(rc, f"sgn_assign_ips: host {bad.value}: {what}")
    return ips


def gml_parse(text, lib=None):
    """GML text -> (GraphArrays, [(up_bits|None, down_bits|None) per node]) through libsgn's
    sgn_gml_parse (gml_parser + NetworkGraph::parse, network/graph/mod.rs:28-179)."""
    L = lib or load()
    b = text.encode() if isinstance(text, str) else bytes(text)
    h = C.c_void_p()
    err = C.create_string_buffer(512)
    rc = L.sgn_gml_parse(b, len(b), C.byref(h), err, 512)
    if rc != 0:
        raise SgnError(rc, err.value.decode(errors="replace"))
    try:
        g = Graph()
        L.sgn_gml_graph(h, C.byref(g))
        n, e = g.n_nodes, g.n_edges
        arr = lambda p, k: np.ctypeslib.as_array(p, (k,)).copy() if k else []
        ga = GraphArrays(arr(g.node_id, n), arr(g.edge_src, e), arr(g.edge_dst, e),
                         arr(g.edge_latency_ns, e), arr(g.edge_loss, e), g.directed)
        bws = []
        for i in range(n):
            up, down = C.c_uint64(), C.c_uint64()
            hu, hd = C.c_int32(), C.c_int32()
            L.sgn_gml_node_bandwidth(h, i, C.byref(up), C.byref(hu), C.byref(down), C.byref(hd))
            bws.append((up.value if hu.value else None, down.value if hd.value else None))
    finally:
        L.sgn_gml_free(h)
    return ga, bws


def packet_bytes(src_ip, dst_ip, payload_len, tag=0, lib=None):
    """Packet::display_bytes of one path packet (sgn_packet_bytes)."""
    L = lib or load()
    n = L.sgn_packet_bytes(src_ip, dst_ip, payload_len, tag, None, 0)
    out = np.zeros(n, dtype=np.uint8)
    L.sgn_packet_bytes(src_ip, dst_ip, payload_len, tag, ptr(out, C.c_uint8), n)
    return out.tobytes()


def write_pcaps(trace, host_ips, out_dir, names=None, hosts=None, capture_len=65535, lib=None):
    """Per-host interface captures from trace records (sgn_trace_pcap), one file per host in
    `hosts` (default: every host with a captured packet), laid out like the reference's
    <data_directory>/hosts/<hostname>/eth0.pcap (interface.rs:45-51, namespace.rs:42) when
    names are given (else <out_dir>/h<id>/eth0.pcap). Returns {host: (path, packets)}."""
    L = lib or load()
    tr = np.ascontiguousarray(trace, dtype=TRACE_DTYPE)
    ips = np.ascontiguousarray(host_ips, dtype=np.uint32)
    if hosts is None:
        cap = tr[np.isin(tr["kind"], [TRACE_IF_POP, TRACE_DELIVER, TRACE_LOCAL])]
        hosts = np.unique(cap["host"]).tolist()
    out = {}
    for h in hosts:
        d = os.path.join(out_dir, "hosts", names[h]) if names is not None else os.path.join(out_dir, f"h{h}")
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, "eth0.pcap")
        n = L.sgn_trace_pcap(tr.ctypes.data_as(C.POINTER(TraceRec)), len(tr), int(h), ptr(ips, C.c_uint32),
                             len(ips), path.encode(), capture_len)
        if n < 0:
            raise SgnError(int(n), f"sgn_trace_pcap host {h}")
        out[int(h)] = (path, int(n))
    return out


def derive_seeds(sim_seed, names, lib=None):
    L = lib or load()
    arr = (C.c_char_p * len(names))(*[s.encode() for s in names])
    out = np.zeros(len(names), dtype=np.uint64)
    rc = L.sgn_derive_host_seeds(sim_seed, arr, len(names), ptr(out, C.c_uint64))
    if rc != 0:
        raise SgnError(rc, "sgn_derive_host_seeds")
    return out


def random_graph(V, mean_degree=6, seed=42, lat_lo_us=1000, lat_hi_us=50000,
                 loss_frac=0.2, loss_hi=0.02):
    """Config B graph: undirected spanning tree + random extra edges to the mean degree,
    one self-loop per node (1 ms, loss 0). Loss values are rounded to 6 decimals as they
    would be printed into GML, then parsed as f32."""
    rng = np.random.default_rng(seed)
    src, dst = [], []
    perm = rng.permutation(V)
    for i in range(1, V):
        j = int(rng.integers(0, i))
        src.append(int(perm[i]))
        dst.append(int(perm[j]))
    extra = max(0, V * mean_degree // 2 - (V - 1))
    seen = set((min(a, b), max(a, b)) for a, b in zip(src, dst))
    while extra > 0:
        a, b = (int(x) for x in rng.integers(0, V, 2))
        if a == b or (min(a, b), max(a, b)) in seen:
            continue
        seen.add((min(a, b), max(a, b)))
        src.append(a)
        dst.append(b)
        extra -= 1
    E = len(src)
    lat = rng.integers(lat_lo_us, lat_hi_us + 1, E).astype(np.uint64) * 1000
    lossy = rng.random(E) < loss_frac
    loss = np.where(lossy, np.round(rng.uniform(1e-4, loss_hi, E), 6), 0.0)
    loss = np.array([np.float32(float(f"{x:.6f}")) for x in loss], dtype=np.float32)
    src += list(range(V))
    dst += list(range(V))
    lat = np.concatenate([lat, np.full(V, 1_000_000, dtype=np.uint64)])
    loss = np.concatenate([loss, np.zeros(V, dtype=np.float32)])
    return GraphArrays(np.arange(V), src, dst, lat, loss, directed=False)


def tor_graph(V, seed=42):
    """Config C graph: complete graph over V 'city' nodes. Latency = 1 ms + a distance term
    (5-150 ms) from random points on a sphere; loss 0-0.5 %; self-loop 1 ms."""
    rng = np.random.default_rng(seed)
    z = rng.uniform(-1, 1, V)
    t = rng.uniform(0, 2 * np.pi, V)
    r = np.sqrt(1 - z * z)
    P = np.stack([r * np.cos(t), r * np.sin(t), z], 1)
    iu, ju = np.triu_indices(V, 1)
    ang = np.arccos(np.clip((P[iu] * P[ju]).sum(1), -1, 1)) / np.pi
    lat_us = (1000 + 5000 + ang * 145000).astype(np.uint64)
    loss = np.round(rng.uniform(0, 0.005, len(iu)), 6).astype(np.float32)
    src = np.concatenate([iu, np.arange(V)])
    dst = np.concatenate([ju, np.arange(V)])
    lat = np.concatenate([lat_us * 1000, np.full(V, 1_000_000, dtype=np.uint64)])
    loss = np.concatenate([loss, np.zeros(V, dtype=np.float32)])
    return GraphArrays(np.arange(V), src, dst, lat, loss, directed=False)


def bandwidth_classes(n, seed=3, classes=(10_000_000, 100_000_000, 1_000_000_000)):
    rng = np.random.default_rng(seed)
    return np.array(classes, dtype=np.uint64)[rng.integers(0, len(classes), n)]


def zipf_nodes(n_hosts, V, seed=5, s=1.0):
    """Host -> node with a Zipf(s) node popularity (config C)."""
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, V + 1) ** s
    w /= w.sum()
    order = rng.permutation(V)
    return order[rng.choice(V, size=n_hosts, p=w)].astype(np.uint32)
