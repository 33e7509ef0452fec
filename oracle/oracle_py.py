"""ctypes binding of the parity oracle (oracle/liboracle.so). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the timed CPU baseline. Nothing under
shadow-gen_amd/ imports it.
"""
from __future__ import annotations

import ctypes as C
import pathlib
import subprocess
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent / "shadow-gen_amd"))
import sgn  # noqa: E402  (struct definitions only)

LIB = HERE / "liboracle.so"
_L = None


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def load():
    global _L
    if _L is not None:
        return _L
    if not LIB.exists():
        build()
    L = C.CDLL(str(LIB))
    vp = C.c_void_p
    u32p, u64p, f32p = sgn.u32p, sgn.u64p, sgn.f32p
    sig = {
        "ora_siphash": (C.c_uint64, [C.c_int, C.c_int, C.c_uint64, C.c_uint64, C.c_char_p, C.c_size_t]),
        "ora_xoshiro_seed_from_u64": (None, [C.c_uint64, u64p]),
        "ora_xoshiro_next_u64": (C.c_uint64, [u64p]),
        "ora_xoshiro_next_f64": (C.c_double, [u64p]),
        "ora_splitmix_next": (C.c_uint64, [u64p]),
        "ora_host_seeds": (None, [C.c_uint32, C.POINTER(C.c_char_p), C.c_uint32, u64p]),
        "ora_units_parse": (C.c_int, [C.c_int, C.c_char_p, u64p]),
        "ora_tb_new": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, vp]),
        "ora_tb_remove": (C.c_int, [vp, C.c_uint64, C.c_uint64, u64p]),
        "ora_codel_control_law": (C.c_uint64, [C.c_uint64, C.c_uint64]),
        "ora_codel_new": (vp, []),
        "ora_codel_free": (None, [vp]),
        "ora_codel_push": (None, [vp, C.c_uint32, C.c_uint64]),
        "ora_codel_pop": (C.c_int, [vp, C.c_uint64, u32p]),
        "ora_codel_process_standing_delay": (C.c_int, [vp, C.c_uint64, C.c_uint64]),
        "ora_codel_get": (None, [vp, vp]),
        "ora_codel_set_mode": (None, [vp, C.c_int]),
        "ora_codel_was_dropping_recently": (C.c_int, [vp, C.c_uint64]),
        "ora_codel_should_drop": (C.c_int, [vp, C.c_uint64]),
        "ora_assign_ips": (C.c_int, [C.c_uint32, C.POINTER(C.c_uint8), u32p]),
        "ora_gml_parse": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(vp), C.c_char_p, C.c_size_t]),
        "ora_gml_free": (None, [vp]),
        "ora_gml_graph": (C.c_int, [vp, C.POINTER(sgn.Graph)]),
        "ora_gml_node_bandwidth": (C.c_int, [vp, C.c_uint32, u64p, C.POINTER(C.c_int32), u64p,
                                             C.POINTER(C.c_int32)]),
        "ora_routes": (C.c_int, [C.POINTER(sgn.Graph), u32p, C.c_uint32, C.c_int, u64p, f32p,
                                 C.c_char_p, C.c_size_t]),
        "ora_sim_create": (C.c_int, [u32p, C.c_uint32, u64p, f32p, C.POINTER(sgn.Hosts),
                                     C.POINTER(sgn.SimConfig), C.POINTER(sgn.Traffic), C.c_int,
                                     C.POINTER(vp), C.c_char_p, C.c_size_t]),
        "ora_sim_free": (None, [vp]),
        "ora_sim_set_threads": (C.c_int, [vp, C.c_int]),
        "ora_sim_set_faithful": (C.c_int, [vp, C.c_int]),
        "ora_routes_mode": (C.c_int, [C.POINTER(sgn.Graph), u32p, C.c_uint32, C.c_int, C.c_int, C.c_int,
                                      u64p, f32p, C.c_char_p, C.c_size_t]),
        "ora_sim_window": (C.c_int, [vp, u64p, u64p, C.POINTER(C.c_int32)]),
        "ora_sim_round": (C.c_int, [vp, u64p]),
        "ora_sim_run": (C.c_int, [vp, C.c_uint64, u64p]),
        "ora_sim_stats": (C.c_int, [vp, C.POINTER(sgn.Stats)]),
        "ora_sim_host_digests": (C.c_int, [vp, C.c_uint32, C.c_uint32, C.POINTER(sgn.HostDigest)]),
        "ora_sim_trace_count": (C.c_uint64, [vp]),
        "ora_sim_trace_read": (C.c_uint64, [vp, C.POINTER(sgn.TraceRec), C.c_uint64]),
        "ora_sim_host_next_event_time": (C.c_int, [vp, C.c_uint32, u64p]),
        "ora_sim_set_shard": (C.c_int, [vp, C.c_uint32, C.c_uint32]),
        "ora_sim_shard_execute": (C.c_int, [vp, u64p]),
        "ora_sim_shard_take_exports": (C.c_uint64, [vp, u64p, C.c_uint64]),
        "ora_sim_shard_import": (C.c_int, [vp, u64p, C.c_uint64]),
        "ora_sim_shard_local_min": (C.c_int, [vp, u64p, u64p]),
        "ora_sim_shard_advance": (C.c_int, [vp, C.c_uint64, C.c_uint64]),
        "ora_sim_submit": (C.c_int, [vp, C.POINTER(sgn.PktSoa)]),
        "ora_sim_drain": (C.c_int, [vp, C.c_uint32, C.c_uint32, C.POINTER(sgn.DrainRec), C.c_uint64, u64p]),
        "ora_sim_set_window": (C.c_int, [vp, C.c_uint64, C.c_uint64]),
        "ora_sim_rng_next_u64": (C.c_int, [vp, C.c_uint32, u64p]),
        "ora_sim_rng_double": (C.c_int, [vp, C.c_uint32, C.POINTER(C.c_double)]),
        "ora_sim_rng_fill_bytes": (C.c_int, [vp, C.c_uint32, C.POINTER(C.c_uint8), C.c_size_t]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _L = L
    return L


class TB(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("capacity", "balance", "refill_increment",
                                          "refill_interval", "last_refill")]


class CodelState(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("len", "total_bytes", "mode", "has_interval_end",
                                          "interval_end", "has_drop_next", "drop_next",
                                          "current_drop_count", "previous_drop_count",
                                          "dropped_total")]


def routes(g: sgn.GraphArrays, used, shortest=True, faithful=False, threads=1):
    """compute_shortest_paths / get_direct_paths (network/graph/mod.rs:181-250) -> dense U x U
    (latency u64, loss f32). faithful: the reference's hash-map data structures; threads:
    sources in parallel (rayon). Identical results in every mode."""
    L = load()
    used = np.ascontiguousarray(used, dtype=np.uint32)
    U = len(used)
    lat = np.zeros(U * U, dtype=np.uint64)
    loss = np.zeros(U * U, dtype=np.float32)
    err = C.create_string_buffer(512)
    gs = g.struct()
    rc = L.ora_routes_mode(C.byref(gs), sgn.ptr(used, C.c_uint32), U, 1 if shortest else 0,
                           1 if faithful else 0, threads, sgn.ptr(lat, C.c_uint64),
                           sgn.ptr(loss, C.c_float), err, 512)
    if rc != 0:
        raise sgn.SgnError(rc, err.value.decode())
    return lat.reshape(U, U), loss.reshape(U, U)


def gml_parse(text: str):
    """Returns (GraphArrays, bandwidth dict) or raises SgnError."""
    L = load()
    b = text.encode()
    h = C.c_void_p()
    err = C.create_string_buffer(512)
    rc = L.ora_gml_parse(b, len(b), C.byref(h), err, 512)
    if rc != 0:
        raise sgn.SgnError(rc, err.value.decode())
    g = sgn.Graph()
    L.ora_gml_graph(h, C.byref(g))
    n, e = g.n_nodes, g.n_edges
    ga = sgn.GraphArrays(np.ctypeslib.as_array(g.node_id, (n,)).copy() if n else [],
                         np.ctypeslib.as_array(g.edge_src, (e,)).copy() if e else [],
                         np.ctypeslib.as_array(g.edge_dst, (e,)).copy() if e else [],
                         np.ctypeslib.as_array(g.edge_latency_ns, (e,)).copy() if e else [],
                         np.ctypeslib.as_array(g.edge_loss, (e,)).copy() if e else [],
                         g.directed)
    bws = []
    for i in range(n):
        up, down = C.c_uint64(), C.c_uint64()
        hu, hd = C.c_int32(), C.c_int32()
        L.ora_gml_node_bandwidth(h, i, C.byref(up), C.byref(hu), C.byref(down), C.byref(hd))
        bws.append((up.value if hu.value else None, down.value if hd.value else None))
    L.ora_gml_free(h)
    return ga, bws


def host_seeds(sim_seed, names):
    L = load()
    arr = (C.c_char_p * len(names))(*[s.encode() for s in names])
    out = np.zeros(len(names), dtype=np.uint64)
    L.ora_host_seeds(sim_seed, arr, len(names), sgn.ptr(out, C.c_uint64))
    return out


def assign_ips(n, explicit=None):
    """ora_assign_ips: (rc, ips) with the reference's per-host vacancy loop (oracle.cpp)."""
    L = load()
    ips = np.zeros(n, dtype=np.uint32)
    flags = np.zeros(n, dtype=np.uint8)
    for i, ip in (explicit or {}).items():
        ips[i] = ip
        flags[i] = 1
    rc = L.ora_assign_ips(n, flags.ctypes.data_as(C.POINTER(C.c_uint8)), sgn.ptr(ips, C.c_uint32))
    return rc, ips


class Sim:
    """The reference-structured round loop (core/manager.rs:541-656) on the CPU."""

    def __init__(self, used, lat, loss, hosts: sgn.HostArrays, cfg, traffic, trace=False, threads=1,
                 faithful=False):
        self.L = load()
        used = np.ascontiguousarray(used, dtype=np.uint32)
        lat = np.ascontiguousarray(lat, dtype=np.uint64).ravel()
        loss = np.ascontiguousarray(loss, dtype=np.float32).ravel()
        self._keep = (used, lat, loss, hosts, traffic)
        self.h = C.c_void_p()
        err = C.create_string_buffer(512)
        hs = hosts.struct()
        rc = self.L.ora_sim_create(sgn.ptr(used, C.c_uint32), len(used), sgn.ptr(lat, C.c_uint64),
                                   sgn.ptr(loss, C.c_float), C.byref(hs), C.byref(cfg),
                                   C.byref(traffic), 1 if trace else 0, C.byref(self.h), err, 512)
        if rc != 0:
            raise sgn.SgnError(rc, err.value.decode())
        self.n = hosts.n
        if threads != 1:
            assert self.L.ora_sim_set_threads(self.h, threads) == 0
        if faithful:
            assert self.L.ora_sim_set_faithful(self.h, 1) == 0

    def set_threads(self, n):
        assert self.L.ora_sim_set_threads(self.h, n) == 0

    def set_faithful(self, on):
        assert self.L.ora_sim_set_faithful(self.h, 1 if on else 0) == 0

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ora_sim_free(self.h)
            self.h = None

    def window(self):
        s, e, a = C.c_uint64(), C.c_uint64(), C.c_int32()
        self.L.ora_sim_window(self.h, C.byref(s), C.byref(e), C.byref(a))
        return s.value, e.value, bool(a.value)

    def round(self):
        m = C.c_uint64()
        rc = self.L.ora_sim_round(self.h, C.byref(m))
        if rc != 0:
            raise sgn.SgnError(rc, "oracle round")
        return m.value

    def run(self, max_rounds=1 << 62):
        d = C.c_uint64()
        self.L.ora_sim_run(self.h, max_rounds, C.byref(d))
        return d.value

    def stats(self):
        s = sgn.Stats()
        self.L.ora_sim_stats(self.h, C.byref(s))
        return s.as_dict()

    def digests(self, lo=0, hi=None):
        hi = self.n if hi is None else hi
        out = np.zeros(hi - lo, dtype=sgn.DIGEST_DTYPE)
        self.L.ora_sim_host_digests(self.h, lo, hi, out.ctypes.data_as(C.POINTER(sgn.HostDigest)))
        return out

    def trace(self):
        n = self.L.ora_sim_trace_count(self.h)
        out = np.zeros(n, dtype=sgn.TRACE_DTYPE)
        self.L.ora_sim_trace_read(self.h, out.ctypes.data_as(C.POINTER(sgn.TraceRec)), n)
        return out

    def next_event_time(self, host):
        t = C.c_uint64()
        self.L.ora_sim_host_next_event_time(self.h, host, C.byref(t))
        return t.value

    # sharded protocol (round-edge rehearsal)
    def set_shard(self, lo, hi):
        assert self.L.ora_sim_set_shard(self.h, lo, hi) == 0

    def shard_execute(self):
        n = C.c_uint64()
        rc = self.L.ora_sim_shard_execute(self.h, C.byref(n))
        if rc != 0:
            raise sgn.SgnError(rc, "oracle shard execute")
        out = np.zeros(6 * n.value, dtype=np.uint64)
        self.L.ora_sim_shard_take_exports(self.h, sgn.ptr(out, C.c_uint64), n.value)
        return out.reshape(-1, 6)

    def shard_import(self, recs):
        recs = np.ascontiguousarray(recs, dtype=np.uint64)
        assert self.L.ora_sim_shard_import(self.h, sgn.ptr(recs, C.c_uint64), len(recs)) == 0

    def shard_local_min(self):
        a, b = C.c_uint64(), C.c_uint64()
        self.L.ora_sim_shard_local_min(self.h, C.byref(a), C.byref(b))
        return a.value, b.value

    def shard_advance(self, gmin, gmin_used):
        self.L.ora_sim_shard_advance(self.h, gmin, gmin_used)

    # CPU-resident applications (TRAFFIC_EXTERNAL) and the host RNG: libsgn's contract
    def _ok(self, rc, what):
        if rc != 0:
            raise sgn.SgnError(rc, "oracle " + what)

    def submit(self, src_host, dst_ip, payload_len, send_time, handle=None, wire_len=None):
        b, keep = sgn.pkt_soa(src_host, dst_ip, payload_len, send_time, handle, wire_len)
        self._ok(self.L.ora_sim_submit(self.h, C.byref(b)), "submit")

    def drain(self, lo=0, hi=0xFFFFFFFF, cap=1 << 22):
        out = np.zeros(cap, dtype=sgn.DRAIN_DTYPE)
        n = C.c_uint64()
        self._ok(self.L.ora_sim_drain(self.h, lo, hi, out.ctypes.data_as(C.POINTER(sgn.DrainRec)), cap,
                                      C.byref(n)), "drain")
        return out[: n.value]

    def set_window(self, start, end):
        self._ok(self.L.ora_sim_set_window(self.h, start, end), "set_window")

    def rng_next_u64(self, host):
        v = C.c_uint64()
        self._ok(self.L.ora_sim_rng_next_u64(self.h, host, C.byref(v)), "rng")
        return v.value

    def rng_double(self, host):
        v = C.c_double()
        self._ok(self.L.ora_sim_rng_double(self.h, host, C.byref(v)), "rng")
        return v.value

    def rng_fill_bytes(self, host, n):
        buf = (C.c_uint8 * max(1, n))()
        self._ok(self.L.ora_sim_rng_fill_bytes(self.h, host, buf, n), "rng")
        return bytes(buf[:n])
