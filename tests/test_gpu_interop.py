"""GPU parity of the CPU-interop exports and of the per-thread
staging handles (§8b), through the C ABI against the oracle:

* sgn_host_next_event_time / sgn_hosts_next_event_time -> Host::next_event_time
  (host/host.rs:832-834), the input of worker_maxEventRunaheadTime (core/worker.rs:774-777);
* sgn_route_get / sgn_min_latency -> RoutingInfo::path / get_smallest_latency_ns
  (network/graph/mod.rs:442,472);
* sgn_rng_next_u64_batch -> host_rngDouble / host_rngNextNBytes's stream (host.rs:1324-1336);
* sgn_stage_push + sgn_stage_flush == one sgn_submit of the concatenated stages.
"""
import numpy as np
import pytest

import sgn

pytestmark = pytest.mark.gpu


def _pair(oracle, n=300, V=40, stop_ns=400_000_000, kind=sgn.TRAFFIC_TGEN):
    g = sgn.tor_graph(V, seed=4)
    used = np.arange(V)
    names = sgn.host_names(n)
    seeds = sgn.derive_seeds(1, names)
    bw = np.where(np.arange(n) % 10 == 0, 100_000_000, 5_000_000).astype(np.uint64)
    hosts = sgn.HostArrays(sgn.assign_ips(n), (np.arange(n) * 7) % V, bw, bw, seeds)
    cfg = sgn.make_config(stop_ns, out_fifo_cap=64, codel_cap=4096, event_capacity=1 << 20)
    tr = sgn.make_traffic(kind, period_ns=50_000_000, period_jitter_ns=50_000_000,
                          start_jitter_ns=20_000_000, servers=np.arange(0, n, 10),
                          file_bytes=(20 * 1024, 100 * 1024, 300 * 1024))
    lat, loss = oracle.routes(g, used)
    o = oracle.Sim(used, lat, loss, hosts, cfg, tr)
    c = sgn.Context()
    c.routes_build(g, used)
    c.hosts_set(hosts)
    c.sim_init(cfg, tr)
    return o, c, hosts, g, used, lat


def test_next_event_times_match_oracle(oracle):
    o, c, hosts, *_ = _pair(oracle)
    n = hosts.n
    checked = 0
    for r in range(120):
        if r % 10 == 3:
            want = np.array([o.next_event_time(h) for h in range(n)], dtype=np.uint64)
            got = c.next_event_times(0, n)
            assert np.array_equal(want, got), np.nonzero(want != got)[0][:5]
            # single-host form and a sub-range
            for h in (0, 1, n // 2, n - 1):
                assert c.next_event_time(h) == want[h]
            assert np.array_equal(c.next_event_times(17, 90), want[17:90])
            checked += int((want != sgn.EMUTIME_INVALID).sum())
        assert o.round() == c.round()
    assert checked > 1000
    with pytest.raises(sgn.SgnError, match="not owned"):
        c.next_event_times(0, n + 1)


def test_route_get_and_min_latency(oracle):
    _, c, _, g, used, lat = _pair(oracle, n=50, V=30)
    L = c.L
    lo, ls = sgn.C.c_uint64(), sgn.C.c_float()
    _, loss = oracle.routes(g, used)
    for i in range(0, 30, 3):
        for j in range(0, 30, 4):
            c.check(L.sgn_route_get(c.h, int(used[i]), int(used[j]), sgn.C.byref(lo), sgn.C.byref(ls)))
            assert lo.value == lat[i, j]
            assert np.float32(ls.value).view(np.uint32) == loss[i, j].view(np.uint32)
    assert L.sgn_route_get(c.h, 12345, 0, sgn.C.byref(lo), sgn.C.byref(ls)) == -2  # SGN_ENOENT
    m = sgn.C.c_uint64()
    c.check(L.sgn_min_latency(c.h, sgn.C.byref(m)))
    assert m.value == lat.min()  # over every entry incl. self-loops (graph/mod.rs:472)


def test_rng_batch_is_the_host_stream(oracle):
    o, c, hosts, *_ = _pair(oracle, n=64, V=16, kind=sgn.TRAFFIC_PERIODIC)
    for _ in range(30):
        assert o.round() == c.round()
    hs = np.array([5, 0, 63, 17], dtype=np.uint32)
    ks = np.array([3, 0, 1000, 7], dtype=np.uint32)
    got = c.rng_next_u64_batch(hs, ks)
    want = []
    for h, k in zip(hs, ks):
        want += [o.rng_next_u64(int(h)) for _ in range(int(k))]
    assert got.tolist() == want
    # the simulation continues on the advanced streams identically
    for _ in range(30):
        assert o.round() == c.round()
    d_o, d_c = o.digests(0, 64), c.digests(0, 64)
    assert np.array_equal(d_o["rng"], d_c["rng"]) and np.array_equal(d_o["tx"], d_c["tx"])
    with pytest.raises(sgn.SgnError, match="distinct"):
        c.rng_next_u64_batch([3, 3], [1, 1])


def test_rng_single_draws_cpu_held(oracle):
    """sgn_rng_next_u64 / _double / _fill_bytes between rounds: the host's state is read once,
    stepped on the CPU and written back (with the stream position) before the next device
    operation — interleaved with batch draws, rounds and digests, draw for draw the host
    stream; the per-call cost is reported (a device round trip only on a host's first draw
    after a device operation)."""
    import time
    o, c, hosts, *_ = _pair(oracle, n=64, V=16, kind=sgn.TRAFFIC_PERIODIC)
    for _ in range(10):
        assert o.round() == c.round()
    t0 = time.perf_counter()
    for _ in range(2000):
        assert c.rng_double(9) == o.rng_double(9)
    per_call_us = (time.perf_counter() - t0) / 2000 * 1e6
    print(f"sgn_rng_double per call: {per_call_us:.2f} us (incl. the oracle's call)")
    assert c.rng_next_u64(9) == o.rng_next_u64(9)
    # a batch draw of the same host continues the CPU-held stream
    got = c.rng_next_u64_batch(np.array([9, 4], np.uint32), np.array([5, 2], np.uint32))
    want = [o.rng_next_u64(9) for _ in range(5)] + [o.rng_next_u64(4) for _ in range(2)]
    assert got.tolist() == want
    for _ in range(3):
        assert c.rng_next_u64(4) == o.rng_next_u64(4)
    assert c.rng_fill_bytes(4, 13) == o.rng_fill_bytes(4, 13)
    d_o, d_c = o.digests(0, 64), c.digests(0, 64)  # digests see the CPU-held states
    assert np.array_equal(d_o["rng"], d_c["rng"])
    for _ in range(20):
        assert o.round() == c.round()
    d_o, d_c = o.digests(0, 64), c.digests(0, 64)
    assert np.array_equal(d_o["rng"], d_c["rng"]) and np.array_equal(d_o["tx"], d_c["tx"])
    assert per_call_us < 50


class _Staged:
    """A CPU controller with three worker threads: each host's datagrams go through the
    stage of the thread that owns the host (host % 3), then one flush per round."""

    def __init__(self, ctx, n_stages=3):
        self.c = ctx
        self.st = [ctx.stage_create() for _ in range(n_stages)]

    def __getattr__(self, k):
        return getattr(self.c, k)

    def submit(self, src, dip, pay, t, handle, wire_len=None):
        src = np.asarray(src)
        for k, st in enumerate(self.st):
            m = (src % len(self.st)) == k
            if m.any():
                self.c.stage_push(st, src[m], np.asarray(dip)[m], np.asarray(pay)[m], np.asarray(t)[m],
                                  np.asarray(handle)[m], np.asarray(wire_len)[m])
        self.c.stage_flush()
        assert all(self.c.L.sgn_stage_pending(st) == 0 for st in self.st)


class _StageOrder:
    """The oracle fed the same datagrams in the flush's concatenation order."""

    def __init__(self, sim, n_stages=3):
        self.s = sim
        self.k = n_stages

    def __getattr__(self, k):
        return getattr(self.s, k)

    def submit(self, src, dip, pay, t, handle, wire_len=None):
        src = np.asarray(src)
        order = np.argsort(src % self.k, kind="stable")
        self.s.submit(src[order], np.asarray(dip)[order], np.asarray(pay)[order], np.asarray(t)[order],
                      np.asarray(handle)[order], wire_len=np.asarray(wire_len)[order])


def test_stage_flush_equals_submit(oracle):
    from external_common import datagrams, drive, external_world
    world = external_world()
    g, used, hosts, cfg, tr = world
    lat, loss = oracle.routes(g, used)
    o = oracle.Sim(used, lat, loss, hosts, cfg, tr, trace=True)
    c = sgn.Context()
    c.routes_build(g, used)
    c.hosts_set(hosts)
    c.drain_enable(1 << 16)
    c.sim_init(cfg, tr)
    dg = datagrams(hosts)
    (do, dc), rounds = drive([_StageOrder(o), _Staged(c)], dg)
    assert rounds > 50 and len(do) == len(dg[3]) == len(dc)
    for f in sgn.DRAIN_DTYPE.names:
        assert np.array_equal(do[f], dc[f]), f
