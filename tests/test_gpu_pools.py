"""Device pools that grow instead of refusing a scenario (-m gpu).

The reference's queues are unbounded: the router's CoDelQueue has no limit
(network/router/codel_queue.rs:33,303-317) and each host's EventQueue is a BinaryHeap
(core/work/event_queue.rs:12,57-66). libsgn keeps them in device pools sized at sim_init; a
round edge holds the rounds before a round that could outgrow a pool (nothing of that round
has run), the host grows the pool, and the round runs:
  * CoDel page pool: a round takes at most (D + 15 min(D, hosts)) / 16 pages for D due runs;
  * calendar slabs: a run whose slab is full goes to a spill area, the round edge holds, and
    the calendar is re-laid out with larger slabs before the run can be due.
Every case is bit-exact against the oracle (which has unbounded std containers) and checks
that the pools really grew and that no CoDel page was lost.
"""
import ctypes as C

import numpy as np
import pytest

import sgn
from test_gpu_parity import assert_same_run, ctxf, run_both, scenario  # noqa: F401 (ctxf: fixture)

pytestmark = pytest.mark.gpu


def _codel_args(n=300, codel=1):
    # slow down-links make CoDel queues stand (thousands of runs at the slow hosts); codel=1:
    # the pool starts at one page per host plus 64
    bw = np.where(np.arange(n) % 10 == 0, 100_000_000, 4_000_000).astype(np.uint64)
    return scenario(n=n, V=30, kind=sgn.TRAFFIC_TGEN, stop_ns=2_000_000_000, bw=bw, tor=True,
                    tgen_think=200_000_000, codel=codel)


def _pages_ok(info):
    assert info["codel_pages_free"] + info["codel_pages_chained"] == info["codel_pages"], info


@pytest.mark.parametrize("persistent,trace", [("1", False), ("0", False), ("0", True)])
def test_codel_pool_grows(ctxf, oracle, monkeypatch, persistent, trace):
    monkeypatch.setenv("SGN_PERSISTENT", persistent)
    args = _codel_args()
    o, c = run_both(ctxf, oracle, args, trace=trace)
    st, info = c.stats(), c.engine_info()
    assert st["codel_dropped"] > 0 and st["max_codel_len"] > 1000, st
    assert info["codel_pool_grows"] >= 1 and info["rounds_held"] >= 1, info
    assert info["codel_pages"] > args[2].n + 64, info
    assert (info["persistent_grid"] > 0) == (persistent == "1" and not trace), info
    _pages_ok(info)
    assert_same_run(o, c, args[2].n, trace=trace)


@pytest.mark.parametrize("persistent,trace,hpw", [("1", False, "64"), ("0", False, "32"), ("0", True, "64")])
def test_calendar_spill_relayout(ctxf, oracle, monkeypatch, persistent, trace, hpw):
    # 16-run slabs and two datagrams per host per 1-ms bucket to random peers: ~128 runs per
    # (bucket, host group) slab, so the first rounds spill and the calendar is re-laid out
    monkeypatch.setenv("SGN_PERSISTENT", persistent)
    monkeypatch.setenv("SGN_SLAB_CAP", "16")
    monkeypatch.setenv("SGN_HOSTS_PER_WAVE", hpw)
    n = 2000
    args = scenario(n=n, V=100, period_ns=500_000, stop_ns=150_000_000, bw=100_000_000)
    o, c = run_both(ctxf, oracle, args, trace=trace)
    info = c.engine_info()
    assert info["calendar_grows"] >= 1 and info["calendar_spill_runs"] > 0, info
    assert info["slab_capacity"] > 16 and info["rounds_held"] >= 1, info
    assert c.stats()["packets_sent"] > 100_000
    assert_same_run(o, c, n, trace=trace)


@pytest.mark.parametrize("slot", [1 << 16, 16])
def test_two_shards_grow_together(ctxf, oracle, monkeypatch, slot):
    """The multi-shard device path: every shard evaluates every shard's CoDel guard and spill
    flag from the round-edge messages, so both hold the same round; each grows its own pools
    (local shard-group transport on one GPU), identical to one unsharded shard. slot = 16:
    runs past a peer's exchange slot spill, the round is held on both shards, the slots grow
    alike and the round is exchanged again."""
    monkeypatch.setenv("SGN_SLAB_CAP", "16")
    if slot == 16:  # (every import through the slots: persistent rounds' inbox bins would take them)
        monkeypatch.setenv("SGN_XBIN", "0")
    n = 300
    args = _codel_args(n=n)
    g, used, hosts, cfg, tr = args
    one = ctxf()
    one.routes_build(g, used)
    one.hosts_set(hosts)
    one.sim_init(cfg, tr)
    one.run()
    # the unsharded run against the oracle first (so a failure below names the sharded side)
    lat, loss = oracle.routes(g, used)
    o = oracle.Sim(used, lat, loss, hosts, cfg, tr)
    o.run()
    assert_same_run(o, one, n, trace=False)
    shards = [ctxf(shard_rank=r, shard_count=2) for r in range(2)]
    arr = (C.c_void_p * 2)(*[s.h.value for s in shards])
    for s in shards:
        s.routes_build(g, used)
        s.hosts_set(hosts)
    shards[0].check(shards[0].L.sgn_comm_init_local(arr, 2, slot))
    for s in shards:
        s.sim_init(cfg, tr)
    done = C.c_uint64()
    shards[0].check(shards[0].L.sgn_run_local_group(arr, 2, 1 << 40, C.byref(done)))
    assert done.value == one.stats()["rounds"]
    held = [s.engine_info()["rounds_held"] for s in shards]
    assert held[0] == held[1] >= 1, held
    assert max(s.engine_info()["codel_pool_grows"] for s in shards) >= 1
    if slot == 16:
        info = [s.engine_info() for s in shards]
        if info[0]["exchange_mode"] == 2:  # persistent rounds: the inbox slots grow
            assert all(i["inbox_grows"] >= 1 for i in info), info
            assert info[0]["inbox_slot_runs"] == info[1]["inbox_slot_runs"] > 16
        else:
            assert all(i["exchange_slot_grows"] >= 1 for i in info)
            assert info[0]["exchange_slot_runs"] == info[1]["exchange_slot_runs"] > 16
    for r, s in enumerate(shards):
        lo, hi = C.c_uint32(), C.c_uint32()
        s.L.sgn_shard_range(n, r, 2, C.byref(lo), C.byref(hi))
        d1, d2 = one.digests(lo.value, hi.value), s.digests(lo.value, hi.value)
        for f in ("tx", "rx", "app", "rng", "next_event_id", "n_sent", "n_popped", "n_delivered",
                  "n_codel_dropped"):
            bad = np.nonzero(d1[f] != d2[f])[0] if d1[f].ndim == 1 else np.nonzero((d1[f] != d2[f]).any(1))[0]
            assert len(bad) == 0, (r, f, len(bad), lo.value + bad[:5], [x.engine_info() for x in shards])
        assert s.window() == one.window()
        _pages_ok(s.engine_info())


def test_bandwidths_beyond_32bit_increments(ctxf, oracle):
    """Token-bucket refill increments (bytes per ms) above 2^32 — a host above 34 Tbit/s — run
    bit-exact: the round kernels keep every per-host field at its full width (LaneRc), in
    registers for PERIODIC traffic and in LDS for TGEN, so no bandwidth the reference accepts
    is refused or truncated."""
    for kind in (sgn.TRAFFIC_PERIODIC, sgn.TRAFFIC_TGEN):
        n = 60
        args = list(scenario(n=n, V=8, kind=kind, stop_ns=60_000_000))
        bwv = np.full(n, 10_000_000, dtype=np.uint64)
        bwv[::7] = 40_000_000_000_000  # 40 Tbit/s: 5e9 bytes per ms
        h = args[2]
        args[2] = sgn.HostArrays(h.ip, h.node_id, bwv, bwv, h.seed)
        o, c = run_both(ctxf, oracle, tuple(args), trace=True)
        assert c.stats()["rounds"] > 0
        assert_same_run(o, c, n, trace=True)


# ---- hot slabs: fan-in beyond one slab and beyond one workgroup's LDS (a10) ----
def _hot_args(n, V=2, servers=4, stop_ns=300_000_000, think=1_000_000_000, seed=1):
    """Every client fetches a one-packet file from one of `servers` TGEN servers (HostIds
    0..servers-1: slots put servers first, so all of them share host group 0) at the same
    instant: the requests land in the servers' (bucket, group) slabs, ~n / V runs each — the
    fan-in the reference's unbounded per-host BinaryHeap takes (core/work/event_queue.rs:12,
    57-66; pushes from any thread, core/worker.rs:603-613)."""
    g = sgn.tor_graph(V, seed=3)
    used = np.arange(V)
    names = sgn.host_names(n)
    hosts = sgn.HostArrays(sgn.assign_ips(n), (np.arange(n) * 7) % V, np.full(n, 1_000_000_000, np.uint64),
                           np.full(n, 1_000_000_000, np.uint64), sgn.derive_seeds(seed, names))
    cfg = sgn.make_config(stop_ns, event_capacity=1 << 20, codel_cap=64)
    tr = sgn.make_traffic(sgn.TRAFFIC_TGEN, period_ns=think, period_jitter_ns=think, start_jitter_ns=0,
                          servers=np.arange(servers), file_bytes=(1000, 1400, 1400))
    return g, used, hosts, cfg, tr


@pytest.mark.parametrize("persistent,trace", [("1", False), ("0", False), ("0", True)])
def test_hot_slab_extension_and_pieces(ctxf, oracle, monkeypatch, persistent, trace):
    """16-run slabs that may grow to 32 (test hooks): ~600 request runs per (bucket, server
    group) slab spill, the re-layout gives the hot slabs extensions, and their gathers order the
    runs in pieces of at most 32 (radix-selected bounds on Shadow's key) — bit-exact, per packet
    when traced."""
    monkeypatch.setenv("SGN_PERSISTENT", persistent)
    monkeypatch.setenv("SGN_SLAB_CAP", "16")
    monkeypatch.setenv("SGN_SLAB_LIM", "32")
    n = 1200
    args = _hot_args(n)
    o, c = run_both(ctxf, oracle, args, trace=trace)
    info, st = c.engine_info(), c.stats()
    assert info["slab_extensions"] >= 1 and info["slab_extension_runs"] > 0, info
    assert info["big_slab_pieces"] > 10 and info["slab_capacity"] <= 32, info
    assert st["max_pending_events"] > 500, st
    assert (info["persistent_grid"] > 0) == (persistent == "1" and not trace), info
    assert_same_run(o, c, n, trace=trace)


def test_hot_slab_beyond_lds(ctxf, oracle):
    """No hooks: 12 k clients hit 4 servers at once, ~6 k request runs per (bucket, group) slab
    — more than one workgroup's LDS orders (sgn_engine_info.slab_capacity stays at the default
    since few slabs overflow). Persistent rounds, bit-exact against the oracle."""
    n = 12_000
    args = _hot_args(n)
    o, c = run_both(ctxf, oracle, args, trace=False)
    info, st = c.engine_info(), c.stats()
    assert st["max_pending_events"] > 4000, st
    assert info["big_slab_pieces"] > 0 and info["slab_extensions"] >= 1, info
    assert info["persistent_grid"] > 0 and info["persistent_fallbacks"] == 0, info
    assert_same_run(o, c, n, trace=False)


@pytest.mark.parametrize("defer", ["0", "1"])
def test_hot_slab_two_shards(ctxf, oracle, monkeypatch, defer):
    """The multi-shard device path with hot slabs: servers in shard 0, clients in both, so the
    requests of shard 1's clients reach the servers' slabs through k_import (local shard-group
    transport); identical to one unsharded shard. defer = 1: runs k_import spilled past a slab
    stay in the spill area until a round is held, as between the RCCL transport's batch syncs,
    so the next round's gathers read them there (the big-slab path's spill scan)."""
    monkeypatch.setenv("SGN_SLAB_CAP", "16")
    monkeypatch.setenv("SGN_SLAB_LIM", "32")
    monkeypatch.setenv("SGN_LOCAL_DEFER", defer)
    n = 1200
    args = _hot_args(n)
    g, used, hosts, cfg, tr = args
    one = ctxf()
    one.routes_build(g, used)
    one.hosts_set(hosts)
    one.sim_init(cfg, tr)
    one.run()
    lat, loss = oracle.routes(g, used)
    o = oracle.Sim(used, lat, loss, hosts, cfg, tr)
    o.run()
    assert_same_run(o, one, n, trace=False)
    shards = [ctxf(shard_rank=r, shard_count=2) for r in range(2)]
    arr = (C.c_void_p * 2)(*[s.h.value for s in shards])
    for s in shards:
        s.routes_build(g, used)
        s.hosts_set(hosts)
    shards[0].check(shards[0].L.sgn_comm_init_local(arr, 2, 1 << 16))
    for s in shards:
        s.sim_init(cfg, tr)
    done = C.c_uint64()
    shards[0].check(shards[0].L.sgn_run_local_group(arr, 2, 1 << 40, C.byref(done)))
    assert done.value == one.stats()["rounds"]
    assert shards[0].engine_info()["big_slab_pieces"] > 0
    for r, s in enumerate(shards):
        lo, hi = C.c_uint32(), C.c_uint32()
        s.L.sgn_shard_range(n, r, 2, C.byref(lo), C.byref(hi))
        d1, d2 = one.digests(lo.value, hi.value), s.digests(lo.value, hi.value)
        for f in ("tx", "rx", "app", "rng", "next_event_id", "n_sent", "n_popped", "n_delivered",
                  "n_codel_dropped"):
            bad = np.nonzero(d1[f] != d2[f])[0] if d1[f].ndim == 1 else np.nonzero((d1[f] != d2[f]).any(1))[0]
            assert len(bad) == 0, (r, f, len(bad), lo.value + bad[:5])
        assert s.window() == one.window()
