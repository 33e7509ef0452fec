"""Persistent multi-shard rounds (k_rounds_x): N shards, each a range of workgroups of
ONE launch on one GPU — the device code of the N-GPU path (direct stores into the receivers'
inboxes: bins per receiving host group, read by its next gather, and per-sender slots; per-round
tagged messages, every shard computing the same window from the N messages), with the inboxes in
ordinary device memory instead of peer-mapped uncached memory. Each run is checked against ONE unsharded run (itself
checked against the oracle by the other GPU tests) and, for config C, against the oracle:
every host's digests, every counter and the window, bit for bit."""
import ctypes as C
import os
import pathlib
import sys

import numpy as np
import pytest

import sgn
from test_gpu_parity import scenario

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parent.parent
DIGESTS = ("tx", "rx", "app", "rng", "next_event_id", "n_sent", "n_popped", "n_delivered", "n_codel_dropped")
ADD = ("packets_sent", "packets_loss_dropped", "packets_unknown_dst", "packet_events_popped", "delivered",
       "codel_dropped", "local_events", "local_delivered", "app_blocked", "bytes_delivered", "host_executions")


def local_group(args, k, slot=1 << 14, rounds=1 << 40, event_capacity=None):
    """k shards of the scenario as one local group (one launch per batch of rounds)."""
    g, used, hosts, cfg, tr = args
    shards = [sgn.Context(shard_rank=r, shard_count=k, flags=2) for r in range(k)]
    arr = (C.c_void_p * k)(*[c.h.value for c in shards])
    for c in shards:
        c.routes_build(g, used)
        c.hosts_set(hosts)
    shards[0].check(shards[0].L.sgn_comm_init_local(arr, k, slot))
    if event_capacity is not None:
        cfg = type(cfg).from_buffer_copy(cfg)
        cfg.event_capacity = event_capacity
    for c in shards:
        c.sim_init(cfg, tr)
    done = C.c_uint64()
    shards[0].check(shards[0].L.sgn_run_local_group(arr, k, rounds, C.byref(done)))
    return shards, arr, done.value


def unsharded(args, rounds=1 << 40):
    g, used, hosts, cfg, tr = args
    c = sgn.Context(flags=2)
    c.routes_build(g, used)
    c.hosts_set(hosts)
    c.sim_init(cfg, tr)
    c.run(rounds)
    return c


def compare(one, shards, n):
    k = len(shards)
    s1 = one.stats()
    tot = {key: 0 for key in ADD}
    for r, c in enumerate(shards):
        lo, hi = C.c_uint32(), C.c_uint32()
        c.L.sgn_shard_range(n, r, k, C.byref(lo), C.byref(hi))
        d1, d2 = one.digests(lo.value, hi.value), c.digests(lo.value, hi.value)
        for f in DIGESTS:
            bad = np.nonzero(d1[f] != d2[f])[0] if d1[f].ndim == 1 else np.nonzero((d1[f] != d2[f]).any(1))[0]
            assert len(bad) == 0, (r, f, lo.value + bad[:5])
        assert c.window() == one.window(), r
        st = c.stats()
        assert st["rounds"] == s1["rounds"], r
        for key in ADD:
            tot[key] += st[key]
    for key in ADD:
        assert tot[key] == s1[key], (key, tot[key], s1[key])
    return s1


@pytest.mark.parametrize("k", [2, 3, 8])
@pytest.mark.parametrize("kind,dynamic", [("periodic", False), ("tgen", False), ("periodic", True)])
def test_xpersist_shards_match_single(k, kind, dynamic):
    n = 400
    if kind == "tgen":
        bw = np.where(np.arange(n) % 10 == 0, 100_000_000, 4_000_000).astype(np.uint64)
        args = scenario(n=n, V=30, kind=sgn.TRAFFIC_TGEN, stop_ns=600_000_000, bw=bw, tor=True,
                        tgen_think=100_000_000)
    else:
        args = scenario(n=n, dynamic=dynamic, runahead_ns=0 if dynamic else 1_000_000, stop_ns=300_000_000)
    one = unsharded(args)
    shards, _, done = local_group(args, k)
    info = shards[0].engine_info()
    if info["calendar_buckets"] <= 256:  # (longer calendars run per-round launches, as on one shard)
        assert info["exchange_mode"] == 2 and info["persistent_x_launches"] > 0, info
        assert shards[0].kernel_times()["k_rounds_x"][0] > 0
    else:
        assert info["exchange_mode"] == 1 and one.engine_info()["persistent_grid"] == 0
    s1 = compare(one, shards, n)
    assert s1["packets_sent"] > 1000 and done == s1["rounds"]


@pytest.mark.parametrize("xown", ["0", "1", "16"])
def test_xpersist_import_modes(monkeypatch, xown):
    """A round's imports are filed by the receiving shard's workgroups either for their own
    groups at the next round's start (few: no second barrier) or shared out before a second local
    barrier (many); SGN_XOWN moves the threshold (0: always shared) — identical either way."""
    monkeypatch.setenv("SGN_XOWN", xown)
    n = 500
    bw = np.where(np.arange(n) % 10 == 0, 100_000_000, 4_000_000).astype(np.uint64)
    args = scenario(n=n, V=30, kind=sgn.TRAFFIC_TGEN, stop_ns=400_000_000, bw=bw, tor=True, tgen_think=50_000_000)
    one = unsharded(args)
    shards, _, _ = local_group(args, 4)
    assert shards[0].engine_info()["exchange_mode"] == 2
    compare(one, shards, n)


def test_xpersist_matches_per_round_group(monkeypatch):
    """The same group through the per-round launches and local copies (SGN_LOCAL_PERSIST=0) and
    through k_rounds_x: identical."""
    args = scenario(n=300, V=40, stop_ns=200_000_000, unknown=20)
    a, _, _ = local_group(args, 3)
    monkeypatch.setenv("SGN_LOCAL_PERSIST", "0")
    b, _, _ = local_group(args, 3)
    assert b[0].engine_info()["exchange_mode"] == 1
    assert a[0].engine_info()["exchange_mode"] == 2
    for r in range(3):
        lo, hi = C.c_uint32(), C.c_uint32()
        a[r].L.sgn_shard_range(300, r, 3, C.byref(lo), C.byref(hi))
        da, db = a[r].digests(lo.value, hi.value), b[r].digests(lo.value, hi.value)
        for f in DIGESTS:
            assert np.array_equal(da[f], db[f]), (r, f)
        assert a[r].stats()["packets_sent"] == b[r].stats()["packets_sent"]


@pytest.mark.parametrize("islot", [1, 6, 64])
def test_xpersist_inbox_overflow_and_growth(monkeypatch, islot):
    """Inbox slots far below a round's exports (no bins: SGN_XBIN=0, every import through the
    slots): runs past a slot wait in the sender's spill area, the round edge is held on every
    shard, the host moves them into their shards' calendars and grows every inbox; slots filled
    past half are grown before the next round. Bit-exact."""
    monkeypatch.setenv("SGN_XBIN", "0")
    monkeypatch.setenv("SGN_XISLOT", str(islot))
    n = 500
    bw = np.where(np.arange(n) % 10 == 0, 100_000_000, 4_000_000).astype(np.uint64)
    args = scenario(n=n, V=30, kind=sgn.TRAFFIC_TGEN, stop_ns=400_000_000, bw=bw, tor=True, tgen_think=50_000_000)
    monkeypatch.delenv("SGN_XISLOT")
    one = unsharded(args)
    monkeypatch.setenv("SGN_XISLOT", str(islot))
    shards, _, _ = local_group(args, 4)
    info = [c.engine_info() for c in shards]
    assert all(i["exchange_mode"] == 2 for i in info)
    if islot <= 6:
        assert info[0]["inbox_grows"] > 0 and info[0]["inbox_slot_runs"] > islot, info[0]
    if islot == 1:
        assert info[0]["inbox_overflow_rounds"] > 0 and sum(i["inbox_moved_runs"] for i in info) > 0, info
    compare(one, shards, n)


@pytest.mark.parametrize("xbin,islot", [("1", None), ("2", "1"), ("4", None)])
def test_xpersist_inbox_bins(monkeypatch, xbin, islot):
    """The inbox bins (runs binned by receiving host group, read by that group's next gather):
    bins of 1, 2 and 4 runs overflow into the slots every round (and, with 1-run slots, past
    them into the senders' spill areas: held rounds, moved runs, grown inboxes); runs due in the
    window they arrive for go into their slabs ahead of the gathers. Bit-exact either way."""
    n = 500
    bw = np.where(np.arange(n) % 10 == 0, 100_000_000, 4_000_000).astype(np.uint64)
    args = scenario(n=n, V=30, kind=sgn.TRAFFIC_TGEN, stop_ns=400_000_000, bw=bw, tor=True, tgen_think=50_000_000)
    one = unsharded(args)
    monkeypatch.setenv("SGN_XBIN", xbin)
    if islot:
        monkeypatch.setenv("SGN_XISLOT", islot)
    shards, _, _ = local_group(args, 4)
    info = [c.engine_info() for c in shards]
    assert all(i["exchange_mode"] == 2 for i in info)
    if islot:
        assert max(i["inbox_overflow_rounds"] for i in info) > 0, info
    compare(one, shards, n)


def test_xpersist_hot_fan_in(monkeypatch):
    """Clients on every shard fetching from a few servers on shard 0 within one bucket width
    (16-run slabs that may grow to 32: test hooks): imported runs past their slab's capacity go to
    the spill area, the next round's gathers read them there and order the hot slabs in pieces
    (the big-slab path), and the spill flag holds the round after for the re-layout, which gives
    the hot slabs extensions."""
    from test_gpu_pools import _hot_args
    monkeypatch.setenv("SGN_SLAB_CAP", "16")
    monkeypatch.setenv("SGN_SLAB_LIM", "32")
    n = 1600
    args = _hot_args(n)
    one = unsharded(args)
    shards, _, done = local_group(args, 4)
    assert shards[0].engine_info()["exchange_mode"] == 2
    assert shards[0].engine_info()["big_slab_pieces"] > 0
    assert sum(c.engine_info()["calendar_spill_runs"] for c in shards) > 0
    compare(one, shards, n)


def test_config_c_eight_shards_one_launch(oracle):
    """Config C exactly as bench.py builds it (100k hosts, Tor-like 1000-node graph, tgen
    trains) as 8 shards of 12.5k hosts in ONE launch per batch of rounds — the driver's N = 8
    configuration rehearsed on one GPU: bit-exact against one unsharded run and the oracle over
    600 rounds; the per-round time of both is printed."""
    sys.path.insert(0, str(ROOT))
    import bench
    g, used, hosts, cfg, tr = bench.build_workload(100_000, 1000)
    rounds = 600
    one = unsharded((g, used, hosts, cfg, tr), rounds=rounds)
    c8 = type(cfg).from_buffer_copy(cfg)
    c8.event_capacity = -(-cfg.event_capacity // 8)
    shards, _, done = local_group((g, used, hosts, c8, tr), 8, slot=1 << 13, rounds=rounds)
    assert done == rounds
    s1 = compare(one, shards, hosts.n)
    assert s1["packets_sent"] > 1_500_000
    lat, loss = oracle.routes(g, used)
    o = oracle.Sim(used, lat, loss, hosts, cfg, tr, threads=max(1, min(16, os.cpu_count() or 1)))
    assert o.run(rounds) == rounds
    so = o.stats()
    for key in ADD:
        assert so[key] == s1[key], key
    assert o.window() == one.window()
    for lo in range(0, hosts.n, 50_000):
        do, d1 = o.digests(lo, lo + 50_000), one.digests(lo, lo + 50_000)
        for f in DIGESTS:
            assert np.array_equal(do[f], d1[f]), (lo, f)
    kt1, kt8 = one.kernel_times()["k_rounds"], shards[0].kernel_times()["k_rounds_x"]
    print(f"per-round kernel time: unsharded {kt1[1] / rounds * 1e3:.2f} us, 8 shards in one launch "
          f"{kt8[1] / rounds * 1e3:.2f} us (grid {[c.engine_info()['persistent_x_grid'] for c in shards]})")


def test_config_d_1m_eight_shards_one_launch():
    """Config D as bench.py builds it (1M hosts, every host sending 64 B to a uniform random peer
    every 1 ms: 7/8 of all runs cross shards) as 8 shards of 125k hosts in ONE k_rounds_x launch
    per batch — the round-edge exchange BASELINE's config #4 stresses, rehearsed on one GPU —
    for 320 rounds, past the first deliveries into the steady state where every host pops about
    one imported packet a round (worker.rs:603-613 is the cross-host push the inbox replaces).
    Bit for bit against one unsharded run (itself checked against the oracle at the same size,
    test_gpu_scale.py::test_config_d_1m_hosts_bit_exact); the inboxes grow under this load."""
    sys.path.insert(0, str(ROOT))
    import bench
    n, k, rounds = 1_000_000, 8, 320
    g, used, hosts, cfg, tr = bench.build_workload_d(n, 1000)
    cfg.event_capacity = 257 * (n // 64 + 1) * 128
    one = unsharded((g, used, hosts, cfg, tr), rounds=rounds)
    s1 = one.stats()
    assert s1["rounds"] == rounds
    shards, _, done = local_group((g, used, hosts, cfg, tr), k, slot=1 << 13, rounds=rounds,
                                  event_capacity=257 * (-(-n // k) // 64 + 1) * 128)
    assert done == rounds
    info = [c.engine_info() for c in shards]
    assert all(i["exchange_mode"] == 2 for i in info), info[0]
    compare(one, shards, n)
    assert s1["packets_sent"] > 300_000_000 and s1["packet_events_popped"] > 150_000_000
    kt1, kt8 = one.kernel_times()["k_rounds"], shards[0].kernel_times()["k_rounds_x"]
    print(f"config D per-round kernel time: unsharded {kt1[1] / rounds * 1e3:.1f} us, 8 shards in one launch "
          f"{kt8[1] / rounds * 1e3:.1f} us; inbox slot {info[0]['inbox_slot_runs']} runs, grown "
          f"{info[0]['inbox_grows']}x, hwm {info[0]['exchange_hwm_runs']}")
