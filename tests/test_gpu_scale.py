"""GPU parity at the sizes BASELINE.json names (north_star: bit-exact at 100k simulated hosts),
and the calendar-horizon case of dynamic runahead. libsgn through the C ABI against the
oracle (threaded: the same results as one thread, tests/test_oracle_threads.py) on identical
seeds and graphs: every stats counter, the final window, and every host's order-sensitive
digests (tx = every send_packet outcome with its delivery time, rx = every packet event in pop
order, app = every delivery / CoDel drop), RNG state and next event id.
"""
import os
import pathlib
import sys

import numpy as np
import pytest

import sgn

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parent.parent
THREADS = max(1, min(16, os.cpu_count() or 1))
SKIP_STATS = ("max_pending_events", "sched_heavy_hosts", "sched_sorted_segments", "event_runs")
DIGEST_FIELDS = ("tx", "rx", "app", "rng", "next_event_id", "n_sent", "n_popped", "n_delivered",
                 "n_codel_dropped")


def _compare(o, c, n):
    so, sg = o.stats(), c.stats()
    for k in so:
        if k not in SKIP_STATS:
            assert so[k] == sg[k], (k, so[k], sg[k])
    assert o.window() == c.window()
    for lo in range(0, n, 50_000):
        hi = min(n, lo + 50_000)
        do, dg = o.digests(lo, hi), c.digests(lo, hi)
        for f in DIGEST_FIELDS:
            bad = np.nonzero(do[f] != dg[f])[0]
            assert len(bad) == 0, (f, lo + bad[:5])
    return sg


def _run_pair(oracle, g, used, hosts, cfg, tr, rounds=None):
    lat, loss = oracle.routes(g, used)
    o = oracle.Sim(used, lat, loss, hosts, cfg, tr, threads=THREADS)
    c = sgn.Context()
    c.routes_build(g, used)
    glat, gloss = c.routes_copy()
    assert np.array_equal(lat, glat) and np.array_equal(loss.view(np.uint32), gloss.view(np.uint32))
    c.hosts_set(hosts)
    c.sim_init(cfg, tr)
    if rounds is None:
        o.run()
        c.run()
    else:
        assert o.run(rounds) == rounds
        assert c.run(rounds) == rounds
    return o, c


def test_config_c_100k_hosts_bit_exact(oracle):
    """Config C (BASELINE.json configs[2]) exactly as bench.py builds it: 100k hosts, Zipf
    placement on a 1000-node complete Tor-like graph, bandwidth classes, 10 % servers, tgen
    trains through token buckets and CoDel; 1000 rounds (1 simulated second)."""
    sys.path.insert(0, str(ROOT))
    import bench
    g, used, hosts, cfg, tr = bench.build_workload(100_000, 1000)
    o, c = _run_pair(oracle, g, used, hosts, cfg, tr, rounds=1000)
    st = _compare(o, c, hosts.n)
    assert st["rounds"] == 1000
    assert st["packets_sent"] > 3_000_000 and st["packet_events_popped"] > 3_000_000
    assert st["packets_loss_dropped"] > 0 and st["codel_dropped"] > 0


def test_config_b_10k_hosts_full_10s(oracle):
    """Config B (configs[1]) in full: 10k hosts on a 1000-node random graph (mean degree 6,
    20 % lossy edges), UDP 1024 B every 10 ms to seeded random peers, 100 Mbit, 10 s."""
    n, V = 10_000, 1000
    g = sgn.random_graph(V, seed=42)
    used = np.arange(V)
    seeds = sgn.derive_seeds(1, sgn.host_names(n))
    bw = np.full(n, 100_000_000, dtype=np.uint64)
    hosts = sgn.HostArrays(sgn.assign_ips(n), np.arange(n) % V, bw, bw, seeds)
    cfg = sgn.make_config(10_000_000_000, out_fifo_cap=64, codel_cap=4096, event_capacity=1 << 22)
    tr = sgn.make_traffic(sgn.TRAFFIC_PERIODIC, flow_seed=7, period_ns=10_000_000,
                          start_jitter_ns=10_000_000, payload_len=1024, unknown_dst_permille=1)
    o, c = _run_pair(oracle, g, used, hosts, cfg, tr)
    st = _compare(o, c, n)
    assert st["packets_sent"] > 9_000_000 and st["packets_loss_dropped"] > 0


def test_dynamic_runahead_slow_paths_calendar_horizon(oracle):
    """Dynamic runahead where every used path is far slower than the smallest route latency
    (1 ms self-loops): windows of ~200 ms and deliveries up to ~700 ms past the window start,
    more than max_latency / bucket width buckets ahead (the calendar must cover
    window + max latency)."""
    V, n = 24, 240
    rng = np.random.default_rng(8)
    iu, ju = np.triu_indices(V, 1)
    lat = rng.integers(200_000, 480_000, len(iu)).astype(np.uint64) * 1000
    loss = np.round(rng.uniform(0, 0.01, len(iu)), 6).astype(np.float32)
    g = sgn.GraphArrays(np.arange(V), np.concatenate([iu, np.arange(V)]), np.concatenate([ju, np.arange(V)]),
                        np.concatenate([lat, np.full(V, 1_000_000, np.uint64)]),
                        np.concatenate([loss, np.zeros(V, np.float32)]), False)
    used = np.arange(V)
    # servers on nodes 0..3, clients on nodes 4..V-1: no host ever talks over a self-loop
    node = np.where(np.arange(n) % 10 == 0, (np.arange(n) // 10) % 4, 4 + np.arange(n) % (V - 4))
    seeds = sgn.derive_seeds(3, sgn.host_names(n))
    bw = np.full(n, 50_000_000, dtype=np.uint64)
    hosts = sgn.HostArrays(sgn.assign_ips(n), node, bw, bw, seeds)
    cfg = sgn.make_config(6_000_000_000, runahead_ns=0, dynamic=True, out_fifo_cap=64, codel_cap=4096,
                          event_capacity=1 << 20)
    tr = sgn.make_traffic(sgn.TRAFFIC_TGEN, period_ns=100_000_000, period_jitter_ns=300_000_000,
                          start_jitter_ns=100_000_000, servers=np.arange(0, n, 10),
                          file_bytes=(10 * 1024, 60 * 1024, 200 * 1024))
    o, c = _run_pair(oracle, g, used, hosts, cfg, tr)
    st = _compare(o, c, n)
    assert st["min_used_latency_ns"] >= 200_000_000
    info = c.engine_info()
    # windows of min_used (>= 200 buckets) plus the longest path must fit the calendar
    assert info["calendar_buckets"] * info["bucket_width_ns"] > 2 * 480_000_000
    assert st["packets_sent"] > 10_000


def test_config_d_1m_hosts_bit_exact(oracle):
    """Config D (configs[3]) at its full size on one GPU: 1M hosts, every host sends 64 B to a
    uniform random peer every 1 ms (dense all-to-all; 15,625 host groups, so every workgroup
    of the persistent round kernel serves ~9 groups per round). 320 rounds: ~320M sends, and
    past the first deliveries of the longest paths the steady state — every host popping about
    one packet a round through its CoDel queue and relay (host.rs:762-830, event_queue.rs:57-90)
    — for the last ~200 rounds."""
    sys.path.insert(0, str(ROOT))
    import bench
    g, used, hosts, cfg, tr = bench.build_workload_d(1_000_000, 1000)
    cfg.event_capacity = 257 * (1_000_000 // 64 + 1) * 128
    rounds = 320
    o, c = _run_pair(oracle, g, used, hosts, cfg, tr, rounds=rounds)
    st = _compare(o, c, hosts.n)
    assert st["packets_sent"] > 300_000_000
    # steady-state receive: most of the sends of the first ~200 rounds have been popped
    assert st["packet_events_popped"] > 150_000_000, st["packet_events_popped"]
    info = c.engine_info()
    assert info["host_groups"] == 15_625 and info["persistent_fallbacks"] == 0
