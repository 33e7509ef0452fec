"""The oracle's threaded round loop (a persistent worker pool over host chunks, per-host queue
locks, as the reference's thread-per-core scheduler with Mutex<EventQueue>) and its
reference-faithful mode (hash-map lookups, the global packet-counter lock, heap packet copies)
give exactly the single-threaded optimised results: counters, per-host order-sensitive
digests, traces and windows. The same holds for the APSP restatement in both modes."""
import numpy as np
import pytest

import sgn


def workload(kind):
    n, V = 400, 30
    g = sgn.tor_graph(V, seed=6) if kind == "tgen" else sgn.random_graph(V, seed=6)
    used = np.arange(V)
    bw = np.where(np.arange(n) % 5 == 0, 100_000_000, 3_000_000).astype(np.uint64)
    return g, used, n, bw


@pytest.mark.parametrize("kind,dynamic,mode", [("periodic", False, "threads"), ("tgen", False, "threads"),
                                               ("periodic", True, "threads"), ("tgen", False, "faithful"),
                                               ("periodic", True, "faithful1")])
def test_threaded_oracle_matches_sequential(oracle, kind, dynamic, mode):
    g, used, n, bw = workload(kind)
    lat, loss = oracle.routes(g, used)
    hosts = sgn.HostArrays(sgn.assign_ips(n), (np.arange(n) * 7) % len(used), bw, bw,
                           oracle.host_seeds(1, sgn.host_names(n)))
    cfg = sgn.make_config(300_000_000, runahead_ns=0 if dynamic else 1_000_000, dynamic=dynamic,
                          codel_cap=1 << 14)
    if kind == "tgen":
        tr = sgn.make_traffic(sgn.TRAFFIC_TGEN, period_ns=40_000_000, period_jitter_ns=40_000_000,
                              start_jitter_ns=20_000_000, servers=np.arange(0, n, 10),
                              file_bytes=(20_000, 80_000, 300_000))
    else:
        tr = sgn.make_traffic(period_ns=1_000_000, start_jitter_ns=2_000_000, unknown_dst_permille=10)
    a = oracle.Sim(used, lat, loss, hosts, cfg, tr, trace=True)
    b = oracle.Sim(used, lat, loss, hosts, cfg, tr, trace=True, threads=1 if mode == "faithful1" else 4,
                   faithful=mode.startswith("faithful"))
    a.run()
    # switching modes and thread counts mid-run changes nothing either
    b.run(100)
    b.set_threads(3)
    b.run(50)
    b.set_faithful(mode == "threads")
    b.run()
    sa, sb = a.stats(), b.stats()
    assert sa["packets_sent"] > 1000
    assert sa == sb
    assert a.window() == b.window()
    da, db = a.digests(), b.digests()
    for f in da.dtype.names:
        assert np.array_equal(da[f], db[f]), f
    ta, tb = a.trace(), b.trace()
    ta = ta[np.lexsort((ta["seq"], ta["host"]))]
    tb = tb[np.lexsort((tb["seq"], tb["host"]))]
    assert np.array_equal(ta, tb)


@pytest.mark.parametrize("V,directed,seed", [(60, False, 1), (120, True, 2), (300, False, 3)])
def test_routes_modes_agree(oracle, V, directed, seed):
    g = sgn.random_graph(V, seed=seed, loss_frac=0.6)
    if directed:
        rs = np.concatenate([g.src, g.dst[: len(g.src) - V]])
        rd = np.concatenate([g.dst, g.src[: len(g.src) - V]])
        rl = np.concatenate([g.lat, g.lat[: len(g.src) - V][::-1]])
        rp = np.concatenate([g.loss, g.loss[: len(g.src) - V]])
        g = sgn.GraphArrays(g.node_id, rs, rd, rl, rp, True)
    used = np.sort(np.random.default_rng(seed).choice(V, size=V * 2 // 3, replace=False))
    l0, p0 = oracle.routes(g, used)
    for faithful in (False, True):
        for threads in (1, 4):
            l1, p1 = oracle.routes(g, used, faithful=faithful, threads=threads)
            assert np.array_equal(l0, l1) and np.array_equal(p0.view(np.uint32), p1.view(np.uint32))
    disc = sgn.GraphArrays([0, 1, 2], [0, 1, 2], [0, 1, 2], [1, 1, 1], [0, 0, 0], False)
    for faithful in (False, True):
        with pytest.raises(sgn.SgnError, match="0 -> 2 are not connected"):
            oracle.routes(disc, [0, 2], faithful=faithful, threads=2)


def test_round_robin_qdisc_interleaves_sockets(oracle):
    """experimental.interface_qdisc: with FIFO a server sends its response trains (one socket
    each) one after another; with round-robin the interface takes one packet per socket in
    turn (host/network/interface.rs:216-256, queuing.rs:57-180)."""
    g, used, n, bw = workload("tgen")
    lat, loss = oracle.routes(g, used)
    hosts = sgn.HostArrays(sgn.assign_ips(n), (np.arange(n) * 7) % len(used), bw, bw,
                           oracle.host_seeds(1, sgn.host_names(n)))
    tr = sgn.make_traffic(sgn.TRAFFIC_TGEN, period_ns=5_000_000, period_jitter_ns=5_000_000,
                          start_jitter_ns=5_000_000, servers=np.arange(0, n, 10),
                          file_bytes=(20_000, 80_000, 300_000))
    alternations = {}
    for qd in (sgn.QDISC_FIFO, sgn.QDISC_ROUND_ROBIN):
        cfg = sgn.make_config(150_000_000, codel_cap=1 << 14, qdisc=qd)
        o = oracle.Sim(used, lat, loss, hosts, cfg, tr, trace=True)
        o.run()
        t = o.trace()
        t = t[np.lexsort((t["seq"], t["host"]))]
        s = t[(t["kind"] == 1) & (t["flags"] == 0) & (t["host"] % 10 == 0)]  # servers' sends
        # consecutive sends of one server at one time to different peers that come back
        same = (s["host"][2:] == s["host"][:-2]) & (s["a"][2:] == s["a"][:-2])
        alt = same & (s["peer"][2:] == s["peer"][:-2]) & (s["peer"][1:-1] != s["peer"][2:])
        alternations[qd] = int(alt.sum())
        assert o.stats()["packets_sent"] > 1000
    assert alternations[sgn.QDISC_FIFO] == 0
    assert alternations[sgn.QDISC_ROUND_ROBIN] > 100
