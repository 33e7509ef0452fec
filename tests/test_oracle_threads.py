"""The oracle's threaded round loop (worker threads over host chunks, per-host queue locks,
as the reference's thread-per-core scheduler with Mutex<EventQueue>) gives exactly the
single-threaded results: counters, per-host order-sensitive digests, traces and windows."""
import numpy as np
import pytest

import sgn


def workload(kind):
    n, V = 400, 30
    g = sgn.tor_graph(V, seed=6) if kind == "tgen" else sgn.random_graph(V, seed=6)
    used = np.arange(V)
    bw = np.where(np.arange(n) % 5 == 0, 100_000_000, 3_000_000).astype(np.uint64)
    return g, used, n, bw


@pytest.mark.parametrize("kind,dynamic", [("periodic", False), ("tgen", False), ("periodic", True)])
def test_threaded_oracle_matches_sequential(oracle, kind, dynamic):
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
    b = oracle.Sim(used, lat, loss, hosts, cfg, tr, trace=True, threads=4)
    a.run()
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
