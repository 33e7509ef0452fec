"""GPU parity: libsgn (HIP, gfx950) against the oracle on identical inputs.

Bar (BASELINE.json north_star): bit-exact routing tables, per-packet delivery times, drop
decisions and event order. Small cases compare full per-packet traces; larger cases
compare per-host order-sensitive digests ("checksum of checksums") and counters.
"""
import numpy as np
import pytest

import sgn

pytestmark = pytest.mark.gpu

SIM_START = sgn.SIMULATION_START


@pytest.fixture(scope="module")
def ctxf():
    def make(**kw):
        return sgn.Context(**kw)
    return make


def ref_graph(directed):
    # network/graph/mod.rs:559-644 test_shortest_path
    node = np.array([0, 1, 2])
    src = [0, 1, 2, 0, 1, 0, 2]
    dst = [0, 1, 2, 1, 0, 2, 1]
    lat = [3333, 5555, 7777, 3, 5, 7, 11]
    return sgn.GraphArrays(node, src, dst, lat, np.zeros(7, np.float32), directed)


@pytest.mark.parametrize("directed", [True, False])
def test_apsp_reference_shortest_path(ctxf, directed):
    c = ctxf()
    c.routes_build(ref_graph(directed), [0, 1, 2])
    lat, _ = c.routes_copy()
    if directed:
        exp = [[3333, 3, 7], [5, 5555, 12], [16, 11, 7777]]
    else:
        exp = [[3333, 3, 7], [3, 5555, 10], [7, 10, 7777]]
    assert lat.tolist() == exp


@pytest.mark.parametrize("V,directed,seed", [(16, False, 1), (100, False, 2), (100, True, 3),
                                             (333, False, 4), (1000, False, 42)])
def test_apsp_random_vs_oracle(ctxf, oracle, V, directed, seed):
    g = sgn.random_graph(V, seed=seed, loss_frac=0.5)
    if directed:
        # add reverse arcs so the directed graph stays strongly connected
        rs = np.concatenate([g.src, g.dst[: len(g.src) - V]])
        rd = np.concatenate([g.dst, g.src[: len(g.src) - V]])
        rl = np.concatenate([g.lat, g.lat[: len(g.src) - V][::-1]])
        rp = np.concatenate([g.loss, g.loss[: len(g.src) - V]])
        g = sgn.GraphArrays(g.node_id, rs, rd, rl, rp, True)
    rng = np.random.default_rng(seed)
    used = np.sort(rng.choice(V, size=max(2, V * 3 // 4), replace=False))
    ol, op = oracle.routes(g, used)
    c = ctxf()
    c.routes_build(g, used)
    gl, gp = c.routes_copy()
    assert np.array_equal(ol, gl)
    assert np.array_equal(op.view(np.uint32), gp.view(np.uint32))
    assert c.routes_timing()["latency_bf"] == 1  # sparse: per-source relaxation


def test_apsp_complete_graph_vs_oracle(ctxf, oracle):
    g = sgn.tor_graph(200, seed=9)
    used = np.arange(200)
    ol, op = oracle.routes(g, used)
    c = ctxf()
    c.routes_build(g, used)
    gl, gp = c.routes_copy()
    assert np.array_equal(ol, gl)
    assert np.array_equal(op.view(np.uint32), gp.view(np.uint32))
    # direct-path mode (use_shortest_path: false) on the same complete graph
    ol2, op2 = oracle.routes(g, used, shortest=False)
    c.routes_build(g, used, shortest=False)
    gl2, gp2 = c.routes_copy()
    assert np.array_equal(ol2, gl2)
    assert np.array_equal(op2.view(np.uint32), gp2.view(np.uint32))


def test_apsp_paths_beyond_u32_fall_back(ctxf, oracle, monkeypatch):
    """Paths of 2^32 ns (4.29 s) or more: the u32 min-plus form (forced with SGN_APSP_SQ on this
    sparse graph) cannot hold them, the build redoes the latency phase with the u64
    Floyd-Warshall; the sparse graph's own form, per-source relaxation in u64, is exact anyway."""
    V = 40
    g = sgn.random_graph(V, seed=5, lat_lo_us=1_500_000, lat_hi_us=3_500_000)  # 1.5-3.5 s edges
    used = np.arange(V)
    ol, op = oracle.routes(g, used)
    assert ol.max() >= 1 << 32
    c = ctxf()
    c.routes_build(g, used)  # sparse: per-source relaxation
    gl, gp = c.routes_copy()
    assert np.array_equal(ol, gl) and np.array_equal(op.view(np.uint32), gp.view(np.uint32))
    assert c.routes_timing()["latency_bf"] == 1
    monkeypatch.setenv("SGN_APSP_SQ", "1")
    c.routes_build(g, used)
    gl, gp = c.routes_copy()
    assert np.array_equal(ol, gl) and np.array_equal(op.view(np.uint32), gp.view(np.uint32))
    t = c.routes_timing()
    assert t["latency_u64"] == 1 and t["latency_bf"] == 0
    c.routes_build(sgn.random_graph(V, seed=5), used)
    t = c.routes_timing()
    assert t["latency_u64"] == 0 and 1 <= t["latency_passes"] <= 8 and t["latency_bf"] == 0


def test_apsp_squaring_one_launch_many_passes(ctxf, oracle, monkeypatch):
    """sq_run (every squaring pass in one launch, grid barrier between passes, K split over four
    slices per workgroup) on graphs whose direct edges are NOT their shortest paths, so several
    passes change entries across many tiles (cross-XCD hand-offs between passes): a complete graph
    with random latencies (CSR row build, sq_rows) and a sparse graph forced onto the squaring
    form (V = 1000: 256 tiles, ~10 passes); against the oracle and against one launch per pass
    (SGN_APSP_SQ_PASSES)."""
    V = 700
    rng = np.random.default_rng(11)
    iu, ju = np.triu_indices(V, 1)
    lat = rng.integers(1_000, 100_000, len(iu)).astype(np.uint64) * 1000
    loss = np.round(rng.uniform(0, 0.01, len(iu)), 6).astype(np.float32)
    dense = sgn.GraphArrays(np.arange(V), np.concatenate([iu, np.arange(V)]), np.concatenate([ju, np.arange(V)]),
                            np.concatenate([lat, np.full(V, 1_000_000, np.uint64)]),
                            np.concatenate([loss, np.zeros(V, np.float32)]), False)
    cases = [(dense, {}), (sgn.random_graph(1000, seed=21, loss_frac=0.5), {"SGN_APSP_SQ": "1"})]
    for k, (g, env) in enumerate(cases):
        used = np.arange(len(g.node_id))
        ol, op = oracle.routes(g, used)
        passes = []
        for one in (True, False):
            for key, val in env.items():
                monkeypatch.setenv(key, val)
            if not one:
                monkeypatch.setenv("SGN_APSP_SQ_PASSES", "1")
            c = ctxf()
            c.routes_build(g, used)
            t = c.routes_timing()
            for key in list(env) + ([] if one else ["SGN_APSP_SQ_PASSES"]):
                monkeypatch.delenv(key)
            gl, gp = c.routes_copy()
            assert np.array_equal(ol, gl) and np.array_equal(op.view(np.uint32), gp.view(np.uint32)), (k, one)
            assert t["latency_bf"] == 0 and t["latency_u64"] == 0, (k, t)
            passes.append(t["latency_passes"])
        assert min(passes) >= 2, (k, passes)  # (in place, the two forms may converge a pass apart)


def test_apsp_loss_forms_agree(ctxf, oracle, monkeypatch):
    """The loss phase's multi-source arc sweep (complete graphs; 48 KB of rows per workgroup
    at V = 1500) against the oracle and against the one-source kernel (SGN_APSP_LOSS1; sparse
    graphs take it anyway), and a graph whose sources have more tight arcs than a list holds
    (complete bipartite layers of equal latency: |A| x |B| ties), which falls back to it."""
    cases = [sgn.tor_graph(600, seed=3), sgn.tor_graph(1500, seed=4), sgn.random_graph(1500, seed=8, loss_frac=0.5)]
    a, b = 90, 90  # s -> A (1 ms) -> B (1 ms): every A x B arc is tight for s
    src = [0] * a + [1 + i for i in range(a) for _ in range(b)]
    dst = list(range(1, a + 1)) + [1 + a + j for _ in range(a) for j in range(b)]
    n = 1 + a + b
    rng = np.random.default_rng(1)
    lossy = np.round(rng.uniform(0, 0.01, len(src)), 6).astype(np.float32)
    cases.append(sgn.GraphArrays(np.arange(n), src + list(range(n)), dst + list(range(n)),
                                 [1_000_000] * len(src) + [1_000_000] * n,
                                 np.concatenate([lossy, np.zeros(n, np.float32)]), False))
    for k, g in enumerate(cases):
        used = np.arange(len(g.node_id))
        ol, op = oracle.routes(g, used)
        forms = []
        for env in ({}, {"SGN_APSP_LOSS1": "1"}):
            for key, val in env.items():
                monkeypatch.setenv(key, val)
            c = ctxf()
            c.routes_build(g, used)
            forms.append(c.routes_timing()["loss_multi"])
            for key in env:
                monkeypatch.delenv(key)
            gl, gp = c.routes_copy()
            assert np.array_equal(ol, gl) and np.array_equal(op.view(np.uint32), gp.view(np.uint32)), (k, env)
        assert forms[1] == 0
        assert (forms[0] >= 4) == (k < 2), (k, forms)  # sparse graph / list overflow: one-source


def test_apsp_dense_sweep_form(ctxf, oracle, monkeypatch):
    """The dense form of the loss sweep (loss_sweep_dense: a lane per head, the S sources'
    d[s][v] in registers, -d[s][u] by scalar loads, negated latency and arc-index matrices; the
    sources' own out-arcs by loss_self_tails) and its fused form (the sweep on the direct arcs
    before the squaring, as its first pass: complete graphs) against the oracle, against the
    unfused dense sweep (SGN_APSP_FUSED=0) and against the CSR sweep (SGN_APSP_DENSE=0):
    - Tor graphs: complete, every arc its own shortest path — fused, nothing to shorten;
    - points on a line (complete, every collinear triple a tie): fused, tight arcs through
      other tails in nearly every wave step;
    - a complete graph with random latencies and a directed complete graph: the fused pass finds
      paths to shorten, the squaring runs and the loss phase sweeps the final matrix;
    - a used subset of the nodes (padded source tiles, sources that are not tails 0..U-1), the
      other workgroup shapes (unfused), and a dense graph with one parallel arc (CSR form)."""
    V = 300
    rng = np.random.default_rng(5)
    iu, ju = np.triu_indices(V, 1)
    lat = rng.integers(1, 40, len(iu)).astype(np.uint64) * 1_000_000  # coarse: many ties
    loss = np.round(rng.uniform(0, 0.02, len(iu)), 6).astype(np.float32)
    rand_c = sgn.GraphArrays(np.arange(V), np.concatenate([iu, np.arange(V)]), np.concatenate([ju, np.arange(V)]),
                             np.concatenate([lat, np.full(V, 1_000_000, np.uint64)]),
                             np.concatenate([loss, np.zeros(V, np.float32)]), False)
    Vd = 200
    ii, jj = np.nonzero(~np.eye(Vd, dtype=bool))
    dlat = rng.integers(1, 60, len(ii)).astype(np.uint64) * 500_000
    dloss = np.round(rng.uniform(0, 0.01, len(ii)), 6).astype(np.float32)
    directed = sgn.GraphArrays(np.arange(Vd), np.concatenate([ii, np.arange(Vd)]), np.concatenate([jj, np.arange(Vd)]),
                               np.concatenate([dlat, np.full(Vd, 1_000_000, np.uint64)]),
                               np.concatenate([dloss, np.zeros(Vd, np.float32)]), True)
    Vl = 60
    x = rng.permutation(Vl).astype(np.int64)
    li, lj = np.triu_indices(Vl, 1)
    llat = (np.abs(x[li] - x[lj]) * 1_000_000).astype(np.uint64)
    lloss = np.round(rng.uniform(0, 0.01, len(li)), 6).astype(np.float32)
    line = sgn.GraphArrays(np.arange(Vl), np.concatenate([li, np.arange(Vl)]), np.concatenate([lj, np.arange(Vl)]),
                           np.concatenate([llat, np.full(Vl, 1_000_000, np.uint64)]),
                           np.concatenate([lloss, np.zeros(Vl, np.float32)]), False)
    par = sgn.GraphArrays(rand_c.node_id, np.concatenate([rand_c.src, [3]]), np.concatenate([rand_c.dst, [7]]),
                          np.concatenate([rand_c.lat, [2_000_000]]).astype(np.uint64),
                          np.concatenate([rand_c.loss, [0.001]]).astype(np.float32), False)
    tor = sgn.tor_graph(700, seed=12)
    # a directed metric graph (asymmetric: +1 ms one way), complete: fused with nothing to
    # shorten, its transposed rows built by ndt_build (sq_rows builds them for undirected ones)
    Vm = 240
    P = rng.uniform(0, 1, (Vm, 2))
    mi, mj = np.nonzero(~np.eye(Vm, dtype=bool))
    mlat = (6_000_000 + np.round(np.hypot(*(P[mi] - P[mj]).T) * 50_000_000) + np.where(mi < mj, 1_000_000, 0)).astype(np.uint64)
    mloss = np.round(rng.uniform(0, 0.01, len(mi)), 6).astype(np.float32)
    dmetric = sgn.GraphArrays(np.arange(Vm), np.concatenate([mi, np.arange(Vm)]), np.concatenate([mj, np.arange(Vm)]),
                              np.concatenate([mlat, np.full(Vm, 1_000_000, np.uint64)]),
                              np.concatenate([mloss, np.zeros(Vm, np.float32)]), True)
    # (graph, used, env, expected (loss_dense, loss_fused) of the default run)
    cases = [(tor, None, {}, (1, 1)), (tor, None, {"SGN_APSP_DENSE_H": "1"}, (1, 0)),
             (sgn.tor_graph(500, seed=13), np.arange(1, 500, 3), {}, (1, 1)), (line, None, {}, (1, 1)),
             (rand_c, None, {}, (1, 0)), (rand_c, None, {"SGN_APSP_DENSE_S": "32"}, (1, 0)),
             (directed, None, {}, (1, 0)), (dmetric, None, {}, (1, 1)), (dmetric, np.arange(0, Vm, 7), {}, (1, 1)),
             (par, None, {}, (0, 0))]
    for k, (g, used, env, want) in enumerate(cases):
        used = np.arange(len(g.node_id)) if used is None else used
        ol, op = oracle.routes(g, used)
        forms = []
        for form_env in ({}, {"SGN_APSP_FUSED": "0"}, {"SGN_APSP_DENSE": "0"}):
            for key, val in {**env, **form_env}.items():
                monkeypatch.setenv(key, val)
            c = ctxf()
            c.routes_build(g, used)
            t = c.routes_timing()
            forms.append((t["loss_dense"], t["loss_fused"], t["loss_multi"]))
            for key in {**env, **form_env}:
                monkeypatch.delenv(key)
            gl, gp = c.routes_copy()
            assert np.array_equal(ol, gl) and np.array_equal(op.view(np.uint32), gp.view(np.uint32)), (k, form_env)
        assert forms[0][:2] == want and forms[0][2] >= 4, (k, forms)
        assert forms[1][:2] == (want[0], 0) and forms[1][2] >= 4, (k, forms)
        assert forms[2][:2] == (0, 0) and forms[2][2] >= 4, (k, forms)


@pytest.mark.parametrize("n_shards", [2, 3, 8])
def test_apsp_sharded_blocks_equal_whole(ctxf, oracle, monkeypatch, n_shards):
    """The sharded build's block arithmetic (every shard computes a block of used
    sources, and a block of row tiles per squaring pass) on one GPU: SGN_APSP_VSHARDS runs the n
    blocks in turn over one buffer, through every form — per-source relaxation, squaring with
    the multi-source sweep, the one-source loss pass, the u64 Floyd-Warshall fallback — with
    uneven blocks, blocks without a row tile (V <= 64), and more shards than used sources.
    The RCCL exchange between the blocks runs in the multi-GPU bench (bench.py shard_check)."""
    Vl = 40
    long_g = sgn.random_graph(Vl, seed=5, lat_lo_us=1_500_000, lat_hi_us=3_500_000)
    cases = [(sgn.random_graph(333, seed=4, loss_frac=0.5), np.arange(0, 333, 2), {}),
             (sgn.tor_graph(600, seed=3), np.arange(600), {}),
             (sgn.tor_graph(200, seed=9), np.arange(200), {"SGN_APSP_LOSS1": "1"}),
             (long_g, np.arange(Vl), {"SGN_APSP_SQ": "1"}),
             (sgn.tor_graph(50, seed=2), np.array([3, 17, 41]), {})]
    for k, (g, used, env) in enumerate(cases):
        ol, op = oracle.routes(g, used)
        for key, val in env.items():
            monkeypatch.setenv(key, val)
        c = ctxf()
        c.routes_build(g, used)
        whole = c.routes_timing()
        monkeypatch.setenv("SGN_APSP_VSHARDS", str(n_shards))
        c.routes_build(g, used)
        t = c.routes_timing()
        monkeypatch.delenv("SGN_APSP_VSHARDS")
        for key in env:
            monkeypatch.delenv(key)
        gl, gp = c.routes_copy()
        assert np.array_equal(ol, gl) and np.array_equal(op.view(np.uint32), gp.view(np.uint32)), k
        assert whole["shards"] == 1 and t["shards"] == n_shards and t["shard_sources"] == len(used)
        for f in ("latency_bf", "latency_u64", "loss_multi"):
            assert t[f] == whole[f], (k, f)


def test_apsp_errors(ctxf):
    c = ctxf()
    g = sgn.GraphArrays([0, 1], [0, 0, 1], [1, 0, 1], [5, 3, 3], [0, 0, 0], False)
    c.routes_build(g, [0, 1])  # fine
    bad = sgn.GraphArrays([0, 1], [0, 1], [1, 1], [5, 3], [0, 0], False)  # node 0: no self-loop
    with pytest.raises(sgn.SgnError, match="No edge connecting node 0 to 0"):
        c.routes_build(bad, [0, 1])
    disc = sgn.GraphArrays([0, 1, 2], [0, 1, 2], [0, 1, 2], [1, 1, 1], [0, 0, 0], False)
    with pytest.raises(sgn.SgnError, match="not connected"):
        c.routes_build(disc, [0, 2])
    dup = sgn.GraphArrays([0, 1], [0, 0, 1, 0], [0, 0, 1, 1], [1, 2, 1, 1], [0, 0, 0, 0], False)
    with pytest.raises(sgn.SgnError, match="More than one edge"):
        c.routes_build(dup, [0, 1])


def test_codel_control_law_on_device(ctxf, oracle):
    c = ctxf()
    n = 1 << 20
    out = np.zeros(n, dtype=np.uint64)
    c.check(c.L.sgn_selftest_codel_law(c.h, n, sgn.ptr(out, sgn.C.c_uint64)))
    x = 1e8 / np.sqrt(np.maximum(np.arange(n, dtype=np.float64), 1.0))
    fl = np.floor(x)
    exp = np.where(x - fl >= 0.5, fl + 1, fl).astype(np.uint64)  # f64::round, half away
    assert np.array_equal(out, exp)
    # spot-check against the oracle's restatement
    for i in (0, 1, 2, 3, 7, 19, 1000, n - 1):
        assert oracle.load().ora_codel_control_law(SIM_START, i) - SIM_START == int(out[i])


def scenario(n=200, V=50, *, kind=sgn.TRAFFIC_PERIODIC, stop_ns=500_000_000, bw=10_000_000,
             seed=1, graph_seed=1, dynamic=False, runahead_ns=1_000_000, bootstrap_ns=0,
             unknown=10, period_ns=1_000_000, fifo=64, codel=4096, tgen_think=50_000_000,
             tor=False, qdisc=0, loss_hi=None):
    if tor:
        g = sgn.tor_graph(V, seed=graph_seed)
    elif loss_hi is not None:
        g = sgn.random_graph(V, seed=graph_seed, loss_frac=0.5, loss_hi=loss_hi)
    else:
        g = sgn.random_graph(V, seed=graph_seed)
    used = np.arange(V)
    names = sgn.host_names(n)
    seeds = sgn.derive_seeds(seed, names)
    bwv = bw if np.ndim(bw) else np.full(n, bw, dtype=np.uint64)
    hosts = sgn.HostArrays(sgn.assign_ips(n), (np.arange(n) * 7) % V, bwv, bwv, seeds)
    cfg = sgn.make_config(stop_ns, runahead_ns=runahead_ns, dynamic=dynamic,
                          bootstrap_end_ns=bootstrap_ns, out_fifo_cap=fifo, codel_cap=codel,
                          event_capacity=1 << 20, qdisc=qdisc)
    if kind == sgn.TRAFFIC_PERIODIC:
        tr = sgn.make_traffic(period_ns=period_ns, start_jitter_ns=3_000_000,
                              unknown_dst_permille=unknown, payload_len=1024)
    else:
        servers = np.arange(0, n, 10)
        tr = sgn.make_traffic(sgn.TRAFFIC_TGEN, period_ns=tgen_think,
                              period_jitter_ns=tgen_think, start_jitter_ns=20_000_000,
                              servers=servers, file_bytes=(50 * 1024, 300 * 1024, 1024 * 1024))
    return g, used, hosts, cfg, tr


def run_both(ctxf, oracle, args, trace=True, round_by_round=0):
    g, used, hosts, cfg, tr = args
    lat, loss = oracle.routes(g, used)
    o = oracle.Sim(used, lat, loss, hosts, cfg, tr, trace=trace)
    c = ctxf()
    c.routes_build(g, used)
    c.hosts_set(hosts)
    if trace:
        c.trace_enable(1 << 22)
    c.sim_init(cfg, tr)
    for _ in range(round_by_round):
        wo, wg = o.window(), c.window()
        assert wo == wg
        if not wo[2]:
            break
        assert o.round() == c.round()
    o.run()
    c.run()
    return o, c


def sort_trace(t):
    return t[np.lexsort((t["seq"], t["host"]))]


def assert_same_run(o, c, n, trace=True):
    so, sg = o.stats(), c.stats()
    for k in so:
        if k in ("max_pending_events", "sched_heavy_hosts", "sched_sorted_segments", "event_runs"):
            continue
        assert so[k] == sg[k], (k, so[k], sg[k])
    assert o.window() == c.window()
    do, dg = o.digests(0, n), c.digests(0, n)
    for f in ("tx", "rx", "app", "rng", "next_event_id", "n_sent", "n_popped", "n_delivered",
              "n_codel_dropped"):
        assert np.array_equal(do[f], dg[f]), f
    if trace:
        to, tg = sort_trace(o.trace()), sort_trace(c.trace())
        assert len(to) == len(tg)
        for f in ("kind", "host", "peer", "flags", "a", "b", "c", "seq", "rng_pos"):
            bad = np.nonzero(to[f] != tg[f])[0]
            assert len(bad) == 0, (f, to[bad[:3]], tg[bad[:3]])


def test_engine_periodic_trace(ctxf, oracle):
    args = scenario()
    o, c = run_both(ctxf, oracle, args, round_by_round=300)
    assert c.stats()["packets_sent"] > 10000
    assert c.stats()["packets_unknown_dst"] > 0 and c.stats()["packets_loss_dropped"] > 0
    assert_same_run(o, c, args[2].n)


@pytest.mark.parametrize("loss_hi", [0.02, 0.2])
def test_engine_tgen_untraced_loss_tests(ctxf, oracle, loss_hi):
    """Untraced TGEN trains take the batched loss test (engine.hip send_batch): eight draws
    per test, screened on the carry-less high words for paths losing <= 1/32, exact for
    lossier ones. Edges losing up to 2 % (mostly screened) and up to 20 % (both forms)."""
    args = scenario(n=300, V=30, kind=sgn.TRAFFIC_TGEN, stop_ns=2_000_000_000, loss_hi=loss_hi,
                    tgen_think=100_000_000)
    o, c = run_both(ctxf, oracle, args, trace=False)
    st = c.stats()
    assert st["packets_sent"] > 40_000 and st["packets_loss_dropped"] > (400 if loss_hi < 0.1 else 4000), st
    assert_same_run(o, c, args[2].n, trace=False)


def test_engine_tgen_trace_codel(ctxf, oracle):
    # slow down-links make CoDel queues stand and drop
    bw = np.where(np.arange(300) % 10 == 0, 100_000_000, 4_000_000).astype(np.uint64)
    args = scenario(n=300, V=30, kind=sgn.TRAFFIC_TGEN, stop_ns=2_000_000_000, bw=bw, tor=True,
                    tgen_think=200_000_000)
    o, c = run_both(ctxf, oracle, args)
    st = c.stats()
    assert st["codel_dropped"] > 0, st
    assert_same_run(o, c, args[2].n)


@pytest.mark.parametrize("trace", [True, False])
def test_engine_codel_page_pool(ctxf, oracle, trace):
    # CoDel queues as chains of pool pages: 160 run slots per host on average (3000 pages of
    # 16 runs for 300 hosts) while the slow hosts' standing queues need ~2.7k pages beyond
    # their first at peak: pages leave the free ring, come back as queues drain and are
    # taken again by other hosts in later rounds — traced (k_execute) and persistent rounds
    bw = np.where(np.arange(300) % 10 == 0, 100_000_000, 4_000_000).astype(np.uint64)
    args = scenario(n=300, V=30, kind=sgn.TRAFFIC_TGEN, stop_ns=2_000_000_000, bw=bw, tor=True,
                    tgen_think=200_000_000, codel=160)
    o, c = run_both(ctxf, oracle, args, trace=trace)
    st, info = c.stats(), c.engine_info()
    assert st["codel_dropped"] > 0, st
    # (the pool may grow once the next round's bound exceeds its free pages: test_gpu_pools.py)
    assert info["codel_pages"] >= 3000
    assert info["codel_page_allocs"] > 3000 - 300, info  # more allocations than spare pages: reuse
    assert info["codel_pages_free"] + info["codel_pages_chained"] == info["codel_pages"], info
    assert_same_run(o, c, args[2].n, trace=trace)


def test_engine_tgen_round_robin_qdisc(ctxf, oracle):
    # experimental.interface_qdisc: round_robin; short think times keep several response
    # trains (sockets) queued at a server, so the interface interleaves them packet by packet
    bw = np.where(np.arange(300) % 10 == 0, 100_000_000, 8_000_000).astype(np.uint64)
    args = scenario(n=300, V=30, kind=sgn.TRAFFIC_TGEN, stop_ns=600_000_000, bw=bw, tor=True,
                    tgen_think=10_000_000, qdisc=sgn.QDISC_ROUND_ROBIN)
    o, c = run_both(ctxf, oracle, args)
    assert c.stats()["packets_sent"] > 10000
    assert_same_run(o, c, args[2].n)


def test_engine_dynamic_runahead_bootstrap(ctxf, oracle):
    args = scenario(n=150, dynamic=True, runahead_ns=0, bootstrap_ns=100_000_000,
                    stop_ns=400_000_000)
    o, c = run_both(ctxf, oracle, args, round_by_round=100)
    assert_same_run(o, c, args[2].n)


def test_engine_tiny_fifo_blocks(ctxf, oracle):
    args = scenario(n=100, bw=1_000_000, fifo=2, period_ns=500_000, stop_ns=300_000_000)
    o, c = run_both(ctxf, oracle, args)
    assert c.stats()["app_blocked"] > 0
    assert_same_run(o, c, args[2].n)


def test_engine_large_digests(ctxf, oracle):
    n = 10000
    args = scenario(n=n, V=1000, graph_seed=42, stop_ns=300_000_000, period_ns=10_000_000,
                    bw=100_000_000)
    o, c = run_both(ctxf, oracle, args, trace=False)
    assert_same_run(o, c, n, trace=False)


@pytest.mark.parametrize("grid", [1, 7])
def test_persistent_grid_smaller_than_groups(ctxf, oracle, monkeypatch, grid):
    # every workgroup of the persistent round kernel serves several host groups per round
    # (as at 1 M hosts, where the groups outnumber the resident workgroups)
    monkeypatch.setenv("SGN_PERSIST_GRID", str(grid))
    n = 2000
    args = scenario(n=n, V=100, kind=sgn.TRAFFIC_TGEN, stop_ns=400_000_000, tor=True,
                    bw=np.where(np.arange(n) % 10 == 0, 100_000_000, 10_000_000).astype(np.uint64))
    o, c = run_both(ctxf, oracle, args, trace=False)
    assert c.stats()["packets_sent"] > 1000
    assert_same_run(o, c, n, trace=False)


def test_persistent_census_fallback(ctxf, oracle, monkeypatch):
    # a persistent grid larger than the chip holds (4096 one-wave workgroups of the round
    # kernel): the residency census sends every workgroup home before any state is touched,
    # the host falls back to per-round launches, and the run is still bit-exact
    monkeypatch.setenv("SGN_PERSIST_GRID_FORCE", "4096")
    n = 2000
    args = scenario(n=n, V=100, kind=sgn.TRAFFIC_TGEN, stop_ns=300_000_000, tor=True,
                    bw=np.where(np.arange(n) % 10 == 0, 100_000_000, 10_000_000).astype(np.uint64))
    o, c = run_both(ctxf, oracle, args, trace=False)
    info = c.engine_info()
    assert info["persistent_fallbacks"] >= 1 and info["persistent_grid"] == 0, info
    assert c.stats()["packets_sent"] > 1000
    assert_same_run(o, c, n, trace=False)


@pytest.mark.parametrize("tor", [False, True])
def test_persistent_idle_gaps_wrap_calendar(ctxf, oracle, tor):
    # idle gaps between rounds longer than the calendar's span (NB x BW) with routes
    # of mixed latency: the next round's sends reach bucket indices the previous round
    # consumed. The persistent kernel then does the round's bucket bookkeeping before a second
    # grid barrier (no send can race it); bit-exact against the oracle
    # (a datagram per host every 700 ms within 3 ms of each other, deliveries over 1..89 ms
    # (random graph) or 1..150 ms (Tor-like): ~550 ms idle between bursts)
    n = 600
    args = scenario(n=n, V=60 if not tor else 40, tor=tor, period_ns=700_000_000, stop_ns=5_000_000_000,
                    unknown=0)
    o, c = run_both(ctxf, oracle, args, trace=False)
    info = c.engine_info()
    assert info["persistent_grid"] > 0 and info["persistent_fallbacks"] == 0, info
    span = info["calendar_buckets"] * info["bucket_width_ns"]
    assert span < 700_000_000, info  # the gaps exceed the calendar's span
    assert c.stats()["packets_sent"] > 1000
    assert_same_run(o, c, n, trace=False)


def test_worker_exports(ctxf, oracle):
    g, used, hosts, cfg, tr = scenario(n=20, V=10)
    c = ctxf()
    c.routes_build(g, used)
    c.hosts_set(hosts)
    lat, _ = oracle.routes(g, used)
    be = lambda ip: int.from_bytes(int(ip).to_bytes(4, "big"), "little")
    for a in range(0, 20, 3):
        for b in range(0, 20, 5):
            got = c.L.sgn_worker_get_latency(c.h, be(hosts.ip[a]), be(hosts.ip[b]))
            assert got == lat[hosts.node_id[a], hosts.node_id[b]]
            assert c.L.sgn_worker_is_routable(c.h, be(hosts.ip[a]), be(hosts.ip[b])) == 1
    assert c.L.sgn_worker_get_latency(c.h, be(0x0A000001), be(hosts.ip[0])) == sgn.EMUTIME_INVALID
    assert c.L.sgn_worker_get_bandwidth_up_bytes(c.h, be(hosts.ip[3])) == hosts.bw_up[3] // 8


@pytest.mark.parametrize("kind,dynamic", [("periodic", False), ("tgen", False), ("periodic", True)])
def test_two_shards_one_gpu_match_single(ctxf, oracle, kind, dynamic):
    """The multi-shard device path (per-peer exchange slots, k_import, local round edge,
    min all-reduce, window advance) with two shards on one GPU through the local shard-group
    transport: identical per-host digests, counters and final window to one shard (and so
    to the oracle)."""
    import ctypes as C
    n = 300
    if kind == "tgen":
        bw = np.where(np.arange(n) % 10 == 0, 100_000_000, 4_000_000).astype(np.uint64)
        args = scenario(n=n, V=30, kind=sgn.TRAFFIC_TGEN, stop_ns=600_000_000, bw=bw, tor=True,
                        tgen_think=100_000_000)
    else:
        args = scenario(n=n, dynamic=dynamic, runahead_ns=0 if dynamic else 1_000_000,
                        stop_ns=300_000_000)
    g, used, hosts, cfg, tr = args
    one = ctxf()
    one.routes_build(g, used)
    one.hosts_set(hosts)
    one.sim_init(cfg, tr)
    one.run()
    shards = [ctxf(shard_rank=r, shard_count=2) for r in range(2)]
    arr = (C.c_void_p * 2)(*[c.h.value for c in shards])
    for c in shards:
        c.routes_build(g, used)
        c.hosts_set(hosts)
    shards[0].check(shards[0].L.sgn_comm_init_local(arr, 2, 1 << 16))
    for c in shards:
        c.sim_init(cfg, tr)
    done = C.c_uint64()
    shards[0].check(shards[0].L.sgn_run_local_group(arr, 2, 1 << 40, C.byref(done)))
    s1 = one.stats()
    tot = {k: 0 for k in s1}
    for r, c in enumerate(shards):
        lo, hi = C.c_uint32(), C.c_uint32()
        c.L.sgn_shard_range(n, r, 2, C.byref(lo), C.byref(hi))
        d1, d2 = one.digests(lo.value, hi.value), c.digests(lo.value, hi.value)
        for f in ("tx", "rx", "app", "rng", "next_event_id", "n_sent", "n_popped", "n_delivered",
                  "n_codel_dropped"):
            assert np.array_equal(d1[f], d2[f]), (r, f)
        assert c.window() == one.window()
        st = c.stats()
        for k in ("packets_sent", "packets_loss_dropped", "packets_unknown_dst",
                  "packet_events_popped", "delivered", "codel_dropped", "local_events"):
            tot[k] += st[k]
    assert s1["packets_sent"] > 1000
    for k in ("packets_sent", "packets_loss_dropped", "packets_unknown_dst", "packet_events_popped",
              "delivered", "codel_dropped", "local_events"):
        assert tot[k] == s1[k], k
    assert done.value == s1["rounds"]


# ---- CPU-resident applications (SGN_TRAFFIC_EXTERNAL) and the device-held host RNG ----
def _external_pair(ctxf, oracle, world, drain_cap=1 << 16):
    g, used, hosts, cfg, tr = world
    lat, loss = oracle.routes(g, used)
    o = oracle.Sim(used, lat, loss, hosts, cfg, tr, trace=True)
    c = ctxf()
    c.routes_build(g, used)
    c.hosts_set(hosts)
    c.trace_enable(1 << 20)
    c.drain_enable(drain_cap)
    c.sim_init(cfg, tr)
    return o, c


def test_external_apps_submit_drain_rng(ctxf, oracle):
    from external_common import datagrams, drive, external_world
    world = external_world()
    o, c = _external_pair(ctxf, oracle, world)
    dg = datagrams(world[2])
    (do, dc), rounds = drive([o, c], dg)
    assert rounds > 50 and len(do) == len(dg[3])
    for f in sgn.DRAIN_DTYPE.names:
        bad = np.nonzero(do[f] != dc[f])[0]
        assert len(bad) == 0, (f, do[bad[:3]], dc[bad[:3]])
    st = np.bincount(dc["status"], minlength=6)
    assert st[sgn.DRAIN_DELIVERED] > 0 and st[sgn.DRAIN_LOSS] > 0 and st[sgn.DRAIN_BLOCKED] > 0
    assert_same_run(o, c, world[2].n)


def test_trace_captures_identical(ctxf, oracle, tmp_path):
    """§8f row 1: the per-host interface captures (pcap, utility/pcap_writer.rs) built from
    libsgn's trace and from the oracle's are byte-identical: external apps (unknown addresses,
    loopback, TCP sizes, CPU-side RNG draws) and a PERIODIC run with unknown destinations."""
    from external_common import datagrams, drive, external_world
    world = external_world()
    o, c = _external_pair(ctxf, oracle, world)
    drive([o, c], datagrams(world[2]))
    runs = [(o, c, world[2])]
    args = scenario(n=120, V=30, unknown=50, stop_ns=200_000_000)
    o2, c2 = run_both(ctxf, oracle, args)
    runs.append((o2, c2, args[2]))
    for k, (o, c, hosts) in enumerate(runs):
        names = sgn.host_names(hosts.n)
        po = sgn.write_pcaps(o.trace(), hosts.ip, tmp_path / f"o{k}", names=names)
        pc = sgn.write_pcaps(c.trace(), hosts.ip, tmp_path / f"c{k}", names=names)
        assert po.keys() == pc.keys() and len(po) > 10
        for h in po:
            assert po[h][1] == pc[h][1] > 0
            assert open(po[h][0], "rb").read() == open(pc[h][0], "rb").read(), h


def test_external_rules_on_device(ctxf, oracle):
    from external_common import RUNAHEAD, external_world
    world = external_world(n=10, V=5, stop_ns=10_000_000_000)
    o, c = _external_pair(ctxf, oracle, world)
    S = SIM_START
    ip = world[2].ip
    c.round()
    assert c.window()[2] is False
    with pytest.raises(sgn.SgnError, match="empty window"):
        c.set_window(S + 10, S + 10)
    with pytest.raises(sgn.SgnError, match="longer than the runahead"):
        c.set_window(S + 10, S + 10 + 10 * RUNAHEAD)
    c.set_window(S + 5_000_000, S + 5_000_000 + RUNAHEAD)
    with pytest.raises(sgn.SgnError, match="outside"):
        c.submit([0], [ip[1]], [100], [S + 4_000_000])
    with pytest.raises(sgn.SgnError, match="horizon"):
        c.submit([0], [ip[1]], [100], [S + 5_000_000 + 5 * 10 ** 9])
    with pytest.raises(sgn.SgnError, match="wire_len"):
        c.submit([0], [ip[1]], [100], [S + 5_500_000], wire_len=[100])
    with pytest.raises(sgn.SgnError, match="not owned"):
        c.submit([10], [ip[1]], [100], [S + 5_500_000])
    c.submit([0], [ip[1]], [100], [S + 5_500_000], handle=[77], wire_len=[128])
    c.round()
    ws, we, active = c.window()
    assert active and ws > S + 5_500_000
    with pytest.raises(sgn.SgnError, match="after the device"):
        c.set_window(ws + 1, ws + 2)
    with pytest.raises(sgn.SgnError, match="previous window"):
        c.set_window(S + 5_000_000, S + 5_000_001)
    while c.window()[2]:
        c.round()
    d = c.drain()
    assert len(d) == 1 and d["handle"][0] == 77 and d["payload_len"][0] == 100
    # the device RNG is the host's Xoshiro256++ stream (seeded as host.rs:234)
    L = oracle.load()
    st = np.zeros(4, dtype=np.uint64)
    L.ora_xoshiro_seed_from_u64(int(world[2].seed[5]), sgn.ptr(st, sgn.C.c_uint64))
    exp = [int(L.ora_xoshiro_next_u64(sgn.ptr(st, sgn.C.c_uint64))) for _ in range(3)]
    assert c.rng_next_u64(5) == exp[0]
    assert c.rng_double(5) == (exp[1] >> 11) * 2.0 ** -53
    assert c.rng_fill_bytes(5, 3) == (exp[2] >> 32).to_bytes(4, "little")[:3]
    with pytest.raises(sgn.SgnError):
        sgn.Context().submit([0], [0], [0], [S])  # no simulation
