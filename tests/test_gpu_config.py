"""End to end from the reference's own shadow.yaml files: shadow_config builds the inputs
(graph, hosts in hostname order, IPs incl. explicit ip_addr, seeds, runahead, qdisc, CLI
overrides), libsgn runs the packet core on the GPU, the oracle runs the same inputs on the
CPU, and every counter and per-host digest must be identical. The reference's processes are
replaced by synthetic traffic (shadow.yaml has no key for it)."""
import json
import pathlib

import numpy as np
import pytest

import sgn
import shadow_config as sc

pytestmark = pytest.mark.gpu
GOLD = json.loads((pathlib.Path(__file__).parent / "golden" / "reference_configs.json").read_text(encoding="utf-8"))
SKIP_STATS = ("max_pending_events", "sched_heavy_hosts", "sched_sorted_segments", "event_runs")


def _run(oracle, setup, tr, rounds, **engine):
    lat, loss = oracle.routes(setup.graph, setup.used_nodes, setup.use_shortest_path)
    cfg = setup.sim_config(**engine)
    o = oracle.Sim(setup.used_nodes, lat, loss, setup.hosts, cfg, tr)
    c = sgn.Context()
    c.routes_build(setup.graph, setup.used_nodes, shortest=setup.use_shortest_path)
    c.hosts_set(setup.hosts)
    c.sim_init(cfg, tr)
    assert o.run(rounds) == c.run(rounds)
    so, sg = o.stats(), c.stats()
    for k in so:
        if k not in SKIP_STATS:
            assert so[k] == sg[k], k
    assert o.window() == c.window()
    n = setup.hosts.n
    do, dg = o.digests(0, n), c.digests(0, n)
    for f in ("tx", "rx", "app", "rng", "next_event_id", "n_sent", "n_popped", "n_delivered"):
        assert np.array_equal(do[f], dg[f]), f
    return sg


def test_phold_rr_qdisc_config_tgen(oracle):
    t = next(t for t in GOLD["tests"] if t["name"] == "phold-rr-qdisc-shadow")
    cli = sc.parse_cli(t["argv"])
    cfg = sc.ConfigOptions.new(sc.parse_config_file(sc.load_yaml(GOLD["corpus"][t["config"]]["text"])), cli)
    s = sc.sim_setup(cfg)
    assert s.qdisc == sgn.QDISC_ROUND_ROBIN and s.hosts.n == 10
    # one 50-ms window per round (the graph's only latency) holds a whole round of a 10-host
    # group's runs in one calendar slab (<= 1024 runs): file sizes keep a round below that
    tr = sgn.make_traffic(sgn.TRAFFIC_TGEN, period_ns=100_000_000, period_jitter_ns=100_000_000,
                          start_jitter_ns=10_000_000, servers=np.arange(0, 10, 3),
                          file_bytes=(20 * 1024, 100 * 1024, 300 * 1024))
    st = _run(oracle, s, tr, 180, out_fifo_cap=64, codel_cap=4096, event_capacity=1 << 18)
    assert st["packets_sent"] > 5_000


def test_mytest_config_explicit_ips_periodic(oracle):
    s = sc.sim_setup(sc.load(text=GOLD["mytest"]["config"]))
    assert s.runahead_ns == 1_000_000 and s.hosts.n == 10
    # explicit ip_addr entries kept; routing by IP goes through them
    names = s.names
    assert s.hosts.ip[names.index("geth-node")] == 0x0B00000A
    tr = sgn.make_traffic(sgn.TRAFFIC_PERIODIC, period_ns=200_000, start_jitter_ns=100_000, payload_len=1200,
                          unknown_dst_permille=5)
    st = _run(oracle, s, tr, 3000, out_fifo_cap=64, codel_cap=4096, event_capacity=1 << 18)
    assert st["packets_sent"] > 10_000
    # "--runahead null": rounds shrink to the 1 us graph latency (runahead.rs:44-57)
    s = sc.sim_setup(sc.load(text=GOLD["mytest"]["config"], argv=["--runahead", "null"]))
    assert s.runahead_ns == 0
    st = _run(oracle, s, tr, 3000, out_fifo_cap=64, codel_cap=4096, event_capacity=1 << 18)
    assert st["packets_sent"] > 50
