"""Config #1 (BASELINE.json configs[0], getting_started_basic): the reference's
`examples/docs/basic-file-transfer/shadow.yaml` — `server` + `client1..3` on `1_gbit_switch`,
seed 1, hosts in hostname (BTreeMap) order — with its http.server / curl conversation played by
a scripted stand-in through the CPU-resident-application path (tests/http_exchange.py).

CPU: the oracle alone runs the conversation to completion (protocol and timing invariants).
GPU: libsgn and the oracle in lockstep under the same controller — every drain record, counter,
host digest and the per-host interface captures (pcap) identical."""
import numpy as np
import pytest

import sgn
from http_exchange import BODY, MSS, Exchange, basic_file_transfer, decode, drive

ENGINE = dict(out_fifo_cap=64, codel_cap=1024, event_capacity=1 << 16)


def _setup():
    s = basic_file_transfer()
    # the config as the reference resolves it (configuration.rs:1367-1381, sim_config.rs)
    assert s.names == ["client1", "client2", "client3", "server"]
    assert s.seed == 1 and s.stop_time_ns == 10 * 10**9 and s.runahead_ns == 1_000_000
    assert s.graph.node_id.tolist() == [0] and s.used_nodes.tolist() == [0]
    assert s.hosts.bw_up.tolist() == [1_000_000_000] * 4 and s.hosts.bw_down.tolist() == [1_000_000_000] * 4
    assert s.process_start_ns == [[5 * 10**9]] * 3 + [[3 * 10**9]]
    return s


def _oracle_sim(oracle, s, trace=False):
    lat, loss = oracle.routes(s.graph, s.used_nodes, s.use_shortest_path)
    cfg = s.sim_config(**ENGINE)
    return oracle.Sim(s.used_nodes, lat, loss, s.hosts, cfg, sgn.make_traffic(sgn.TRAFFIC_EXTERNAL), trace=trace), lat


def test_basic_file_transfer_oracle(oracle):
    s = _setup()
    o, lat = _oracle_sim(oracle, s)
    ex = Exchange(s)
    (d,), rounds = drive([o], ex, s.runahead_ns)
    assert ex.finished(), ex.conn
    total = -(-(155 + BODY) // MSS)
    # every datagram delivered (1_gbit_switch has no loss), none before send time + 1 ms
    assert np.all(d["status"] == sgn.DRAIN_DELIVERED)
    per_client = 5 + total + (total + 1) // 2 + 3  # handshake + GET + its ACK, data, ACKs, FINs
    assert len(d) == 3 * per_client, (len(d), per_client)
    assert np.all(d["time"] >= sgn.SIMULATION_START + 5 * 10**9 + int(lat[0, 0]))
    kinds = np.array([decode(h)[1] for h in d["handle"]])
    assert np.bincount(kinds).tolist()[4] == 3 * total  # data segments
    # slow start: the first flight (10 segments), then the rest one round trip later (the
    # 1 Gbit/s token buckets hold 1 ms of traffic, so a flight passes them at once:
    # token_bucket.rs). Each hop of the round trip is the 1 ms latency plus the wait for the
    # window's end: the window opens at the delivery (the earliest event) and the application
    # answers between rounds
    data = d[kinds == 4]
    flights = np.unique(data["time"])
    assert len(flights) == 2 and int(flights[1] - flights[0]) == 2 * (int(lat[0, 0]) + s.runahead_ns)
    assert np.bincount(np.searchsorted(flights, data["time"])).tolist() == [30, 3 * (total - 10)]
    st = o.stats()
    assert st["delivered"] == len(d) and st["packets_loss_dropped"] == 0
    assert rounds > 10


@pytest.mark.gpu
def test_basic_file_transfer_engine_vs_oracle(oracle, tmp_path):
    s = _setup()
    o, _ = _oracle_sim(oracle, s, trace=True)
    c = sgn.Context()
    c.routes_build(s.graph, s.used_nodes, shortest=s.use_shortest_path)
    c.hosts_set(s.hosts)
    c.trace_enable(1 << 16)
    c.drain_enable(1 << 14)
    c.sim_init(s.sim_config(**ENGINE), sgn.make_traffic(sgn.TRAFFIC_EXTERNAL))
    ex = Exchange(s)
    (do, dc), rounds = drive([o, c], ex, s.runahead_ns)
    assert ex.finished() and rounds > 10 and len(do) == len(dc) > 80
    for f in sgn.DRAIN_DTYPE.names:
        bad = np.nonzero(do[f] != dc[f])[0]
        assert len(bad) == 0, (f, do[bad[:3]], dc[bad[:3]])
    so, sg = o.stats(), c.stats()
    for k in so:
        if k not in ("max_pending_events", "sched_heavy_hosts", "sched_sorted_segments", "event_runs"):
            assert so[k] == sg[k], k
    assert o.window() == c.window()
    n = s.hosts.n
    dgo, dgc = o.digests(0, n), c.digests(0, n)
    for f in ("tx", "rx", "app", "rng", "next_event_id", "n_sent", "n_popped", "n_delivered"):
        assert np.array_equal(dgo[f], dgc[f]), f
    # the per-host interface captures (utility/pcap_writer.rs) byte for byte
    po = sgn.write_pcaps(o.trace(), s.hosts.ip, tmp_path / "o", names=s.names)
    pc = sgn.write_pcaps(c.trace(), s.hosts.ip, tmp_path / "c", names=s.names)
    assert po.keys() == pc.keys() and len(po) == 4
    for h in po:
        assert po[h][1] == pc[h][1] > 0
        assert open(po[h][0], "rb").read() == open(pc[h][0], "rb").read(), h
    c.close()
