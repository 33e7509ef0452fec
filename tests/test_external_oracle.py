"""CPU-resident applications (SGN_TRAFFIC_EXTERNAL) and the device-held host RNG, on the
oracle alone: the contract's invariants (every submitted datagram's fate is drained exactly
once, with its handle; delivery times respect the routes; window rules), and the RNG
byte/double encodings against rand_core 0.9's fill_bytes_via_next restated in Python."""
import numpy as np
import pytest

import sgn
from external_common import RUNAHEAD, datagrams, drive, external_world


def make_oracle(oracle, world):
    g, used, hosts, cfg, tr = world
    lat, loss = oracle.routes(g, used)
    return oracle.Sim(used, lat, loss, hosts, cfg, tr), lat, loss


def test_every_datagram_fate_drained_once(oracle):
    world = external_world()
    o, lat, _ = make_oracle(oracle, world)
    hosts = world[2]
    dg = datagrams(hosts)
    recs, rounds = drive([o], dg)
    d = recs[0]
    src, dip, pay, t, handle, wire = dg
    # one record per submitted datagram (the simulation ran dry: nothing in flight)
    slots = d["tag"] & 0x1FFFFFFF
    kinds = (d["tag"] >> 29) & 3  # header kind: 0 UDP, 1 TCP, 2 TCP + window scale
    assert np.all(d["tag"] & sgn.TAG_EXT)
    assert len(d) == len(t) and len(np.unique(slots)) == len(t)
    # the handle and the payload travel with the datagram
    order = np.argsort(slots)
    assert np.array_equal(d["handle"][order], handle)
    assert np.array_equal(d["payload_len"][order], pay)
    hdr = np.array([28, 40, 44])[kinds[order]]
    assert np.array_equal(np.where(wire == 0, pay + 28, wire), pay + hdr)
    assert set(np.unique(kinds).tolist()) == {0, 1, 2}
    st = np.bincount(d["status"], minlength=6)
    for s in (sgn.DRAIN_DELIVERED, sgn.DRAIN_LOCAL, sgn.DRAIN_LOSS, sgn.DRAIN_UNKNOWN,
              sgn.DRAIN_BLOCKED):
        assert st[s] > 0, (s, st)
    # a delivery happens no earlier than send time + path latency, at the destination
    ip2h = {int(ip): i for i, ip in enumerate(hosts.ip)}
    node = np.asarray(hosts.node_id)
    dl = d[order]
    for i in range(len(t)):
        r = dl[i]
        if r["status"] == sgn.DRAIN_DELIVERED:
            dh = ip2h[int(dip[i])]
            assert r["host"] == dh and r["src_host"] == src[i]
            assert r["time"] >= t[i] + lat[node[src[i]], node[dh]]
        elif r["status"] == sgn.DRAIN_UNKNOWN:
            assert int(dip[i]) not in ip2h and r["host"] == src[i]
        elif r["status"] == sgn.DRAIN_LOCAL:
            assert int(dip[i]) == int(hosts.ip[src[i]]) and r["time"] >= t[i]
    stt = o.stats()
    assert stt["app_blocked"] == st[sgn.DRAIN_BLOCKED]
    assert stt["packets_loss_dropped"] == st[sgn.DRAIN_LOSS]
    assert stt["delivered"] == st[sgn.DRAIN_DELIVERED]


def test_drain_filters_by_host_and_keeps_the_rest(oracle):
    world = external_world(n=20, V=8)
    o, _, _ = make_oracle(oracle, world)
    hosts = world[2]
    dg = datagrams(hosts, k=80, span_ns=20_000_000)
    recs, _ = drive([o], dg)
    d = recs[0]
    # drive() drained [0,30) then [30,..) every 5 rounds: the union is all records, each
    # slice ordered by (host, time, src, src eid, tag, status)
    assert len(d) == 80
    assert o.drain().size == 0


def test_set_window_rules(oracle):
    world = external_world(n=10, V=5)
    o, _, _ = make_oracle(oracle, world)
    S = sgn.SIMULATION_START
    o.round()  # [S, S+1): nothing to do; the simulation has no events
    assert o.window()[2] is False
    with pytest.raises(sgn.SgnError):
        o.set_window(S, S)  # empty
    o.set_window(S + 5_000_000, S + 5_000_000 + RUNAHEAD)
    with pytest.raises(sgn.SgnError):  # before the window start
        o.submit([0], [world[2].ip[1]], [100], [S + 4_000_000])
    o.submit([0], [world[2].ip[1]], [100], [S + 5_500_000])
    o.round()
    ws, we, active = o.window()
    assert active and ws > S + 5_500_000
    with pytest.raises(sgn.SgnError):  # after the next event
        o.set_window(ws + 1, ws + 2)
    with pytest.raises(sgn.SgnError):  # before the last window's end
        o.set_window(S + 5_000_000, S + 5_000_001)


def _fill_bytes_py(next_u64, n):
    out = bytearray()
    while n - len(out) >= 8:
        out += next_u64().to_bytes(8, "little")
    r = n - len(out)
    if r > 4:
        out += next_u64().to_bytes(8, "little")[:r]
    elif r > 0:
        out += (next_u64() >> 32).to_bytes(4, "little")[:r]
    return bytes(out)


@pytest.mark.parametrize("nbytes", [0, 1, 3, 4, 5, 7, 8, 9, 12, 13, 16, 31])
def test_host_rng_fill_bytes_and_double(oracle, nbytes):
    world = external_world(n=4, V=3)
    o, _, _ = make_oracle(oracle, world)
    L = oracle.load()
    st = np.zeros(4, dtype=np.uint64)
    L.ora_xoshiro_seed_from_u64(int(world[2].seed[2]), sgn.ptr(st, sgn.C.c_uint64))

    def nxt():
        return int(L.ora_xoshiro_next_u64(sgn.ptr(st, sgn.C.c_uint64)))

    assert o.rng_fill_bytes(2, nbytes) == _fill_bytes_py(nxt, nbytes)
    x = nxt()
    assert o.rng_double(2) == (x >> 11) * 2.0 ** -53
    assert o.rng_next_u64(2) == nxt()


def test_tcp_segments_take_their_wire_length_through_token_buckets(oracle):
    """Packet::len (network/packet.rs:388-390, :617-635): a TCP segment is payload + 40 B on
    the wire (+ 44 with window scale) and the relays' token buckets charge that length, so the
    same payloads drain later from a slow link as TCP than as UDP."""
    finish = {}
    for hdr in (28, 44):
        world = external_world(n=4, V=3, bw=400_000, fifo=1000, stop_ns=3_000_000_000)
        o, _, _ = make_oracle(oracle, world)
        ip = world[2].ip
        k = 60
        t = sgn.SIMULATION_START + 1_000_000 + np.arange(k, dtype=np.uint64)
        o.submit(np.zeros(k), np.full(k, ip[1]), np.full(k, 500), t, wire_len=np.full(k, 500 + hdr))
        while o.window()[2]:
            o.round()
        d = o.drain()
        assert len(d) == k and np.all(d["status"] == sgn.DRAIN_DELIVERED)
        finish[hdr] = int(d["time"].max())
    assert finish[44] > finish[28]
    with pytest.raises(sgn.SgnError):
        o.submit([0], [ip[1]], [500], [o.window()[0]], wire_len=[530])
