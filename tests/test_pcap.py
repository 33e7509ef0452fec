"""Packet capture and the trace's RNG position, CPU side.

* sgn_pcap_* reproduce PcapWriter's bytes exactly: the expected arrays of the reference's own
  tests (utility/pcap_writer.rs test_empty_pcap_writer / test_write_packet);
* sgn_packet_bytes lays out Packet::display_bytes (network/packet.rs:800-934) for UDP, TCP and
  TCP with the window-scale option;
* trace records from the oracle (external applications: unknown addresses, loopback, TCP
  sizes, token-bucket waits, CPU-side RNG draws) convert into per-host captures whose
  packets, times and headers follow the records, and whose RNG positions count the draws.
The GPU side (libsgn's trace == the oracle's, byte-identical pcap files) is in
tests/test_gpu_parity.py.
"""
import pathlib
import struct

import numpy as np
import pytest

import sgn

# utility/pcap_writer.rs tests: the global header and one record {32 s, 128 us, 3 bytes}
GOLD_HEADER = bytes([0xD4, 0xC3, 0xB2, 0xA1, 0x02, 0x00, 0x04, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
                     0x00, 0x00, 0xFF, 0xFF, 0x00, 0x00, 0x65, 0x00, 0x00, 0x00])
GOLD_RECORD = bytes([0x20, 0x00, 0x00, 0x00, 0x80, 0x00, 0x00, 0x00, 0x03, 0x00, 0x00, 0x00, 0x03, 0x00,
                     0x00, 0x00, 0x01, 0x02, 0x03])


def _pcap(lib, path, cap, packets):
    h = sgn.C.c_void_p()
    assert lib.sgn_pcap_open(str(path).encode(), cap, sgn.C.byref(h)) == 0
    for ts, us, data in packets:
        buf = (sgn.C.c_uint8 * len(data)).from_buffer_copy(data) if data else None
        assert lib.sgn_pcap_write_packet(h, ts, us, buf, len(data)) == 0
    assert lib.sgn_pcap_close(h) == 0
    return path.read_bytes()


def test_pcap_writer_reference_vectors(lib, tmp_path):
    assert _pcap(lib, tmp_path / "a.pcap", 65535, []) == GOLD_HEADER
    assert _pcap(lib, tmp_path / "b.pcap", 65535, [(32, 128, b"\x01\x02\x03")]) == GOLD_HEADER + GOLD_RECORD
    # a capture length below the packet keeps the original length and truncates the bytes
    out = _pcap(lib, tmp_path / "c.pcap", 2, [(1, 2, b"\x01\x02\x03")])
    assert out[24:] == struct.pack("<IIII", 1, 2, 2, 3) + b"\x01\x02"


def test_packet_bytes_layout():
    a, b = 0xC0A80101, 0xC0A80102  # 192.168.1.1 -> 192.168.1.2
    udp = sgn.packet_bytes(a, b, 12)
    assert len(udp) == 40
    assert udp[:20] == bytes([0x45, 0, 0, 40, 0, 0, 0x40, 0, 64, 17, 0, 0, 192, 168, 1, 1, 192, 168, 1, 2])
    assert udp[20:28] == bytes([0, 0, 0, 0, 0, 20, 0, 0]) and udp[28:] == bytes(12)
    tcp = sgn.packet_bytes(a, b, 100, sgn.C.c_uint32(1 << 29).value)
    assert len(tcp) == 140 and tcp[9] == 6 and tcp[2:4] == (140).to_bytes(2, "big")
    assert tcp[32] == 0x50 and tcp[20:32] == bytes(12)
    ws = sgn.packet_bytes(a, b, 0, 2 << 29)
    assert len(ws) == 44 and ws[32] == 0x60 and ws[40:44] == bytes([3, 3, 0, 0])


def _read_pcap(path):
    data = path.read_bytes()
    assert data[:24] == GOLD_HEADER
    out, i = [], 24
    while i < len(data):
        ts, us, cap, ln = struct.unpack_from("<IIII", data, i)
        out.append((ts, us, ln, data[i + 16:i + 16 + cap]))
        i += 16 + cap
    return out


@pytest.fixture(scope="module")
def external_trace(oracle):
    from external_common import datagrams, drive, external_world
    g, used, hosts, cfg, tr = world = external_world()
    lat, loss = oracle.routes(g, used)
    o = oracle.Sim(used, lat, loss, hosts, cfg, tr, trace=True)
    dg = datagrams(hosts)
    drive([o], dg)
    return o, world, dg


def test_trace_capture_and_rng_position(external_trace, tmp_path):
    o, (g, used, hosts, cfg, tr), dg = external_trace
    t = o.trace()
    t = t[np.lexsort((t["seq"], t["host"]))]
    kinds = np.bincount(t["kind"], minlength=7)
    assert kinds[sgn.TRACE_IF_POP] > 0 and kinds[sgn.TRACE_LOCAL] > 0 and kinds[sgn.TRACE_DELIVER] > 0
    for h in range(hosts.n):
        th = t[t["host"] == h]
        if len(th) == 0:
            continue
        assert np.all(np.diff(th["seq"].astype(np.int64)) > 0) and np.all(np.diff(th["rng_pos"].astype(np.int64)) >= 0)
        pops = th[th["kind"] == sgn.TRACE_IF_POP]
        sends = th[th["kind"] == sgn.TRACE_SEND]
        # every packet the interface popped was sent, looped back, or still waits in the relay
        assert len(pops) - len(sends) - (th["kind"] == sgn.TRACE_LOCAL).sum() in (0, 1)
        # each send past the DNS check draws once: the position moves by one at those records
        drawn = sends[sends["flags"] != 2]
        prev = np.searchsorted(th["seq"], drawn["seq"]) - 1
        before = np.where(prev >= 0, th["rng_pos"][np.maximum(prev, 0)], 0)
        assert np.all(drawn["rng_pos"] >= before + 1)
        if h not in (1, 2):  # hosts without CPU-side draws: position = number of sends drawn
            assert np.array_equal(drawn["rng_pos"], np.arange(1, len(drawn) + 1))
    # the CPU-side draws (drive(): hosts 1 and 2) are counted in the position too
    for h in (1, 2):
        th = t[t["host"] == h]
        n_drawn = int(((th["kind"] == sgn.TRACE_SEND) & (th["flags"] != 2)).sum())
        assert th["rng_pos"][-1] > n_drawn
    # captures: one packet per IF_POP / DELIVER / LOCAL record, headers from the records
    caps = sgn.write_pcaps(t, hosts.ip, tmp_path, names=sgn.host_names(hosts.n))
    assert sum(n for _, n in caps.values()) == kinds[sgn.TRACE_IF_POP] + kinds[sgn.TRACE_DELIVER] + kinds[sgn.TRACE_LOCAL]
    for h, (path, n) in caps.items():
        assert path.endswith(f"hosts/{sgn.host_names(hosts.n)[h]}/eth0.pcap")
        pk = _read_pcap(pathlib.Path(path))
        assert len(pk) == n
        th = t[(t["host"] == h) & np.isin(t["kind"], [sgn.TRACE_IF_POP, sgn.TRACE_DELIVER, sgn.TRACE_LOCAL])]
        for (ts, us, ln, data), r in zip(pk, th):
            rel = int(r["a"]) - sgn.SIMULATION_START
            assert (ts, us) == (rel // 10**9, rel % 10**9 // 1000)
            pay, tag = int(r["b"]) & 0xFFFFFFFF, int(r["b"]) >> 32
            hdr = {0: 28, 1: 40, 2: 44}[(tag >> 29) & 3]
            assert ln == len(data) == hdr + pay and data[2:4] == ln.to_bytes(2, "big")
            src, dst = int.from_bytes(data[12:16], "big"), int.from_bytes(data[16:20], "big")
            me = int(hosts.ip[h])
            if r["kind"] == sgn.TRACE_IF_POP:
                assert src == me
                assert dst == (int(r["c"]) if r["peer"] == 0xFFFFFFFF else int(hosts.ip[r["peer"]]))
            elif r["kind"] == sgn.TRACE_DELIVER:
                assert dst == me and src == int(hosts.ip[r["peer"]])
            else:
                assert src == dst == me
    unknown = t[(t["kind"] == sgn.TRACE_IF_POP) & (t["peer"] == 0xFFFFFFFF)]
    assert len(unknown) > 0 and np.all((unknown["c"] >> 16) == 0x0AFF)
