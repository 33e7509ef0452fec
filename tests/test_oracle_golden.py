"""Pins the oracle to the reference's own unit-test vectors and the pinned crates' KATs
(tests/golden/reference_unit_vectors.json). CPU only."""
import ctypes as C
import json
import pathlib

import numpy as np
import pytest

import sgn

GOLD = json.loads((pathlib.Path(__file__).parent / "golden" / "reference_unit_vectors.json").read_text())
MS = 1_000_000
START = sgn.SIMULATION_START


def mock_ms(ms):  # network/mod.rs:26-29 mock_time_millis
    return START + ms * MS


def ref_gml(directed, target_override=None):
    v = GOLD["shortest_path"]
    lines = ["graph [", f"  directed {1 if directed else 0}"]
    for n in v["nodes"]:
        lines += ["  node [", f"    id {n}", "  ]"]
    for s, t, lat in v["edges"]:
        lines += ["  edge [", f"    source {s}", f"    target {t}", f'    latency "{lat}"', "  ]"]
    lines.append("]")
    return "\n".join(lines)


def test_xoshiro_splitmix_kats(oracle):
    L = oracle.load()
    st = (C.c_uint64 * 4)(1, 2, 3, 4)
    got = [L.ora_xoshiro_next_u64(st) for _ in range(10)]
    assert got == [int(x) for x in GOLD["crate_kats"]["xoshiro256plusplus_from_state_1_2_3_4"]["outputs"]]
    s = C.c_uint64(1234567)
    got = [L.ora_splitmix_next(C.byref(s)) for _ in range(5)]
    assert got == [int(x) for x in GOLD["crate_kats"]["splitmix64_seed_1234567"]["outputs"]]


def test_siphash_kats(oracle):
    L = oracle.load()
    k0 = int.from_bytes(bytes(range(8)), "little")
    k1 = int.from_bytes(bytes(range(8, 16)), "little")
    for ln, hexv in GOLD["crate_kats"]["siphash24_key_00_0f"]["by_len"].items():
        ln = int(ln)
        assert L.ora_siphash(2, 4, k0, k1, bytes(range(ln)), ln) == int(hexv, 16)


def test_f64_draw_matches_rand_definition(oracle):
    L = oracle.load()
    st = (C.c_uint64 * 4)(1, 2, 3, 4)
    st2 = (C.c_uint64 * 4)(1, 2, 3, 4)
    for _ in range(100):
        x = L.ora_xoshiro_next_u64(st)
        assert L.ora_xoshiro_next_f64(st2) == (x >> 11) * 2.0 ** -53


def test_host_seeds_library_matches_oracle(oracle, lib):
    names = sgn.host_names(500) + ["peer1", "server", "a", "", "x" * 100, "client_17"]
    for sim_seed in (1, 42, 0xFFFFFFFF):
        assert np.array_equal(oracle.host_seeds(sim_seed, names), sgn.derive_seeds(sim_seed, names))


def test_shortest_path_reference_vectors(oracle):
    v = GOLD["shortest_path"]
    for directed in (True, False):
        g, _ = oracle.gml_parse(ref_gml(directed))
        lat, loss = oracle.routes(g, v["nodes"])
        assert lat.tolist() == v["directed" if directed else "undirected"]
        assert (loss == 0).all()


def test_path_add(oracle):
    v = GOLD["path_add"]
    # a two-edge chain reproduces PathProperties::add (graph/mod.rs:316-325)
    g = sgn.GraphArrays([0, 1, 2], [0, 1, 2, 0, 1], [0, 1, 2, 1, 2],
                        [1, 1, 1, v["p1"][0], v["p2"][0]], [0, 0, 0, v["p1"][1], v["p2"][1]], False)
    lat, loss = oracle.routes(g, [0, 2])
    assert lat[0, 1] == v["latency"]
    assert abs(loss[0, 1] - v["loss"]) < v["tol"]
    # exact f32 left fold
    one = np.float32(1)
    exp = one - (one - np.float32(v["p1"][1])) * (one - np.float32(v["p2"][1]))
    assert loss[0, 1] == exp


def test_loss_fold_is_left_fold_not_associative(oracle):
    # the survey's counterexample: fold(fold(fold(0,.1),.2),.3) != fold(fold(0,.1),fold(.2,.3))
    g = sgn.GraphArrays([0, 1, 2, 3], [0, 1, 2, 3, 0, 1, 2], [0, 1, 2, 3, 1, 2, 3],
                        [1, 1, 1, 1, 5, 5, 5], [0, 0, 0, 0, 0.1, 0.2, 0.3], False)
    _, loss = oracle.routes(g, [0, 3])
    f = lambda a, b: np.float32(1) - (np.float32(1) - np.float32(a)) * (np.float32(1) - np.float32(b))
    assert loss[0, 1] == f(f(f(0, 0.1), 0.2), 0.3)
    assert f(f(f(0, 0.1), 0.2), 0.3) != f(f(0, 0.1), f(0.2, 0.3))


def test_nonexistent_id(oracle):
    v = GOLD["nonexistent_id"]
    for tgt, ok in ((v["ok_target"], True), (v["bad_target"], False)):
        text = f'graph [\n node [\n id 1\n ]\n node [\n id 3\n ]\n edge [\n source 1\n target {tgt}\n latency "1 ns"\n ]\n]'
        if ok:
            oracle.gml_parse(text)
        else:
            with pytest.raises(sgn.SgnError):
                oracle.gml_parse(text)


def test_ip_assignment(oracle):
    L = oracle.load()
    n = 600
    ips = np.zeros(n, dtype=np.uint32)
    flags = np.zeros(n, dtype=np.uint8)
    assert L.ora_assign_ips(n, flags.ctypes.data_as(C.POINTER(C.c_uint8)), sgn.ptr(ips, C.c_uint32)) == 0
    assert np.array_equal(ips, sgn.assign_ips(n))
    assert ips[0] == (11 << 24) + 1
    assert not np.isin(ips & 0xFF, [0, 255]).any()
    # 11.0.0.254 -> next skips .255 and .0 (test_increment_address_skip_broadcast)
    k = int(np.nonzero(ips == (11 << 24) + 254)[0][0])
    assert ips[k + 1] == (11 << 24) + 256 + 1
    # explicit addresses are taken first, automatic ones skip them
    flags[1] = 1
    ips2 = np.zeros(n, dtype=np.uint32)
    ips2[1] = (11 << 24) + 1
    L.ora_assign_ips(n, flags.ctypes.data_as(C.POINTER(C.c_uint8)), sgn.ptr(ips2, C.c_uint32))
    assert ips2[0] == (11 << 24) + 2 and len(set(ips2.tolist())) == n


def tb(oracle, cap, inc, interval_ns, now):
    t = oracle.TB()
    rc = oracle.load().ora_tb_new(cap, inc, interval_ns, now, C.byref(t))
    return t if rc == 0 else None


def tb_remove(oracle, t, dec, now):
    out = C.c_uint64()
    ok = oracle.load().ora_tb_remove(C.byref(t), dec, now, C.byref(out))
    return bool(ok), out.value


def test_token_bucket_reference(oracle):
    v = GOLD["token_bucket"]
    for cap, inc, interval in v["invalid"]:
        assert tb(oracle, cap, inc, interval, mock_ms(1000)) is None
    r = v["refill_after_one_interval"]
    now = mock_ms(r["now_ms"])
    t = tb(oracle, r["capacity"], r["increment"], r["interval_ms"] * MS, now)
    assert t.balance == r["capacity"]
    assert tb_remove(oracle, t, r["capacity"], now)[0] and t.balance == 0
    for i in range(1, r["capacity"] // r["increment"] + 1):
        ok, bal = tb_remove(oracle, t, 0, now + i * r["interval_ms"] * MS)
        assert ok and bal == t.balance == r["increment"] * i
    r = v["refill_after_multiple_intervals"]
    now = mock_ms(r["now_ms"])
    t = tb(oracle, r["capacity"], r["increment"], r["interval_ms"] * MS, now)
    tb_remove(oracle, t, r["capacity"], now)
    ok, bal = tb_remove(oracle, t, 0, now + r["later_ms"] * MS)
    assert ok and bal == r["balance"]
    r = v["capacity_limit"]
    now = mock_ms(r["now_ms"])
    t = tb(oracle, r["capacity"], r["increment"], r["interval_ms"] * MS, now)
    tb_remove(oracle, t, r["capacity"], now)
    ok, bal = tb_remove(oracle, t, 0, now + r["later_s"] * 1000 * MS)
    assert ok and bal == r["balance"]
    r = v["remove_error"]
    now = mock_ms(r["now_ms"])
    t = tb(oracle, r["capacity"], r["increment"], r["interval_ms"] * MS, now)
    assert tb_remove(oracle, t, r["capacity"], now) == (True, 0)
    assert tb_remove(oracle, t, r["remove"], now) == (False, r["dur_ms"] * MS)
    assert tb_remove(oracle, t, r["remove"], mock_ms(r["now_ms"] + r["inc_ms"])) == (False, r["dur2_ms"] * MS)


class Codel:
    def __init__(self, oracle):
        self.L = oracle.load()
        self.o = oracle
        self.q = self.L.ora_codel_new()

    def __del__(self):
        self.L.ora_codel_free(self.q)

    def push(self, now, wire=1028):
        self.L.ora_codel_push(self.q, wire, now)

    def pop(self, now):
        w = C.c_uint32()
        return self.L.ora_codel_pop(self.q, now, C.byref(w)) == 1

    def state(self):
        s = self.o.CodelState()
        self.L.ora_codel_get(self.q, C.byref(s))
        return s


def test_codel_reference(oracle):
    L = oracle.load()
    v = GOLD["codel"]
    I, T, ONE = v["interval_ns"], v["target_ns"], MS
    now = mock_ms(1000)
    for i in v["control_law_full_interval_counts"]:
        assert L.ora_codel_control_law(now, i) - now == I
    for i in range(2, 20):
        exp = int(np.floor(I / np.sqrt(i) + 0.5))
        assert L.ora_codel_control_law(now, i) - now == exp
    # push/pop simple
    q = Codel(oracle)
    for _ in range(10):
        q.push(now)
    assert all(q.pop(now) for _ in range(10)) and not q.pop(now)
    # interval
    q = Codel(oracle)
    start = mock_ms(1000)
    for _ in range(5):
        q.push(start)
    psd = lambda t, d: L.ora_codel_process_standing_delay(q.q, t, d)
    assert psd(start + T - ONE, T - ONE) == 0 and q.state().has_interval_end == 0
    assert psd(start + T, T) == 0 and q.state().interval_end == start + T + I
    assert psd(start + T + I, T + I) == 1 and q.state().interval_end == start + T + I
    assert psd(start + T + 2 * I, T + 2 * I) == 1
    assert psd(start + T + 2 * I, ONE) == 0 and q.state().has_interval_end == 0
    # mode
    q = Codel(oracle)
    N = v["mode_N"]
    for _ in range(N):
        q.push(start)
    q.pop(start + T - ONE)
    assert q.state().len == N - 1 and q.state().mode == 0
    q.pop(start + T)
    assert q.state().len == N - 2 and q.state().mode == 0
    q.pop(start + T + I - ONE)
    assert q.state().len == N - 3 and q.state().mode == 0
    q.pop(start + T + I)
    assert q.state().len == N - 5 and q.state().mode == 1
    for _ in range(3):
        q.push(start + T + 2 * I - ONE)
    q.pop(start + T + 2 * I)
    assert q.state().mode == 0
    # drop_empty
    q = Codel(oracle)
    L.ora_codel_set_mode(q.q, 1)
    q.pop(start)
    assert q.state().mode == 0
    # drop_many
    q = Codel(oracle)
    N = v["drop_many_N"]
    end = mock_ms(v["drop_many_end_ms"])
    for _ in range(N):
        q.push(start)
    q.pop(start + T)
    s = q.state()
    assert s.len == N - 1 and s.current_drop_count == 0 and s.previous_drop_count == 0
    assert L.ora_codel_was_dropping_recently(q.q, start + T) == 0
    q.pop(start + T + I)
    s = q.state()
    assert s.len == N - 3 and s.current_drop_count == 1 and s.previous_drop_count == 1
    assert s.has_drop_next == 1 and s.mode == 1
    assert L.ora_codel_was_dropping_recently(q.q, start + T + I) == 1
    assert L.ora_codel_should_drop(q.q, end) == 1
    q.pop(end)
    s = q.state()
    assert s.len == 1 and s.current_drop_count == N - 4 and s.mode == 0


@pytest.mark.parametrize("impl", ["oracle", "libsgn"])
def test_units_reference(oracle, lib, impl):
    v = GOLD["units"]
    if impl == "oracle":
        f = oracle.load().ora_units_parse
    else:
        f = lib.sgn_units_parse
    for kind, ok, err in ((0, v["time_ok"], v["time_err"]), (1, v["bytes_ok"], v["bytes_err"]),
                          (2, v["bits_ok"], v["bits_err"])):
        for s, exp in ok:
            out = C.c_uint64()
            assert f(kind, s.encode(), C.byref(out)) == 0, s
            assert out.value == exp, (s, out.value, exp)
        for s in err:
            out = C.c_uint64()
            assert f(kind, s.encode(), C.byref(out)) != 0, s


def test_one_gbit_switch_graph(oracle):
    v = GOLD["one_gbit_switch"]
    g, bws = oracle.gml_parse(v["gml"])
    assert bws == [(v["bw_bits"], v["bw_bits"])]
    lat, loss = oracle.routes(g, [0])
    assert lat[0, 0] == v["latency_ns"] and loss[0, 0] == 0
