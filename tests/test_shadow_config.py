"""shadow.yaml front end (a5 IP assignment): shadow_config.py and
sgn_assign_ips against the reference's own data.

* MyTest/shadow.yaml -> the merged configuration equals the reference's own output for it,
  MyTest/shadow.data/processed-config.yaml (core/manager.rs:253);
* every configuration the reference's integration harness runs (src/test/**, examples/**),
  with the argv that harness builds (src/test/CMakeLists.txt:62-131): accepted, or rejected
  exactly where the harness says EXPECT_ERROR (duplicate hosts, hostname characters, a start
  time past stop_time);
* the command-line merge table of configuration.rs:1515-1639 (NullableOption);
* deny_unknown_fields at every level, serde_yaml scalar typing, '<<' merges and 'x-' keys;
* units, GML, IPs and seeds go through libsgn's C ABI and agree with the oracle.
All CPU-only: the library is loaded, nothing is launched on a GPU.
"""
import json
import lzma
import pathlib

import numpy as np
import pytest

import sgn
import shadow_config as sc

GOLD = json.loads((pathlib.Path(__file__).parent / "golden" / "reference_configs.json").read_text(encoding="utf-8"))

MINI = """
general:
  stop_time: 1 min
  {general}
network:
  graph:
    type: 1_gbit_switch
{extra}
hosts:
  myhost:
    network_node_id: 0
    processes:
    - path: /bin/true
"""


def mini(general="", extra="", argv=()):
    return sc.load(text=MINI.format(general=general, extra=extra), argv=argv)


def test_mytest_matches_reference_processed_config():
    cfg = sc.load(text=GOLD["mytest"]["config"])
    want = sc.load_yaml(GOLD["mytest"]["processed"])
    got = cfg.processed()
    assert got == want
    assert list(got["hosts"]) == list(want["hosts"])  # BTreeMap (hostname) order


@pytest.mark.parametrize("t", GOLD["tests"], ids=[t["name"] for t in GOLD["tests"]])
def test_reference_harness_configs(t, tmp_path):
    cli = sc.parse_cli(t["argv"])
    assert cli.config == t["config"]
    text = GOLD["corpus"][t["config"]]["text"]
    try:
        cfg = sc.ConfigOptions.new(sc.parse_config_file(sc.load_yaml(text)), cli)
        base = None
        graph = cfg.network["graph"]
        if "file" in graph:
            rel = str(pathlib.PurePosixPath(t["config"]).parent / graph["file"]["path"])
            raw = GOLD["graphs"][rel.removesuffix(".xz")].encode()
            dst = tmp_path / graph["file"]["path"]
            dst.write_bytes(lzma.compress(raw, format=lzma.FORMAT_XZ) if graph["file"]["compression"] == "xz" else raw)
            base = tmp_path
        setup = sc.sim_setup(cfg, base_dir=base)
    except sc.ConfigError as e:
        assert t["expect_error"], f"{t['config']}: {e}"
        return
    assert not t["expect_error"], f"{t['config']} should be rejected"
    # harness flags reached the merged configuration
    assert cfg.experimental["use_cpu_pinning"] == ("--use-cpu-pinning true" in " ".join(t["argv"]))
    assert cfg.general["data_directory"] == t["name"] + ".data"
    want_qdisc = sgn.QDISC_ROUND_ROBIN if "round-robin" in t["argv"] else sgn.QDISC_FIFO
    assert setup.qdisc == want_qdisc
    assert len(setup.names) == len(cfg.hosts) == setup.hosts.n
    assert len(set(setup.hosts.ip.tolist())) == setup.hosts.n


def test_every_corpus_config():
    n_err = 0
    for rel, c in GOLD["corpus"].items():
        try:
            cfg = sc.load(text=c["text"], argv=GOLD["harness_args"])
            if "file" not in cfg.network["graph"]:
                sc.sim_setup(cfg)
        except sc.ConfigError:
            assert c["expect_error"], rel
            n_err += 1
            continue
        assert not c["expect_error"], rel
    assert n_err == 3 and len(GOLD["corpus"]) >= 150


def test_expected_errors_name_the_cause():
    msgs = {}
    for rel, c in GOLD["corpus"].items():
        if c["expect_error"]:
            with pytest.raises(sc.ConfigError) as ei:
                sc.sim_setup(sc.load(text=c["text"]))
            msgs[pathlib.PurePosixPath(rel).stem] = str(ei.value)
    assert "duplicate" in msgs["error-on-duplicate-hosts"]
    assert "invalid hostname character: '_'" in msgs["hostname-invalid-characters"]
    assert "must be earlier than the simulation stop time" in msgs["small_stop_time"]


@pytest.mark.parametrize("file_opt,cli,want", [
    # configuration.rs:1515-1639 (heartbeat_interval is Option<NullableOption<Time>>)
    ("heartbeat_interval: null", [], None),
    ("heartbeat_interval: null", ["--heartbeat-interval", "5s"], "5 sec"),
    ("heartbeat_interval: null", ["--heartbeat-interval", "null"], sc.NULL),
    ("heartbeat_interval: 5s", [], "5 sec"),
    ("heartbeat_interval: 5s", ["--heartbeat-interval", "5s"], "5 sec"),
    ("heartbeat_interval: 5s", ["--heartbeat-interval", "null"], sc.NULL),
    ("", [], "1 sec"),
    ("", ["--heartbeat-interval", "5s"], "5 sec"),
    ("", ["--heartbeat-interval", "null"], sc.NULL),
])
def test_nullable_option_merge(file_opt, cli, want):
    got = mini(file_opt, argv=cli).general["heartbeat_interval"]
    assert (got if got is None or got is sc.NULL else str(got)) == want


def test_runahead_and_sim_fields():
    s = sc.sim_setup(mini())
    assert (s.runahead_ns, s.use_dynamic_runahead, s.qdisc, s.seed) == (1_000_000, False, sgn.QDISC_FIFO, 1)
    assert s.stop_time_ns == 60 * 10**9 and s.bootstrap_end_ns == 0 and s.use_shortest_path
    exp = "experimental:\n  runahead: null\n  use_dynamic_runahead: true\n  interface_qdisc: round-robin"
    s = sc.sim_setup(mini("seed: 7\n  bootstrap_end_time: 2s", exp))
    assert (s.runahead_ns, s.use_dynamic_runahead, s.qdisc, s.seed, s.bootstrap_end_ns) == \
        (0, True, sgn.QDISC_ROUND_ROBIN, 7, 2 * 10**9)
    # the command line wins over the file, "null" clears a NullableOption
    s = sc.sim_setup(mini("", exp, ["--runahead", "5 ms", "--interface-qdisc", "fifo", "--seed", "9",
                                    "--use-shortest-path", "false"]))
    assert (s.runahead_ns, s.qdisc, s.seed, s.use_shortest_path) == (5_000_000, sgn.QDISC_FIFO, 9, False)
    assert sc.sim_setup(mini("", "", ["--runahead", "null"])).runahead_ns == 0
    c = s.sim_config(out_fifo_cap=64, codel_cap=4096, event_capacity=1 << 16)
    assert (c.stop_time_ns, c.runahead_ns, c.interface_qdisc) == (60 * 10**9, 5_000_000, sgn.QDISC_FIFO)


@pytest.mark.parametrize("extra,frag", [
    ("bogus: 1", "unknown field `bogus`"),
    ("experimental:\n  use_cpu_pinnin: true", "unknown field `use_cpu_pinnin`"),
    ("host_option_defaults:\n  pcap: true", "unknown field `pcap`"),
    ("experimental:\n  interface_qdisc: lifo", "unknown variant `lifo`"),
    ("experimental:\n  strace_logging_mode: no", "unknown variant `no`"),
    ("experimental:\n  runahead: -1", "out of range"),
    ("experimental:\n  runahead: 1.5", "invalid type"),
    ("experimental:\n  runahead: 5 parsecs", "unknown unit prefix"),
    ("experimental:\n  socket_send_buffer: 10 Kbit", "unknown unit prefix"),
    ("experimental:\n  use_new_tcp: yes", "expected a boolean"),
])
def test_rejected_fields(extra, frag):
    with pytest.raises(sc.ConfigError, match=frag):
        mini("", extra)


def test_rejected_structure():
    base = MINI.format(general="", extra="")
    for bad, frag in [
        (base.replace("general:\n  stop_time: 1 min\n", ""), "missing field `general`"),
        (base.replace("  stop_time: 1 min", "  stop_tim: 1 min"), "unknown field `stop_tim`"),
        (base.replace("    type: 1_gbit_switch", "    type: gml\n    inline: a\n    file: {path: b}"), "exactly one"),
        (base.replace("    type: 1_gbit_switch", "    type: graphml"), "unknown variant `graphml`"),
        (base.replace("    type: 1_gbit_switch", "    type: gml\n    file: {path: g.gml, compression: gz}"), "unknown variant `gz`"),
        (base.replace("    network_node_id: 0", "    network_node_id: 0\n    bandwith_up: 1 Gbit"), "unknown field `bandwith_up`"),
        (base.replace("    - path: /bin/true", "    - path: /bin/true\n      argv: x"), "unknown field `argv`"),
        (base.replace("    - path: /bin/true", "    - path: /bin/true\n      shutdown_signal: SIGFOO"), "Invalid signal"),
        (base.replace("    - path: /bin/true", "    - path: /bin/true\n      environment: {A=B: x}"), "'='"),
        (base.replace("    network_node_id: 0", "    network_node_id: 0\n    ip_addr: 11.0.0.01"), "invalid IP"),
        (base.replace("  myhost:", "  -myhost:"), "begins with a '-'"),
        (base.replace("  myhost:", "  MyHost:"), "invalid hostname character: 'M'"),
        (base.replace("  myhost:", "  123:"), "string hostname"),
        (base + "  myhost:\n    network_node_id: 0\n    processes: []\n", "duplicate"),
    ]:
        with pytest.raises(sc.ConfigError, match=frag):
            sc.load(text=bad)
    with pytest.raises(sc.ConfigError, match="unexpected argument '--bogus'"):
        sc.load(text=base, argv=["--bogus", "1"])
    with pytest.raises(sc.ConfigError, match="invalid value 'yes' for bool"):
        sc.load(text=base, argv=["--progress", "yes"])


def test_yaml_scalars_follow_serde_yaml():
    r = sc._resolve_plain
    assert [r(x) for x in ("off", "yes", "010", "0x10", "0o17", "0b11", "-7", "+7", "1.5", "1e3", "~", "")] == \
        ["off", "yes", "010", 16, 15, 3, -7, 7, 1.5, 1000.0, None, None]
    assert r("1_000") == "1_000" and r(".inf") == float("inf") and r("TRUE") is True
    # quoted scalars stay strings: a quoted seed is not a u32, a quoted time is a time string
    with pytest.raises(sc.ConfigError, match="u32"):
        mini('seed: "1"')
    assert mini('bootstrap_end_time: "3"').general["bootstrap_end_time"].base() == 3 * 10**9


def test_merge_keys_anchors_and_extension_fields():
    text = """
x-defaults: &defaults
  network_node_id: 1
  bandwidth_down: 10 Mbit
  processes:
  - path: /bin/true
    start_time: 2
general:
  stop_time: 10
network:
  graph:
    type: gml
    inline: |
      graph [
        node [
          id 0
        ]
        node [
          id 1
          host_bandwidth_up "100 Mbit"
          host_bandwidth_down "100 Mbit"
        ]
        edge [
          source 0
          target 1
          latency "5 ms"
        ]
      ]
hosts:
  b-host:
    <<: *defaults
    network_node_id: 0
  a-host:
    <<: [*defaults, {bandwidth_up: 1 Gbit}]
  c-host: *defaults
"""
    cfg = sc.load(text=text)
    assert list(cfg.hosts) == ["a-host", "b-host", "c-host"]
    assert [h["network_node_id"] for h in cfg.hosts.values()] == [1, 0, 1]
    assert str(cfg.hosts["a-host"]["bandwidth_up"]) == "1 Gbit"
    s = sc.sim_setup(cfg)
    # sim_config.rs:249-254: the host-side up value is taken from bandwidth_down
    assert s.hosts.bw_up.tolist() == s.hosts.bw_down.tolist() == [10_000_000] * 3
    assert s.used_nodes.tolist() == [0, 1]
    assert s.process_start_ns == [[2 * 10**9]] * 3
    with pytest.raises(sc.ConfigError, match="merge"):
        sc.load(text=text.replace("<<: *defaults", "<<: 5"))


def test_bandwidth_sources_and_node_checks():
    gml = ('graph [\\n node [\\n id 0\\n host_bandwidth_up \\"2 Mbit\\"\\n host_bandwidth_down \\"3 Mbit\\"\\n ]\\n'
           ' node [\\n id 4\\n ]\\n edge [\\n source 0\\n target 4\\n latency \\"1 ms\\"\\n ]\\n]')
    cfg_t = ("general: {stop_time: 5}\nnetwork:\n  graph: {type: gml, inline: \"%s\"}\nhosts:\n"
             "  a:\n    network_node_id: 0\n    processes: []\n%s")
    s = sc.sim_setup(sc.load(text=cfg_t % (gml, "")))
    assert (int(s.hosts.bw_up[0]), int(s.hosts.bw_down[0])) == (2_000_000, 3_000_000)
    with pytest.raises(sc.ConfigError, match="No downstream bandwidth provided for host 'b'"):
        sc.sim_setup(sc.load(text=cfg_t % (gml, "  b:\n    network_node_id: 4\n    processes: []\n")))
    with pytest.raises(sc.ConfigError, match="network node id 9 for host 'b' does not exist"):
        sc.sim_setup(sc.load(text=cfg_t % (gml, "  b:\n    network_node_id: 9\n    processes: []\n")))
    s = sc.sim_setup(sc.load(text=cfg_t % (gml, "  b:\n    network_node_id: 4\n    bandwidth_down: 7 Kibit\n    processes: []\n")))
    assert s.hosts.bw_up.tolist() == [2_000_000, 7168] and s.hosts.bw_down.tolist() == [3_000_000, 7168]
    with pytest.raises(sc.ConfigError, match="did not contain any hosts"):
        sc.sim_setup(sc.load(text="general: {stop_time: 5}\nnetwork: {graph: {type: 1_gbit_switch}}\nhosts: {}\n"))
    with pytest.raises(sc.ConfigError, match="host to debug 'zz'"):
        sc.sim_setup(sc.load(text=cfg_t % (gml, "")), debug_hosts=["zz"])


def test_seeds_and_ips_through_the_abi(oracle):
    hosts = "".join(f"  h{i:03d}:\n    network_node_id: 0\n    processes: []\n" +
                    ("    ip_addr: 11.0.0.%d\n" % (i // 2) if i % 7 == 3 else "") for i in range(40))
    text = "general: {stop_time: 5, seed: 42}\nnetwork: {graph: {type: 1_gbit_switch}}\nhosts:\n" + hosts
    s = sc.sim_setup(sc.load(text=text))
    assert s.names == sorted(s.names)
    assert np.array_equal(s.hosts.seed, oracle.host_seeds(42, s.names))
    explicit = {i: (11 << 24) + i // 2 for i in range(40) if i % 7 == 3}
    rc, want = oracle.assign_ips(40, explicit)
    assert rc == 0 and np.array_equal(s.hosts.ip, want)
    assert all(s.hosts.ip[i] == v for i, v in explicit.items())
    assert s.hosts.bw_up.tolist() == [1_000_000_000] * 40  # 1_gbit_switch node bandwidth


def test_assign_ips_native_equals_oracle(oracle):
    rng = np.random.default_rng(11)
    for trial in range(200):
        n = int(rng.integers(0, 600))
        explicit = {}
        for i in rng.choice(max(n, 1), size=min(n, int(rng.integers(0, 40))), replace=False) if n else []:
            # mostly inside the dynamic range (collisions to skip), some anywhere, some .0/.255
            base = (11 << 24) + int(rng.integers(0, 2 * n + 10))
            explicit[int(i)] = base if trial % 3 else int(rng.integers(1, 1 << 32))
        rc_o, ips_o = oracle.assign_ips(n, explicit)
        if rc_o == 0:
            assert np.array_equal(sgn.assign_ips(n, explicit), ips_o), trial
        else:
            with pytest.raises(sgn.SgnError, match="already been assigned"):
                sgn.assign_ips(n, explicit)
    # the host whose registration fails is the first repeat in HostId order
    with pytest.raises(sgn.SgnError, match="host 2:"):
        sgn.assign_ips(4, {0: 0x0B000005, 1: 0x0B000009, 2: 0x0B000009, 3: 0x0B000005})
    # the dynamic sequence skips .255/.0 and configured addresses (graph/mod.rs:400-417)
    ips = sgn.assign_ips(3, {0: 0x0B000001})
    assert ips.tolist() == [0x0B000001, 0x0B000002, 0x0B000003]
    L = sgn.load()
    flags = np.zeros(1, np.uint8)
    one = np.array([0], np.uint32)
    assert L.sgn_assign_ips(1, sgn.ptr(flags, sgn.C.c_uint8), sgn.ptr(one, sgn.C.c_uint32), None) == 0
    assert one[0] == (11 << 24) + 1


@pytest.mark.parametrize("kind", ["time", "bytes", "bits"])
def test_units_agree_with_libsgn(lib, kind):
    k = {"time": 0, "bytes": 1, "bits": 2}[kind]
    cases = ["10 ms", "10ms", " 3 min ", "5", "+5 s", "-5 s", "1.5 s", "18446744073709551615 ns",
             "18446744073709551615 s", "1 μs", "1 µs", "10 Mbit", "10Mibit", "81920 Kibit", "7 Ki",
             "1 GiB", "1 gibibyte", "1 gibi", "2 bytes", "2 B", "3 bits", "", "x", "1 hour", "2 hrs"]
    for s in cases:
        out = sgn.C.c_uint64()
        rc = lib.sgn_units_parse(k, s.encode(), sgn.C.byref(out))
        try:
            v = sc.Unit.parse(kind, s).base()
        except sc.ConfigError:
            assert rc != 0, (kind, s)
            continue
        assert rc == 0 and out.value == v, (kind, s)


def test_xz_graph_file_equals_inline(tmp_path):
    gml = GOLD["graphs"]["src/test/compressed-graph/graph-compressed.gml"]
    (tmp_path / "g.gml.xz").write_bytes(lzma.compress(gml.encode(), format=lzma.FORMAT_XZ))
    (tmp_path / "g.gml").write_text(gml)
    body = "general: {stop_time: 5}\nnetwork:\n  graph:\n    type: gml\n%s\nhosts:\n  a: {network_node_id: 0, processes: []}\n"
    a = sc.sim_setup(sc.load(text=body % "    file: {path: g.gml.xz, compression: xz}"), base_dir=tmp_path)
    b = sc.sim_setup(sc.load(text=body % "    file: {path: g.gml}"), base_dir=tmp_path)
    c = sc.sim_setup(sc.load(text=body % ("    inline: " + json.dumps(gml))))
    for x in (a, b):
        assert np.array_equal(x.graph.lat, c.graph.lat) and np.array_equal(x.graph.src, c.graph.src)
        assert np.array_equal(x.hosts.bw_down, c.hosts.bw_down)
    with pytest.raises(sc.ConfigError, match="Failed to load the network graph"):
        sc.sim_setup(sc.load(text=body % "    file: {path: g.gml, compression: xz}"), base_dir=tmp_path)
