"""C-ABI surface and the host-side front end of libsgn (CPU only: no GPU calls).

* libsgn.so loads and exports every function include/sgn.h declares;
* the drop-in GML/units front end (sgn_gml_parse, sgn_units_parse) agrees with the oracle's
  independent restatement of lib/gml-parser + network/graph/mod.rs on the reference's own
  graphs and on a generated corpus of valid and invalid inputs;
* host-seed derivation and shard ranges.
"""
import ctypes as C
import json
import pathlib
import re
import subprocess

import numpy as np
import pytest

import sgn

ROOT = pathlib.Path(__file__).resolve().parent.parent
GOLD = json.loads((ROOT / "tests" / "golden" / "reference_unit_vectors.json").read_text())


def declared_functions():
    text = (ROOT / "include" / "sgn.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sgn_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(lib):
    names = declared_functions()
    assert len(names) >= 35
    out = subprocess.run(["nm", "-D", "--defined-only", str(sgn.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (sgn_[a-z0-9_]+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    extra = sorted(exported - set(names))
    assert not extra, f"undeclared exports: {extra}"
    for n in names:
        assert hasattr(lib, n)
    assert lib.sgn_abi_version() == 10


def test_struct_layouts_match_header(tmp_path):
    # the ctypes mirrors must match what a C compiler makes of include/sgn.h
    structs = {"sgn_graph": sgn.Graph, "sgn_hosts": sgn.Hosts, "sgn_sim_config": sgn.SimConfig,
               "sgn_traffic": sgn.Traffic, "sgn_stats": sgn.Stats, "sgn_host_digest": sgn.HostDigest,
               "sgn_trace_rec": sgn.TraceRec, "sgn_create_opts": sgn.CreateOpts,
               "sgn_routes_timing": sgn.RoutesTiming, "sgn_kernel_times": sgn.KernelTimes,
               "sgn_pkt_soa": sgn.PktSoa, "sgn_drain_rec": sgn.DrainRec,
               "sgn_engine_info": sgn.EngineInfo}
    src = tmp_path / "sz.c"
    body = "".join(f'  printf("{k} %zu\\n", sizeof({k}));\n' for k in structs)
    src.write_text(f'#include <stdio.h>\n#include "sgn.h"\nint main(void) {{\n{body}  return 0;\n}}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    sizes = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                         check=True).stdout.splitlines())
    for k, cls in structs.items():
        assert int(sizes[k]) == C.sizeof(cls), k


def test_shard_range_partitions(lib):
    for n in (1, 7, 100, 100_001):
        for k in (1, 2, 3, 8):
            spans = []
            for r in range(k):
                lo, hi = C.c_uint32(), C.c_uint32()
                assert lib.sgn_shard_range(n, r, k, C.byref(lo), C.byref(hi)) == 0
                spans.append((lo.value, hi.value))
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(k - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def lib_gml(lib, text):
    b = text.encode()
    h = C.c_void_p()
    err = C.create_string_buffer(512)
    rc = lib.sgn_gml_parse(b, len(b), C.byref(h), err, 512)
    if rc != 0:
        raise sgn.SgnError(rc, err.value.decode())
    g = sgn.Graph()
    lib.sgn_gml_graph(h, C.byref(g))
    n, e = g.n_nodes, g.n_edges
    arr = lambda p, k: np.ctypeslib.as_array(p, (k,)).copy() if k else np.zeros(0)
    out = (arr(g.node_id, n).tolist(), arr(g.edge_src, e).tolist(), arr(g.edge_dst, e).tolist(),
           arr(g.edge_latency_ns, e).tolist(), arr(g.edge_loss, e).view(np.uint32).tolist()
           if e else [], g.directed)
    bws = []
    for i in range(n):
        up, down = C.c_uint64(), C.c_uint64()
        hu, hd = C.c_int32(), C.c_int32()
        lib.sgn_gml_node_bandwidth(h, i, C.byref(up), C.byref(hu), C.byref(down), C.byref(hd))
        bws.append((up.value if hu.value else None, down.value if hd.value else None))
    lib.sgn_gml_free(h)
    return out, bws


def oracle_gml(oracle, text):
    g, bws = oracle.gml_parse(text)
    return (g.node_id.tolist(), g.src.tolist(), g.dst.tolist(), g.lat.tolist(),
            g.loss.view(np.uint32).tolist(), g.directed), bws


def same_outcome(lib, oracle, text):
    try:
        a = lib_gml(lib, text)
    except sgn.SgnError:
        a = "error"
    try:
        b = oracle_gml(oracle, text)
    except sgn.SgnError:
        b = "error"
    return a, b


def test_reference_graphs_parse_identically(lib, oracle):
    texts = [GOLD["one_gbit_switch"]["gml"]]
    for directed in (0, 1):
        v = GOLD["shortest_path"]
        lines = ["graph [", f"  directed {directed}"]
        for n in v["nodes"]:
            lines += ["  node [", f"    id {n}", "  ]"]
        for s, t, lat in v["edges"]:
            lines += ["  edge [", f"    source {s}", f"    target {t}", f'    latency "{lat}"', "  ]"]
        lines.append("]")
        texts.append("\n".join(lines))
    for t in texts:
        a, b = same_outcome(lib, oracle, t)
        assert a != "error" and a == b
    a, _ = same_outcome(lib, oracle, GOLD["one_gbit_switch"]["gml"])
    assert a[1] == [(10**9, 10**9)] and a[0][3] == [10**6]


BAD_OR_ODD = [
    'graph [\n node [\n id 1\n ]\n edge [\n source 1\n target 2\n latency "1 ns"\n ]\n]',  # unknown target
    'graph [\n node [\n id 0\n ]\n edge [\n source 0\n target 0\n latency "0 ms"\n ]\n]',  # zero latency
    'graph [\n node [\n id 0\n ]\n edge [\n source 0\n target 0\n latency "1 ms"\n packet_loss 0\n ]\n]',  # int loss
    'graph [\n node [\n id 0\n ]\n edge [\n source 0\n target 0\n latency "1 ms"\n packet_loss 1.5\n ]\n]',
    'graph [\n directed 2\n]',
    'graph [\n directed 1\n directed 0\n]',
    'graph [\n node [\n label "x"\n ]\n]',  # no id
    'graph [\n node [\n id 0\n id 1\n ]\n]',  # duplicate key
    'graph [\n node [\n id "a"\n ]\n]',
    'graph [\n node [\n id 0\n host_bandwidth_up 5\n ]\n]',
    'graph [\n node [\n id 0\n host_bandwidth_up "5 parsecs"\n ]\n]',
    'graph [\n node [\n id 0\n ]\n edge [\n source 0\n target 0\n latency "1 ms"\n jitter "3 ms"\n packet_loss 2.5e-1\n ]\n]',
    'graph [\n node [\n id 0\n ]\n edge [\n source 0\n target 0\n latency "1 ms"\n packet_loss .25\n ]\n]',
    'graph [\n node [\n id 0\n ]\n edge [\n source 0\n target 0\n latency "1 ms"\n packet_loss 1e\n ]\n]',
    'graph [\n label "g"\n node [\n id 4294967295\n ]\n]',  # id overflows i32 -> float -> bad id
    '  graph [\n  node [\n    id 3\n  ]\n]\ntrailing text is ignored',
    'graph[\nnode[\nid 0\n]\n]',
    'graph [ node [ id 0 ] ]',  # no newlines
    'graph [\n node [\n id 0\n ]\n edge [\n source 0\n target 0\n latency "10us"\n ]\n]',
    'graph [\n node [\n id 0\n ]\n edge [\n source 0\n target 0\n latency "10 \xce\xbcs"\n ]\n]',
]


@pytest.mark.parametrize("text", BAD_OR_ODD)
def test_edge_cases_agree(lib, oracle, text):
    a, b = same_outcome(lib, oracle, text)
    assert a == b


def random_gml(rng):
    V = int(rng.integers(1, 12))
    directed = int(rng.integers(0, 2))
    ids = rng.permutation(100)[:V]
    lines = ["graph [", f"  directed {directed}"]
    for i in ids:
        lines += ["  node [", f"    id {i}"]
        if rng.random() < 0.5:
            lines.append(f'    host_bandwidth_up "{int(rng.integers(1, 999))} {rng.choice(["Mbit", "Kbit", "Gbit", "bit", "Kibit"])}"')
        if rng.random() < 0.5:
            lines.append(f'    host_bandwidth_down "{int(rng.integers(1, 999))} Mbit"')
        lines.append("  ]")
    for _ in range(int(rng.integers(0, 3 * V))):
        s, t = rng.choice(ids, 2)
        unit = rng.choice(["ms", "us", "ns", "s", "min"])
        lines += ["  edge [", f"    source {s}", f"    target {t}",
                  f'    latency "{int(rng.integers(0 if rng.random() < 0.05 else 1, 500))} {unit}"']
        if rng.random() < 0.7:
            lines.append(f"    packet_loss {rng.choice(['0.0', f'{rng.random():.6f}', '1.0', '0.5e-2'])}")
        lines.append("  ]")
    lines.append("]")
    return "\n".join(lines)


def test_generated_corpus_agrees(lib, oracle):
    rng = np.random.default_rng(1234)
    n_ok = 0
    for _ in range(300):
        t = random_gml(rng)
        a, b = same_outcome(lib, oracle, t)
        assert a == b, t
        n_ok += a != "error"
    assert n_ok > 100
