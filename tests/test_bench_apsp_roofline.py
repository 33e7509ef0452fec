"""bench.py's APSP roofline block (CPU only): each form of the build is priced against the bound
it meets, with the algorithmic work of that form, and `frac` is achieved / peak. The inputs are
the `apsp` timing dicts libsgn reports (sgn_routes_timing, ABI 10), here as the closing C line
carried them and as the other forms report them."""
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

bench = pytest.importorskip("bench")

V = U = 1000
E = V * (V - 1)
BASE = {"loss_iters": 2, "tile": 64, "n_tight_edges": E, "latency_u64": 0, "latency_bf": 0, "shards": 1,
        "shard_sources": U}


def _check_fracs(out):
    for name in ("latency_phase", "loss_phase"):
        ph = out[name]
        assert ph["frac"] == pytest.approx(ph["achieved"] / ph["peak"], rel=0.02, abs=1e-4), name
        assert 0 < ph["frac"] < 1, name


def test_fused_form_prices_the_sweep_in_the_latency_phase():
    apsp = {**BASE, "total_ms": 0.16, "latency_ms": 0.114, "loss_ms": 0.018, "latency_passes": 1, "loss_multi": 16,
            "loss_dense": 1, "loss_fused": 1}
    out = bench.apsp_roofline(apsp, V, U)
    _check_fracs(out)
    lp, fp = out["latency_phase"], out["loss_phase"]
    # the latency phase did the tight sweep: 1.5 lane-ops per (source, arc) pair
    assert lp["bound"] == "valu" and lp["valu"]["lane_ops"] == int(1.5 * U * E)
    # the loss phase is the fold alone: priced against HBM, no VALU model
    assert fp["bound"] == "hbm" and "valu" not in fp
    assert "fused" in out["form"]["latency"] and "dense" in out["form"]["loss"]


def test_dense_and_csr_forms_price_the_sweep_in_the_loss_phase():
    for dense in (1, 0):
        apsp = {**BASE, "total_ms": 0.25, "latency_ms": 0.095, "loss_ms": 0.125, "latency_passes": 1,
                "loss_multi": 16 if dense else 8, "loss_dense": dense, "loss_fused": 0}
        out = bench.apsp_roofline(apsp, V, U)
        _check_fracs(out)
        Vp = -(-V // 64) * 64
        assert out["latency_phase"]["valu"]["lane_ops"] == int(1.5 * Vp ** 3)
        assert out["loss_phase"]["valu"]["lane_ops"] == int(1.5 * U * E)
        k = apsp["loss_multi"]
        l2 = 4.0 * V * V * -(-U // k) + 4.0 * U * V if dense else 8.0 * E * -(-U // k) + 4.0 * U * V
        assert out["loss_phase"]["l2_bytes"] == int(l2)
        assert ("dense" in out["form"]["loss"]) == bool(dense)


def test_sparse_form():
    apsp = {**BASE, "n_tight_edges": 6000, "total_ms": 0.13, "latency_ms": 0.07, "loss_ms": 0.034, "latency_passes": 12,
            "latency_u64": 1, "latency_bf": 1, "loss_multi": 0, "loss_dense": 0, "loss_fused": 0}
    out = bench.apsp_roofline(apsp, V, U)
    assert out["latency_phase"]["valu"]["lane_ops"] == int(1.5 * U * 6000 * 12)
    assert out["loss_phase"]["bound"] == "hbm"
    assert out["form"]["latency"] == "per-source relaxation"
