"""Randomised parity sweep (-m gpu): libsgn against the oracle on seeded random scenarios
that mix every option of the path at once — traffic kind (PERIODIC / TGEN), static and
dynamic runahead with bootstrapping, per-host bandwidths, lossy random and Tor-like graphs,
unknown destinations, send-queue and CoDel-pool sizes down to the blocking / page-reuse
regime, the interface qdisc, hosts per wave, small calendar slabs (extensions and the
big-slab path), host slot order, the peer table's form, and the round kernel (persistent
k_rounds or per-round k_execute, traced or not). Pools grow instead of refusing a scenario
(test_gpu_pools.py), so no case may be skipped. Bar: every counter, the final window and
every host's order-sensitive digests (tx / rx / app / RNG state / next event id) identical;
with the trace on, every per-packet record (IF_POP, SEND with drop decision and delivery
time, POP order, DELIVER, LOCAL, CODEL_DROP, RNG stream position) identical.

The scenarios are drawn from a fixed seed, so a failure names a reproducible case.
"""
import os

import numpy as np
import pytest

import sgn
from test_gpu_parity import assert_same_run, ctxf, run_both, scenario  # noqa: F401 (ctxf: fixture)

pytestmark = pytest.mark.gpu

CASES = int(os.environ.get("SGN_FUZZ_CASES", "32"))  # the round-end suite runs 32


def draw(i):
    r = np.random.default_rng(1000 + i)
    kind = sgn.TRAFFIC_TGEN if r.random() < 0.5 else sgn.TRAFFIC_PERIODIC
    n = int(r.integers(40, 400))
    V = int(r.integers(8, 60))
    dynamic = bool(r.random() < 0.3)
    bw_choices = np.array([1_000_000, 4_000_000, 10_000_000, 100_000_000, 1_000_000_000], dtype=np.uint64)
    bw = bw_choices[r.integers(0, len(bw_choices), n)]
    kw = dict(n=n, V=V, kind=kind, bw=bw, seed=int(r.integers(1, 1 << 30)), graph_seed=int(r.integers(1, 1000)),
              dynamic=dynamic, runahead_ns=0 if dynamic else int(r.choice([1_000_000, 2_000_000, 5_000_000])),
              bootstrap_ns=int(r.choice([0, 0, 50_000_000])), stop_ns=int(r.integers(200, 600)) * 1_000_000,
              unknown=int(r.choice([0, 10, 50])), fifo=int(r.choice([2, 8, 64])),
              codel=int(r.choice([160, 512, 4096])), tor=bool(r.random() < 0.5),
              qdisc=sgn.QDISC_ROUND_ROBIN if r.random() < 0.3 else 0)
    if kind == sgn.TRAFFIC_TGEN:
        kw["tgen_think"] = int(r.choice([10_000_000, 50_000_000, 200_000_000]))
    else:
        kw["period_ns"] = int(r.choice([500_000, 1_000_000, 10_000_000]))
    env = {"SGN_HOSTS_PER_WAVE": str(int(r.choice([16, 32, 64]))),
           "SGN_PERSISTENT": str(int(r.random() < 0.7))}
    trace = bool(r.random() < 0.5)
    if r.random() < 0.3:  # small slabs that stay small: spills, extensions and big-slab pieces
        env["SGN_SLAB_CAP"] = "16"
        env["SGN_SLAB_LIM"] = "32"
    # (drawn after the fields above, so earlier cases keep their parameters) host slots in
    # HostId order instead of kind / bandwidth / node order, and the 8-byte peer table
    if r.random() < 0.2:
        env["SGN_HOST_ORDER"] = "id"
    if r.random() < 0.2:
        env["SGN_PEER64"] = "1"
    return kw, env, trace


@pytest.mark.parametrize("case", range(CASES))
def test_random_scenario_bit_exact(ctxf, oracle, monkeypatch, case):
    kw, env, trace = draw(case)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    args = scenario(**kw)
    args[3].event_capacity = 1 << 23  # bootstrapping bursts fill the calendar's slabs faster
    # the pools grow (test_gpu_pools.py): no scenario may be refused, whatever its sizes
    o, c = run_both(ctxf, oracle, args, trace=trace)
    assert c.stats()["rounds"] > 0
    info = c.engine_info()
    assert info["codel_pages_free"] + info["codel_pages_chained"] == info["codel_pages"], (case, info)
    assert_same_run(o, c, args[2].n, trace=trace)
