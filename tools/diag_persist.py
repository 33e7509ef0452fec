"""Diagnostic: the persistent round kernel (k_rounds) with SGN_STAMPS=1 (product build plus a
few timer reads): per-round timeline of a 100-round launch (execution span, round edge,
wake-up) and, for the launch's last round, every group's shader cycles, gather / execute
split and start / end on the 100 MHz clock. Usage: diag_persist.py [C|B|D]"""
import os
import sys

os.environ["SGN_STAMPS"] = os.environ.get("SGN_STAMPS", "1")  # 2: + round timeline (perturbs)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "shadow-gen_amd"))
import numpy as np

import bench
import sgn

w = sys.argv[1] if len(sys.argv) > 1 else "C"
if w == "B":
    g, used, hosts, cfg, tr = bench.build_workload_b(10_000, 1000)
elif w == "D":
    g, used, hosts, cfg, tr = bench.build_workload_d(1_000_000, 1000)
    cfg.event_capacity = 257 * 15_626 * 192
else:
    g, used, hosts, cfg, tr = bench.build_workload(100_000, 1000)
ctx = sgn.Context(flags=3)
ctx.routes_build(g, used)
ctx.hosts_set(hosts)
ctx.sim_init(cfg, tr)
warm = 250 if w == "D" else 600
ctx.run(warm)
timeline = os.environ["SGN_STAMPS"] == "2"
tl = np.zeros(3 * 128, dtype=np.uint64)
if timeline:
    ctx.check(ctx.L.sgn_debug_rounds(ctx.h, sgn.ptr(tl, sgn.C.c_uint64)))  # reset
for rep in range(3):
    k0 = ctx.kernel_times()
    ctx.run(warm + 100 * (rep + 1))
    k1 = ctx.kernel_times()
    ms = sum(v[1] for v in k1.values()) - sum(v[1] for v in k0.values())
    print(f"[{w}] 100 rounds: {ms * 1e3 / 100:.1f} us per round (HIP events)")
    if timeline:
        ctx.check(ctx.L.sgn_debug_rounds(ctx.h, sgn.ptr(tl, sgn.C.c_uint64)))
        r = tl.reshape(128, 3)[:100].astype(np.int64)
        start, arr, edge = r[:, 0], r[:, 1], r[:, 2]
        span = (arr - start) / 100.0
        fin = (edge - arr) / 100.0
        wake = (start[1:] - edge[:-1]) / 100.0
        print(f"   timeline: exec span median {np.median(span):.1f} p90 {np.percentile(span, 90):.1f} | "
              f"round edge median {np.median(fin):.2f} | wake-up median {np.median(wake):.2f}")
    n = sgn.C.c_uint64()
    ctx.check(ctx.L.sgn_debug_stamps(ctx.h, None, 0, sgn.C.byref(n)))
    W = n.value
    out = np.zeros(sgn.STAMP_WORDS * W, dtype=np.uint64)
    ctx.check(ctx.L.sgn_debug_stamps(ctx.h, sgn.ptr(out, sgn.C.c_uint64), W, sgn.C.byref(n)))
    s = out.reshape(W, sgn.STAMP_WORDS).astype(np.int64)
    cyc, ev, mx, busy, runs, tg, tx, t0, t1 = (s[:, 0], s[:, 1], s[:, 2], s[:, 3], s[:, 4], s[:, 5], s[:, 6],
                                               s[:, 7], s[:, 30])
    obx = s[:, 8]
    base = t0.min()
    st_us, en_us = (t0 - base) / 100.0, (t1 - base) / 100.0
    mhz = np.median(cyc / np.maximum(t1 - t0, 1) * 100.0)
    print(f"   last round: groups={W} cycles p50={np.median(cyc):.0f} p90={np.percentile(cyc, 90):.0f} "
          f"p99={np.percentile(cyc, 99):.0f} max={cyc.max()} | gather p50={np.median(tg):.0f} exec p50={np.median(tx):.0f} "
          f"| start us p50={np.median(st_us):.2f} max={st_us.max():.2f} | end us p50={np.median(en_us):.1f} "
          f"p99={np.percentile(en_us, 99):.1f} max={en_us.max():.1f} | clock MHz {mhz:.0f}")
    order = np.argsort(en_us)[::-1]
    for i in order[:8]:
        print(f"     group {i:5d} end={en_us[i]:6.1f}us start={st_us[i]:5.2f} cycles={cyc[i]:7d} gather={tg[i]:6d} "
              f"exec={tx[i]:6d} busy={busy[i]:2d} events={ev[i]:5d} max_lane={mx[i]:4d} runs={runs[i]:4d} sent_recs={obx[i]:4d}")
    print(f"     records sent per group: p50={np.median(obx):.0f} max={obx.max()} groups past the outbox (24): {(obx > 24).sum()}")
    # the distribution of group cycles by kind of group (first groups are TGEN servers)
    dec = np.array_split(np.arange(W), 10)
    print("     cycles p50 by tenth of the groups: " + " ".join(f"{np.median(cyc[d]):.0f}" for d in dec))
