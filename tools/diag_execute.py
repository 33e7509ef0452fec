"""Diagnostic: where does k_execute spend its time? Runs the bench workload with SGN_STAMPS
and prints per-wave (= per host group) shader cycles against the events its lanes handled."""
import os
import sys

os.environ["SGN_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "shadow-gen_amd"))
import numpy as np

import bench
import sgn

if len(sys.argv) > 1 and sys.argv[1] == "D":
    g, used, hosts, cfg, tr = bench.build_workload_d(1_000_000, 1000)
    cfg.event_capacity = 257 * 15_626 * 192
elif len(sys.argv) > 1 and sys.argv[1] == "B":
    g, used, hosts, cfg, tr = bench.build_workload_b(10_000, 1000)
else:
    g, used, hosts, cfg, tr = bench.build_workload(int(sys.argv[1]) if len(sys.argv) > 1 else 100_000, 1000)
ctx = sgn.Context(flags=2)
ctx.routes_build(g, used)
ctx.hosts_set(hosts)
ctx.sim_init(cfg, tr)
ctx.run(1000 if len(sys.argv) < 2 or sys.argv[1] != 'D' else 250)
n = sgn.C.c_uint64()
ctx.check(ctx.L.sgn_debug_stamps(ctx.h, None, 0, sgn.C.byref(n)))
W = n.value
for r in range(3):
    k0 = list(ctx.kernel_times().values())[0]
    ctx.round()
    k1 = list(ctx.kernel_times().values())[0]
    print(f"k_execute event-timed: {(k1[1] - k0[1]) * 1e3:.1f} us")
    out = np.zeros(sgn.STAMP_WORDS * W, dtype=np.uint64)
    ctx.check(ctx.L.sgn_debug_stamps(ctx.h, sgn.ptr(out, sgn.C.c_uint64), W, sgn.C.byref(n)))
    s = out.reshape(W, sgn.STAMP_WORDS).astype(np.int64)
    cyc, ev, mx, busy, runs = s[:, 0], s[:, 1], s[:, 2], s[:, 3], s[:, 4]
    tg, tx = s[:, 5], s[:, 6]
    order = np.argsort(cyc)[::-1]
    print(f"round {r}: waves={W} cycles max={cyc.max()} p50={np.median(cyc):.0f} p99={np.percentile(cyc, 99):.0f}"
          f" events total={ev.sum()} runs total={runs.sum()} max-lane={mx.max()}")
    for i in order[:12]:
        print(f"   wave {i:5d} cycles={cyc[i]:8d} events={ev[i]:5d} runs={runs[i]:4d} max_lane={mx[i]:4d}"
              f" busy_lanes={busy[i]:2d}  cyc/event={cyc[i] / max(ev[i], 1):7.1f} gather={tg[i]} exec={tx[i]}")
        if s[i, 80:91].any():
            tn = ["send", "fwdout", "fwdin", "pop", "rngloop", "app", "ld_codelhead", "ld_fifohead",
                  "ld_route", "ld_server", "slab_atomic", "draws(all lanes)", "draw-loop entries"]
            print("      wave cycles in: " + " ".join(f"{n}={s[i, 80 + k]}" for k, n in enumerate(tn)))
            if s[i, 92]:
                print(f"      rngloop cycles per entry {s[i, 84] / s[i, 92]:.0f}, per draw of the wave's lanes {s[i, 84] / max(1, s[i, 91]):.1f}"
                      f"; long-train (lane, entry) pairs {s[i, 93]} in {s[i, 94]} wave entries")
            sec = s[i, 81] + s[i, 82] + s[i, 83] + s[i, 85]
            print(f"      load={s[i, 32]} run={s[i, 33]} store={s[i, 34]} run-outside-handlers={s[i, 33] - sec}"
                  f" iterations={s[i, 35]} | cq_alloc={s[i, 10]} cq_free={s[i, 11]} tb_remove={s[i, 12]}")
    print(f"   median gather={np.median(tg):.0f} exec={np.median(tx):.0f}")
    if s[:, 80:91].any():
        tn = ["send", "fwdout", "fwdin", "pop", "rngloop", "app", "ld_codelhead", "ld_fifohead",
              "ld_route", "ld_server", "slab_atomic"]
        print("   section cycles median/p99/sum-share: " + " ".join(
            f"{n}={np.median(s[:, 80 + k]):.0f}/{np.percentile(s[:, 80 + k], 99):.0f}" for k, n in enumerate(tn)))
    if s[:, 32:35].any():
        wl, wr, ws_ = s[:, 32], s[:, 33], s[:, 34]
        print(f"   wave phases (diag build) median: load={np.median(wl):.0f} run={np.median(wr):.0f} store={np.median(ws_):.0f}"
              f" | p99: load={np.percentile(wl, 99):.0f} run={np.percentile(wr, 99):.0f} store={np.percentile(ws_, 99):.0f}")
        it = s[:, 35:40]
        print(f"   wave loop iterations median: all={np.median(it[:, 0]):.0f} pop={np.median(it[:, 1]):.0f} ro={np.median(it[:, 2]):.0f} ri={np.median(it[:, 3]):.0f} app={np.median(it[:, 4]):.0f}"
              f" | run cycles/iteration median={np.median(wr / np.maximum(it[:, 0], 1)):.0f}")
        ct, cn = s[:, 48:64].sum(0), s[:, 64:80].sum(0)
        names = ["pop", "ro", "ri", "app"]
        rows = [m for m in range(16) if cn[m] > 0]
        for m in rows:
            print(f"     iter combo {'+'.join(n for k, n in enumerate(names) if m >> k & 1) or 'none':16s} n={cn[m]:7d} cycles/iter={ct[m] / cn[m]:8.0f}")
        A = np.array([[(m >> k) & 1 for k in range(4)] + [1] for m in rows], dtype=float)
        w = np.sqrt(cn[rows].astype(float))
        coef, *_ = np.linalg.lstsq(A * w[:, None], (ct[rows] / cn[rows]) * w, rcond=None)
        print("     per-handler cycles (fit): " + " ".join(f"{n}={c:.0f}" for n, c in zip(names + ["base"], coef)))
        top = np.argsort(cyc)[::-1][:3]
        for i in top:
            print(f"     top wave {i}: iters={it[i].tolist()} run={wr[i]} cyc/iter={wr[i] / max(it[i, 0], 1):.0f}")
    r0, r1 = s[:, 7], s[:, 30]
    t0 = r0.min()
    st_us, en_us = (r0 - t0) / 100.0, (r1 - t0) / 100.0
    clk = cyc / np.maximum((r1 - r0) / 100.0, 1e-3)  # cycles per us = MHz
    print(f"   wave start us: p0={st_us.min():.1f} p50={np.median(st_us):.1f} p99={np.percentile(st_us, 99):.1f} max={st_us.max():.1f}"
          f" | end us: p50={np.median(en_us):.1f} max={en_us.max():.1f} | clock MHz p50={np.median(clk):.0f}")
    late = np.argsort(en_us)[::-1][:5]
    print("   last to finish: " + ", ".join(f"w{i} start={st_us[i]:.1f} end={en_us[i]:.1f} cyc={cyc[i]}" for i in late))
    sel = ev > 0
    A = np.stack([ev[sel], mx[sel], runs[sel], np.ones(sel.sum())], 1)
    coef, *_ = np.linalg.lstsq(A, cyc[sel], rcond=None)
    print(f"   fit cycles ~ {coef[0]:.1f}*events + {coef[1]:.1f}*max_lane + {coef[2]:.1f}*runs + {coef[3]:.0f}")
