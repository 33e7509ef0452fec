"""Diagnostic: where does k_execute spend its time? Runs the bench workload with SGN_STAMPS
and prints per-wave cycle counts against the events the wave's lanes handled."""
import os
import sys

os.environ["SGN_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "shadow-gen_amd"))
import numpy as np

import bench
import sgn

g, used, hosts, cfg, tr = bench.build_workload(int(sys.argv[1]) if len(sys.argv) > 1 else 100_000, 1000)
lib = sgn.load(sgn.HERE / "libsgn_diag.so")
ctx = sgn.Context(lib=lib)
ctx.routes_build(g, used)
ctx.hosts_set(hosts)
ctx.sim_init(cfg, tr)
ctx.run(1000)
n = sgn.C.c_uint64()
ctx.check(ctx.L.sgn_debug_stamps(ctx.h, None, 0, sgn.C.byref(n)))
W = n.value
for r in range(3):
    ctx.round()
    out = np.zeros(16 * W, dtype=np.uint64)
    ctx.check(ctx.L.sgn_debug_stamps(ctx.h, sgn.ptr(out, sgn.C.c_uint64), W, sgn.C.byref(n)))
    s = out.reshape(W, 16).astype(np.int64)
    cyc, ev, mx, busy = s[:, 0], s[:, 1], s[:, 2], s[:, 3]
    order = np.argsort(cyc)[::-1]
    print(f"round {r}: waves={W} cycles max={cyc.max()} p50={np.median(cyc):.0f} p99={np.percentile(cyc, 99):.0f}"
          f" events total={ev.sum()} max-lane={mx.max()}")
    for i in order[:12]:
        print(f"   wave {i:5d} cycles={cyc[i]:8d} events={ev[i]:5d} max_lane={mx[i]:4d} busy_lanes={busy[i]:2d}"
              f"  cyc/event={cyc[i] / max(ev[i], 1):7.1f}")
        p = s[i, 4:11]
        pn = [s[i, 11] & 0xFFFFFFFF, s[i, 11] >> 32, s[i, 12] & 0xFFFFFFFF, s[i, 12] >> 32]
        c = [s[i, 13] & 0xFFFFFFFF, s[i, 13] >> 32, s[i, 14] & 0xFFFFFFFF, s[i, 14] >> 32]
        print(f"      lane0: pop {p[0]}c/{pn[0]} chunks, ro {p[1]}c/{pn[1]}, ri {p[2]}c/{pn[2]}, app {p[3]}c/{pn[3]}"
              f" | load {p[4]} run {p[6]} store {p[5]} | {s[i, 15] * 10} ns | popped {c[0]} sends {c[1]} deliv {c[2]} codel {c[3]}")
    sel = ev > 0
    A = np.stack([ev[sel], mx[sel], np.ones(sel.sum())], 1)
    coef, *_ = np.linalg.lstsq(A, cyc[sel], rcond=None)
    print(f"   fit cycles ~ {coef[0]:.1f}*events + {coef[1]:.1f}*max_lane + {coef[2]:.0f}")
