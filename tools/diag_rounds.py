"""Diagnostic: per-round timeline of the persistent round kernel (SGN_STAMPS=1): execution
span (earliest start -> latest arrival), round edge, and barrier wake-up to the next start."""
import os
import sys

os.environ["SGN_STAMPS"] = "2"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "shadow-gen_amd"))
import numpy as np

import bench
import sgn

if len(sys.argv) > 1 and sys.argv[1] == "B":
    g, used, hosts, cfg, tr = bench.build_workload_b(10_000, 1000)
else:
    g, used, hosts, cfg, tr = bench.build_workload(100_000, 1000)
ctx = sgn.Context(flags=2)
ctx.routes_build(g, used)
ctx.hosts_set(hosts)
ctx.sim_init(cfg, tr)
out = np.zeros(3 * 128, dtype=np.uint64)
ctx.run(600)
ctx.check(ctx.L.sgn_debug_rounds(ctx.h, sgn.ptr(out, sgn.C.c_uint64)))  # reset
ctx.run(100)
ctx.check(ctx.L.sgn_debug_rounds(ctx.h, sgn.ptr(out, sgn.C.c_uint64)))
r = out.reshape(128, 3)[:100].astype(np.int64)
start, arr, edge = r[:, 0], r[:, 1], r[:, 2]
span = (arr - start) / 100.0
fin = (edge - arr) / 100.0
wake = (start[1:] - edge[:-1]) / 100.0
tot = (start[1:] - start[:-1]) / 100.0
print(f"round us: total median {np.median(tot):.1f} | exec span median {np.median(span):.1f} p90 {np.percentile(span, 90):.1f}"
      f" | round edge median {np.median(fin):.2f} | wake-up median {np.median(wake):.2f}")
