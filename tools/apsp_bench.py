"""APSP build time at the bench's graph (V=1000 Tor-like complete graph), several builds:
the first includes code-object loading; later ones are the steady-state build time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "shadow-gen_amd"))
import numpy as np

import bench
import sgn

V = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
g, used, hosts, cfg, tr = bench.build_workload(10_000, V)
ctx = sgn.Context()
for i in range(4):
    ctx.routes_build(g, used)
    print(i, ctx.routes_timing(), flush=True)
