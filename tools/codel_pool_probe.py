"""Probe: the CoDel page pool on the TGEN CoDel stress scenario of tests/test_gpu_parity.py —
pages allocated (and whether the pool sufficed) for several codel_cap values."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "shadow-gen_amd")]
import sgn
from test_gpu_parity import scenario

bw = np.where(np.arange(300) % 10 == 0, 100_000_000, 4_000_000).astype(np.uint64)
stop = int(os.environ.get("STOP_S", "2")) * 1_000_000_000
for cap in [int(x) for x in sys.argv[1:]] or [16, 64, 256, 1024]:
    g, used, hosts, cfg, tr = scenario(n=300, V=30, kind=sgn.TRAFFIC_TGEN, stop_ns=stop, bw=bw,
                                       tor=True, tgen_think=200_000_000, codel=cap)
    c = sgn.Context(device=0)
    c.routes_build(g, used)
    c.hosts_set(hosts)
    c.sim_init(cfg, tr)
    try:
        c.run()
        ok = True
    except sgn.SgnError as e:
        ok = str(e)[:80]
    info = c.engine_info()
    print(cap, "pages", info["codel_pages"], "allocs", info["codel_page_allocs"], "free", info["codel_pages_free"],
          "chained", info["codel_pages_chained"], "ok", ok, flush=True)
    c.close()
