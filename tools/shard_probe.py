"""Repeat the two-shard local-group run against one shard (diagnostic): slot / slab-cap variants."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, "shadow-gen_amd")
sys.path.insert(0, "tests")
import sgn  # noqa: E402
from test_gpu_pools import _codel_args  # noqa: E402


def run(slot, cap, rep):
    if cap:
        os.environ["SGN_SLAB_CAP"] = str(cap)
    else:
        os.environ.pop("SGN_SLAB_CAP", None)
    n = 300
    g, used, hosts, cfg, tr = _codel_args(n=n)
    one = sgn.Context()
    one.routes_build(g, used)
    one.hosts_set(hosts)
    one.sim_init(cfg, tr)
    one.run()
    shards = [sgn.Context(shard_rank=r, shard_count=2) for r in range(2)]
    arr = (C.c_void_p * 2)(*[s.h.value for s in shards])
    for s in shards:
        s.routes_build(g, used)
        s.hosts_set(hosts)
    shards[0].check(shards[0].L.sgn_comm_init_local(arr, 2, slot))
    for s in shards:
        s.sim_init(cfg, tr)
    done = C.c_uint64()
    shards[0].check(shards[0].L.sgn_run_local_group(arr, 2, 1 << 40, C.byref(done)))
    bad = []
    for r, s in enumerate(shards):
        lo, hi = C.c_uint32(), C.c_uint32()
        s.L.sgn_shard_range(n, r, 2, C.byref(lo), C.byref(hi))
        d1, d2 = one.digests(lo.value, hi.value), s.digests(lo.value, hi.value)
        for f in ("tx", "rx", "app", "rng", "next_event_id"):
            k = np.nonzero(d1[f] != d2[f])[0] if d1[f].ndim == 1 else np.nonzero((d1[f] != d2[f]).any(1))[0]
            if len(k):
                bad.append((r, f, len(k), int(lo.value + k[0])))
    info = [s.engine_info() for s in shards]
    print(f"slot={slot} cap={cap} rep={rep} rounds {done.value}/{one.stats()['rounds']} mismatches={bad} "
          f"held={[i['rounds_held'] for i in info]} xgrows={[i['exchange_slot_grows'] for i in info]} "
          f"cgrows={[i['calendar_grows'] for i in info]}", flush=True)


for slot, cap in ((16, 16), (16, 0), (1 << 16, 16), (16, 16)):
    for rep in range(2):
        run(slot, cap, rep)
