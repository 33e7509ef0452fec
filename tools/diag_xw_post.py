"""(Round 6 experiment, with libsgn_exp_xpost.so: SGN_LIB) The post-message phase of k_rounds_x
split by two extra stamps: 4 -> 5 the message words staged in LDS, 5 -> 6 the window, guards and
import counts computed, 6 -> 7 the rest of the round end. Per-workgroup timeline of the persistent multi-shard kernel (k_rounds_x) on one GPU
(SGN_STAMPS=3: every workgroup stores its own stamps, no shared words, so the timeline does
not slow the phases it times): config C's workload with H hosts as K shards of one local group.
Per round, on the 100 MHz clock (us), medians over 100 rounds:
  exec    = latest arrival - earliest start (over the shard's workgroups)
  arr_spread = latest - median arrival
  bar1    = last arriver knows it is last - latest arrival issue
  pub     = messages stored - bar1
  seen_1st  = first workgroup (any shard) with all messages - latest message stored
  seen_all  = last workgroup with all messages - latest message stored
  post    = median (round end - all messages seen) per workgroup
  gap     = next round's earliest start - latest round end
usage: python tools/diag_xw.py [hosts] [shards] [warmup_rounds] [C|D]"""
import ctypes as C
import os
import pathlib
import sys

import numpy as np

os.environ["SGN_STAMPS"] = "3"
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "shadow-gen_amd"))
import bench  # noqa: E402
import sgn  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 300
wl = sys.argv[4] if len(sys.argv) > 4 else "C"
if wl == "D":
    g, used, hosts, cfg, tr = bench.build_workload_d(n, 1000, stop_ns=3_000_000_000)
    cfg.event_capacity = 257 * -(-(-(-n // k)) // 64) * 128 * k  # (divided by k below)
else:
    g, used, hosts, cfg, tr = bench.build_workload(n, 1000)
ctxs = [sgn.Context(shard_rank=r, shard_count=k, flags=2) for r in range(k)]
arr = (C.c_void_p * k)(*[c.h.value for c in ctxs])
for c in ctxs:
    c.routes_build(g, used)
    c.hosts_set(hosts)
ctxs[0].check(ctxs[0].L.sgn_comm_init_local(arr, k, 1 << 13))
cfg = type(cfg).from_buffer_copy(cfg)
cfg.event_capacity = -(-cfg.event_capacity // k)
for c in ctxs:
    c.sim_init(cfg, tr)
done = C.c_uint64()
ctxs[0].check(ctxs[0].L.sgn_run_local_group(arr, k, warm, C.byref(done)))
buf = np.zeros(8 * 128 * 2048, dtype=np.uint64)
for c in ctxs:
    c.check(c.L.sgn_debug_rounds_xw(c.h, sgn.ptr(buf, C.c_uint64)))  # reset
ctxs[0].check(ctxs[0].L.sgn_run_local_group(arr, k, 100, C.byref(done)))
R = done.value
st = []
for c in ctxs:
    c.check(c.L.sgn_debug_rounds_xw(c.h, sgn.ptr(buf, C.c_uint64)))
    P = c.engine_info()["persistent_x_grid"]
    st.append(buf.reshape(128, 2048, 8)[:R, :P].astype(np.int64).copy())
post = []
for r in range(R - 1):
    for s in st:
        a4, a5, a6, a7 = (s[r, :, i] for i in (4, 5, 6, 7))
        post.append([np.median(a5 - a4), np.median(a6 - a5), np.median(a7 - a6), np.median(a7 - a4)])
m = np.median(np.array(post), axis=0) / 100.0
print(f"{n} hosts, {k} shards: stage {m[0]:.2f}  compute {m[1]:.2f}  rest {m[2]:.2f}  post {m[3]:.2f} (us, medians)")
