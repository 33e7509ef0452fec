"""Per-round phase timeline of the persistent multi-shard kernel (k_rounds_x) on one GPU: config
C's workload (bench.build_workload) with H hosts as K shards of one local group, SGN_STAMPS=2.
Per shard and phase, the median over the rounds of one launch (us, 100 MHz clock):
exec = latest local arrival - earliest start; bar1 = local barrier seen - latest arrival;
pub = messages sent - barrier seen; wait = latest "all messages seen" - messages sent;
file = latest imports filed - latest seen; bar2 = latest second barrier seen - latest filed;
gap = next round's earliest start - this round's latest bar2.

usage: python tools/diag_xpersist.py [hosts] [shards] [warmup_rounds]"""
import ctypes as C
import os
import pathlib
import sys

import numpy as np

os.environ["SGN_STAMPS"] = "2"
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "shadow-gen_amd"))
import bench  # noqa: E402
import sgn  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 300
g, used, hosts, cfg, tr = bench.build_workload(n, 1000)
if k == 1:  # the single-shard persistent kernel's own timeline: {earliest start, latest arrival,
    # round edge known by the bookkeeping workgroup} (sgn_debug_rounds, 3 words per round)
    c = sgn.Context(flags=2)
    c.routes_build(g, used)
    c.hosts_set(hosts)
    c.sim_init(cfg, tr)
    c.run(warm)
    b3 = np.zeros(3 * 128, dtype=np.uint64)
    c.check(c.L.sgn_debug_rounds(c.h, sgn.ptr(b3, C.c_uint64)))
    c.run(100)
    c.check(c.L.sgn_debug_rounds(c.h, sgn.ptr(b3, C.c_uint64)))
    t = b3.reshape(128, 3)[:100].astype(np.int64)
    d = np.stack([t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], np.append(t[1:, 0] - t[:-1, 2], 0)], axis=1) / 100.0
    med = np.median(d[:-1], axis=0)
    print(f"one shard: exec {med[0]:6.2f}  edge {med[1]:6.2f}  gap {med[2]:6.2f}  round {np.median(np.diff(t[:, 0])) / 100:.2f} us")
    sys.exit(0)
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
buf = np.zeros(8 * 128, dtype=np.uint64)
for c in ctxs:
    c.check(c.L.sgn_debug_rounds_x(c.h, sgn.ptr(buf, C.c_uint64)))  # reset
ctxs[0].check(ctxs[0].L.sgn_run_local_group(arr, k, 100, C.byref(done)))
names = ("exec", "bar1", "pub", "wait", "file", "bar2", "gap")
rows = []
for r, c in enumerate(ctxs):
    c.check(c.L.sgn_debug_rounds_x(c.h, sgn.ptr(buf, C.c_uint64)))
    t = buf.reshape(128, 8)[: done.value].astype(np.int64)
    d = np.stack([t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[:, 4] - t[:, 3],
                  np.where(t[:, 5] > 0, t[:, 5] - t[:, 4], 0), np.where(t[:, 6] > 0, t[:, 6] - t[:, 5], 0),
                  np.append(t[1:, 0] - np.maximum(t[:-1, 6], t[:-1, 4]), 0)], axis=1) / 100.0
    med = np.median(d[:-1], axis=0)
    rows.append(med)
    print(f"shard {r}: " + "  ".join(f"{nm} {v:6.2f}" for nm, v in zip(names, med)) +
          f"  round {np.median(np.diff(t[:, 0])) / 100:.2f} us")
print("mean   : " + "  ".join(f"{nm} {v:6.2f}" for nm, v in zip(names, np.mean(rows, axis=0))))
