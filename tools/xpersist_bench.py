"""Per-round cost of the persistent multi-shard round (k_rounds_x) on ONE GPU, against the
single-shard persistent round (k_rounds): config C's workload (bench.build_workload) with H hosts
in total, run as K shards of one local group — every shard a range of workgroups of one launch —
or as one shard. Prints one JSON line per configuration: HIP-event kernel time per round, wall
time per round, events per second, and (K > 1) the engine's exchange figures.

usage: python tools/xpersist_bench.py [--hosts 12500,100000] [--shards 1,2,8] [--rounds 500]
       [--warmup 200] [--workload C|D|B]"""
import argparse
import ctypes as C
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "shadow-gen_amd"))
import bench  # noqa: E402
import sgn  # noqa: E402


def workload(name, n, k=1):
    if name == "C":
        return bench.build_workload(n, 1000)
    if name == "B":
        return bench.build_workload_b(n, 1000)
    g, used, hosts, cfg, tr = bench.build_workload_d(n, 1000, stop_ns=3_000_000_000)
    # (bench.py's sizing: 128-run slabs per host group of a shard, 257 slab sets)
    cfg.event_capacity = 257 * -(-(-(-n // k)) // 64) * 128
    return g, used, hosts, cfg, tr


def run(name, n, k, rounds, warmup):
    g, used, hosts, cfg, tr = workload(name, n, k)
    if k == 1:
        ctxs = [sgn.Context(flags=2)]
    else:
        ctxs = [sgn.Context(shard_rank=r, shard_count=k, flags=2) for r in range(k)]
    arr = (C.c_void_p * k)(*[c.h.value for c in ctxs])
    for c in ctxs:
        c.routes_build(g, used)
        c.hosts_set(hosts)
    if k > 1:
        ctxs[0].check(ctxs[0].L.sgn_comm_init_local(arr, k, 1 << 13))
        cfg = type(cfg).from_buffer_copy(cfg)
        if name != "D":
            cfg.event_capacity = -(-cfg.event_capacity // k)
    for c in ctxs:
        c.sim_init(cfg, tr)

    def go(nr):
        if k == 1:
            return ctxs[0].run(nr)
        done = C.c_uint64()
        ctxs[0].check(ctxs[0].L.sgn_run_local_group(arr, k, nr, C.byref(done)))
        return done.value

    go(warmup)
    ev0 = sum(bench.events_of(c.stats()) for c in ctxs)
    kname = "k_rounds" if k == 1 else "k_rounds_x"
    kt0 = ctxs[0].kernel_times().get(kname, (0, 0.0))
    t0 = time.perf_counter()
    done = go(rounds)
    el = time.perf_counter() - t0
    kt1 = ctxs[0].kernel_times().get(kname, (0, 0.0))
    ev = sum(bench.events_of(c.stats()) for c in ctxs) - ev0
    info = ctxs[0].engine_info()
    out = {"workload": name, "hosts": n, "shards": k, "rounds": done, "kernel": kname,
           "kernel_us_per_round": round((kt1[1] - kt0[1]) * 1e3 / max(1, done), 2),
           "wall_us_per_round": round(el * 1e6 / max(1, done), 2),
           "events_per_s": round(ev / el), "launches": kt1[0] - kt0[0],
           "grid": [c.engine_info()["persistent_x_grid"] if k > 1 else info["persistent_grid"] for c in ctxs],
           "exchange_mode": info["exchange_mode"]}
    if k > 1:
        out.update({"inbox_slot_runs": info["inbox_slot_runs"], "inbox_grows": info["inbox_grows"],
                    "exchange_hwm_runs": info["exchange_hwm_runs"]})
    print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hosts", default="12500,100000")
    ap.add_argument("--shards", default="1,2,8")
    ap.add_argument("--rounds", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--workload", default="C")
    a = ap.parse_args()
    for n in [int(x) for x in a.hosts.split(",")]:
        for k in [int(x) for x in a.shards.split(",")]:
            run(a.workload, n, k, a.rounds, a.warmup)


if __name__ == "__main__":
    main()
