"""Headline benchmark: simulated packet events/s (whole node) at 100k hosts + APSP build time.

Workload (BASELINE.json configs[2], "config C", the one the metric is quoted on: it fits a
single MI355X): 100k synthetic hosts per GPU on a Tor-like 1000-node complete graph
(latency 1 ms + 5..150 ms distance term, loss 0..0.5 %), Zipf(1.0) host placement,
bandwidth classes 10M/100M/1G, 10 % servers; clients fetch 50 KiB / 1 MiB / 5 MiB files as
1500 B UDP trains paced only by token buckets and CoDel (no TCP congestion control: the
TCP stack is outside the GPU core). Synthetic data, seeded.

A step = ROUNDS_PER_STEP simulation rounds (Shadow scheduling windows). A packet event =
one send_packet call past the DNS check (sent or loss-dropped) or one packet event popped
at its destination. value = all ranks' packet events / max-rank wall time.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU, hosts sharded, RCCL exchange inside libsgn).
"""
import argparse
import json
import os
import pathlib
import subprocess
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "shadow-gen_amd"))
import sgn  # noqa: E402

METRIC = "simulated packet events/sec (whole node) at 100k hosts; APSP build time"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def build_workload(n_hosts, V, seed=1):
    g = sgn.tor_graph(V, seed=42)
    used = np.arange(V, dtype=np.uint32)
    names = sgn.host_names(n_hosts)
    seeds = sgn.derive_seeds(seed, names)
    node = sgn.zipf_nodes(n_hosts, V, seed=5)
    bw = sgn.bandwidth_classes(n_hosts, seed=3)
    hosts = sgn.HostArrays(sgn.assign_ips(n_hosts), node, bw, bw, seeds)
    rng = np.random.default_rng(11)
    servers = np.sort(rng.choice(n_hosts, size=max(1, n_hosts // 10), replace=False)).astype(np.uint32)
    # first fetch uniform over one mean think time: the fetch process is stationary from t=0
    tr = sgn.make_traffic(sgn.TRAFFIC_TGEN, flow_seed=7, start_ns=0, start_jitter_ns=3_000_000_000,
                          period_ns=2_000_000_000, period_jitter_ns=2_000_000_000,
                          req_payload=64, servers=servers,
                          file_bytes=(50 * 1024, 1024 * 1024, 5 * 1024 * 1024))
    cfg = sgn.make_config(3600 * 1_000_000_000, runahead_ns=1_000_000, out_fifo_cap=64,
                          codel_cap=4096, event_capacity=1 << 24)
    return g, used, hosts, cfg, tr


def events_of(st):
    return st["packets_sent"] + st["packets_loss_dropped"] + st["packet_events_popped"]


def cpu_baseline(g, used, hosts, cfg, tr, args, budget_s):
    """The oracle (CPU restatement of the reference's round loop, with the reference's own
    parallel structure: worker threads over host chunks, per-host queue locks, a barrier per
    round) on the same workload and the SAME rounds the GPU timed: warm-up rounds untimed,
    then the timed rounds (bounded by budget_s), then a single-thread sample."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_py

    threads = max(1, min(16, os.cpu_count() or 1))
    t_apsp = time.perf_counter()
    lat, loss = oracle_py.routes(g, used)  # per-source Dijkstra (graph/mod.rs:181-226), 1 thread
    apsp_s = time.perf_counter() - t_apsp
    sim = oracle_py.Sim(used, lat, loss, hosts, cfg, tr, threads=threads)
    sim.run(args.warmup * args.rounds_per_step)

    def timed(rounds_max, budget):
        st0 = sim.stats()
        t0 = time.perf_counter()
        done = 0
        while done < rounds_max and time.perf_counter() - t0 < budget:
            done += sim.run(min(50, rounds_max - done))
        el = time.perf_counter() - t0
        return events_of(sim.stats()) - events_of(st0), el, done

    ev, el, rounds = timed(args.steps * args.rounds_per_step, budget_s)
    sim.L.ora_sim_set_threads(sim.h, 1)
    ev1, el1, rounds1 = timed(args.steps * args.rounds_per_step, budget_s / 3)
    return {
        "value": ev / el,
        "unit": "packet events/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle round loop ({threads} worker threads) over the same {hosts.n}-host "
                  f"workload and the same rounds the GPU timed (rounds "
                  f"{args.warmup * args.rounds_per_step}..{args.warmup * args.rounds_per_step + rounds}"
                  f", {ev} packet events, {el:.1f} s wall; warm-up rounds untimed)",
        "apsp_ms": round(apsp_s * 1e3, 1),
        "apsp_sample": "the oracle's per-source Dijkstra over the same graph (1 thread)",
        "single_core": {"value": ev1 / el1, "cores": 1,
                        "sample": f"the next {rounds1} rounds on 1 thread ({ev1} packet events, {el1:.1f} s)"},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--hosts", type=int, default=100_000, help="hosts per GPU")
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--rounds-per-step", type=int, default=100)
    ap.add_argument("--cpu-budget-s", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")
    n_total = args.hosts * world
    g, used, hosts, cfg, tr = build_workload(n_total, args.nodes)

    ctx = sgn.Context(device=local, shard_rank=rank, shard_count=world,
                      flags=2)  # SGN_CREATE_TIME_EXECUTE: HIP events around the round kernel
    ctx.routes_build(g, used)
    apsp_first = ctx.routes_timing()  # includes loading the APSP kernels' code object
    ctx.routes_build(g, used)         # steady state: the build time proper
    apsp = ctx.routes_timing()
    ctx.hosts_set(hosts)
    if world > 1:
        import torch
        idb = (sgn.C.c_uint8 * 128)()
        if rank == 0:
            ctx.check(ctx.L.sgn_comm_get_unique_id(idb))
        t = torch.tensor(list(bytes(idb)), dtype=torch.uint8)
        dist.broadcast(t, 0)
        idb = (sgn.C.c_uint8 * 128)(*t.tolist())
        # per-peer exchange slot: 8192 event runs (256 KB) per round; a round sends ~700 runs
        # per peer at 100k hosts per GPU (overflow is detected and reported, never silent)
        ctx.check(ctx.L.sgn_comm_init(ctx.h, idb, 1 << 13))
    ctx.sim_init(cfg, tr)

    def barrier():
        if dist:
            dist.barrier()

    for _ in range(args.warmup):
        ctx.run(args.rounds_per_step)
    st0 = ctx.stats()
    # the round kernel: k_rounds (persistent, many rounds per launch) or k_execute
    rk = "k_rounds" if "k_rounds" in ctx.kernel_times() else "k_execute"
    kt0 = ctx.kernel_times()[rk]
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.run(args.rounds_per_step)
    barrier()
    el = time.perf_counter() - t0
    st1 = ctx.stats()
    kt1 = ctx.kernel_times()[rk]
    ev = events_of(st1) - events_of(st0)
    if dist:
        import torch
        m = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        el = float(m.item())
        e = torch.tensor([ev], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.SUM)
        ev = int(e.item())
    d = {k: st1[k] - st0[k] for k in st1}
    rounds = d["rounds"]
    # roofline of the dominant kernel (k_rounds on one shard, k_execute multi-shard): algorithmic bytes per launch
    # = SURVEY.md §8(d)'s packet-path model, 128 B per packet (send record, DNS, node
    # indices, route entry, event record write, sort/merge, pop read) + 96 B per active
    # host-round (RNG state, event-id counter, queue head), over the units one launch
    # processes, / the launch's average duration (HIP events on the engine stream).
    launches = kt1[0] - kt0[0]
    exec_ms = kt1[1] - kt0[1]
    n_pkt = d["packets_sent"] + d["packets_loss_dropped"]
    host_exec = d["host_executions"]
    alg_bytes = 128 * n_pkt + 96 * host_exec
    roof = None
    if launches and exec_ms > 0:
        avg_s = exec_ms / launches / 1e3
        achieved = alg_bytes / launches / avg_s / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                "kernel": rk, "avg_launch_us": round(avg_s * 1e6, 2),
                "alg_bytes_per_launch": int(alg_bytes / launches),
                "units_per_launch": {"packets": round(n_pkt / launches, 1),
                                     "active_host_rounds": round(host_exec / launches, 1)}}
        # HBM bytes per launch measured by PMC (tools/pmc_traffic.sh: FETCH_SIZE x2 +
        # WRITE_SIZE over the same default run's timed dispatches), when it matches this run
        tf = ROOT / "profiles" / "round_kernel_traffic.json"
        default_run = (args.hosts, args.nodes, args.rounds_per_step, args.steps, args.warmup,
                       world) == (100_000, 1000, 100, 10, 5, 1)
        if tf.exists() and default_run:
            t = json.loads(tf.read_text())
            roof["traffic"] = t["traffic_bytes_per_launch"]
            roof["traffic_unit"] = "bytes/launch (PMC, profiles/round_kernel_traffic.json)"
            roof["traffic_GBps"] = round(t["traffic_bytes_per_launch"] / avg_s / 1e9, 2)
    out = {
        "metric": METRIC,
        "value": ev / el,
        "unit": "packet events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {
            "workload": "C: Tor-like 1000-node complete graph, tgen-style UDP trains",
            "hosts_per_gpu": args.hosts, "hosts_total": n_total, "graph_nodes": args.nodes,
            "rounds_per_step": args.rounds_per_step, "runahead_ms": 1,
            "parallelism": f"host-shard x{world}",
        },
        "apsp_build_ms": round(apsp["total_ms"], 3),
        "apsp": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in apsp.items()},
        "apsp_first_build_ms": round(apsp_first["total_ms"], 3),
        "sim_ms_per_step": None,
        "rounds_timed": rounds,
        "packet_events_timed": ev,
        "roofline": roof,
        "cpu_baseline": None,
        "max_slab_fill": st1["max_pending_events"],
    }
    ws, _, _ = ctx.window()
    out["sim_time_reached_ms"] = (ws - sgn.SIMULATION_START) / 1e6
    out["sim_ms_per_step"] = out["sim_time_reached_ms"] / (args.steps + args.warmup)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(g, used, hosts, cfg, tr, args, args.cpu_budget_s)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
