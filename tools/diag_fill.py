"""Diagnostic: calendar slab high-water mark and per-round load of the bench workload.

Runs the bench workload (config C) for N rounds and prints the stats that size the device
capacities (max (bucket, group) slab fill, max CoDel ring length)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "shadow-gen_amd"))
import bench  # noqa: E402
import sgn  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
cap = int(sys.argv[2]) if len(sys.argv) > 2 else 0
g, used, hosts, cfg, tr = bench.build_workload(100_000, 1000)
if cap:
    cfg.event_capacity = cap
ctx = sgn.Context(flags=2)
ctx.routes_build(g, used)
ctx.hosts_set(hosts)
ctx.sim_init(cfg, tr)
t0 = time.perf_counter()
done = 0
while done < rounds:
    done += ctx.run(500)
    st = ctx.stats()
    el = time.perf_counter() - t0
    print(f"rounds {st['rounds']} t={el:.2f}s max_slab_fill={st['max_pending_events']} "
          f"max_codel={st['max_codel_len']} runs={st['event_runs']} popped={st['packet_events_popped']} "
          f"sent={st['packets_sent']} exec_hosts={st['host_executions']} kt={ctx.kernel_times()['k_execute']}",
          flush=True)
