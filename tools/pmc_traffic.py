"""Per-launch HBM traffic of the round kernel (k_rounds: persistent, 100 rounds per launch in
the default bench; k_execute: one round per launch) from the FETCH_SIZE / WRITE_SIZE passes
of tools/pmc_traffic.sh, over the timed part of the default bench run (the last N
dispatches: 10 persistent launches, or 1000 per-round launches). Correction per MI355X_MICROARCH.md (HBM section):
FETCH_SIZE (KB) reports half the bytes of a coalesced read on gfx950, so it is doubled;
WRITE_SIZE (KB) is taken as is. Prints JSON."""
import csv
import json
import sys

d = sys.argv[1]
timed = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
# the bench workload the passes ran (bench.py matches on it before quoting "traffic")
workload = sys.argv[3] if len(sys.argv) > 3 else "C"
hosts = {"C": 100_000, "D": 1_000_000}[workload]


def per_dispatch(counter):
    global kern
    rows = list(csv.DictReader(open(f"{d}/{counter}/run_counter_collection.csv")))
    vals = {}
    for r in rows:
        if ("k_rounds" in r["Kernel_Name"] or "k_execute" in r["Kernel_Name"]) and \
                r["Counter_Name"] == counter:
            kern = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]  # template args dropped
            k = int(r["Dispatch_Id"])
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    v = [vals[k] for k in sorted(vals)]
    return v[-timed:]


kern = "?"
f = per_dispatch("FETCH_SIZE")
w = per_dispatch("WRITE_SIZE")
fetch = 2.0 * 1024 * sum(f) / len(f)
write = 1024 * sum(w) / len(w)
print(json.dumps({
    "kernel": kern, "dispatches_averaged": min(len(f), len(w)),
    "fetch_bytes_per_launch": round(fetch), "write_bytes_per_launch": round(write),
    "traffic_bytes_per_launch": round(fetch + write),
    "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE x1; KB -> bytes x1024",
    "workload": {"name": workload, "hosts_per_gpu": hosts, "graph_nodes": 1000,
                 "rounds_per_launch": 100, "n_gpus": 1},
    "bench_args": f"--workload {workload} (steps 10, warmup 5, {hosts} hosts, 1000 nodes, 100 rounds/step)",
}, indent=1))
