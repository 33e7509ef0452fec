"""Per-launch HBM traffic of the round kernel (k_rounds: persistent, one launch per bench step
of 100 rounds; k_execute: one round per launch) from the FETCH_SIZE / WRITE_SIZE passes of
tools/pmc_traffic.sh over the timed launches of that bench invocation (the last `steps`
dispatches, or steps x 100 per-round ones). Correction per MI355X_MICROARCH.md (HBM section):
FETCH_SIZE (KB) reports half the bytes of a coalesced read on gfx950, so it is doubled;
WRITE_SIZE (KB) is taken as is; the uncorrected sum is kept beside it (the engine's scattered
8-32 B accesses are not the guide's calibrated pattern: tools/pmc_calib.sh measures them).
Prints one JSON entry keyed by the invocation (tools/traffic_merge.py files it)."""
import csv
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent.parent / "shadow-gen_amd"))
import sgn  # noqa: E402

d, workload, steps, warmup = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
hosts = {"B": 10_000, "C": 100_000, "D": 1_000_000}[workload]


def per_dispatch(counter):
    global kern
    rows = list(csv.DictReader(open(f"{d}/{counter}/run_counter_collection.csv")))
    vals = {}
    for r in rows:
        if ("k_rounds" in r["Kernel_Name"] or "k_execute" in r["Kernel_Name"]) and r["Counter_Name"] == counter:
            kern = "k_rounds" if "k_rounds" in r["Kernel_Name"] else "k_execute"
            k = int(r["Dispatch_Id"])
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    v = [vals[k] for k in sorted(vals)]
    timed = steps if kern == "k_rounds" else steps * 100
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
    "traffic_bytes_per_launch_uncorrected": round(fetch / 2 + write),
    "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE x1; KB -> bytes x1024",
    "workload": {"name": workload, "hosts_per_gpu": hosts, "graph_nodes": 1000, "rounds_per_launch": 100,
                 "n_gpus": 1, "steps": steps, "warmup": warmup},
    "bench_args": f"--workload {workload} --steps {steps} --warmup {warmup} (the timed launches of that invocation)",
    # the libsgn sources this was measured on: bench.py quotes the entry for that build only
    "build": sgn.build_id(),
}, indent=1))
