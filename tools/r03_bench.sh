#!/bin/bash
# Benches of configs C, B and D on the GPU box (no CPU leg); $1 = tag, $2 = workloads (default "C B D").
set -u
T=${1:-x}; WS=${2:-C B D}
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in $WS; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 10 --no-cpu-baseline > gpurun_out/b${W}_$T.json 2> gpurun_out/b${W}_$T.err
  rc=$?; echo "BENCH_$W $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/b${W}_$T.err; exit $rc; }
  python - "$W" "gpurun_out/b${W}_$T.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(sys.argv[1], round(d["value"] / 1e6, 1), "M/s", r.get("kernel"), "round_us", (r.get("latency_bound") or {}).get("round_us"),
      "frac", r.get("frac"), "grid", d["engine"]["persistent_grid"], "held", d["engine"].get("rounds_held"))
PY
done
