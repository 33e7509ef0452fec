#!/bin/bash
# HBM traffic of k_execute from PMC counters over the default bench run (steps 10, warmup 5):
# one rocprofv3 pass per counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -u
T=${1:-x}
W=${2:-C}
mkdir -p gpurun_out/traffic_$T
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex 'k_rounds|k_execute' -d gpurun_out/traffic_$T/$c -o run --output-format csv -- python -u bench.py --workload $W --no-cpu-baseline > gpurun_out/traffic_$T/$c.log 2>&1
  rc=$?; echo "PASS $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_traffic.py gpurun_out/traffic_$T 10 $W > gpurun_out/traffic_$T/summary.json; cat gpurun_out/traffic_$T/summary.json
