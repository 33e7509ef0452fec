#!/bin/bash
# HBM traffic of the round kernel from PMC counters over one bench invocation: one rocprofv3
# pass per counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), for the exact
# bench arguments given (the entry is keyed by workload, steps and warmup: bench.py quotes it
# only for the same invocation). $1 = tag, $2 = workload, $3 = steps, $4 = warmup.
set -u
T=${1:-x}; W=${2:-C}; ST=${3:-20}; WU=${4:-5}
mkdir -p gpurun_out/traffic_$T
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex 'k_rounds|k_execute' -d gpurun_out/traffic_$T/$c -o run --output-format csv -- python -u bench.py --workload $W --steps $ST --warmup $WU --no-cpu-baseline > gpurun_out/traffic_$T/$c.log 2>&1
  rc=$?; echo "PASS $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_traffic.py gpurun_out/traffic_$T $W $ST $WU > gpurun_out/traffic_$T/summary.json; cat gpurun_out/traffic_$T/summary.json
