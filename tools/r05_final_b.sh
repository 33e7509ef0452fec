#!/bin/bash
# Round-5 closing measurements, part 2: keyed PMC traffic (FETCH_SIZE, WRITE_SIZE passes) of the
# driver's C invocation and of B and D (--steps 10 --warmup 5), then the B and D bench lines.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
for W in C B D; do
  bash tools/pmc_traffic.sh r05_$W $W 10 5 > gpurun_out/r05/traffic_$W.log 2>&1 || { echo "TRAFFIC $W failed"; exit 1; }
  cp gpurun_out/traffic_r05_$W/summary.json gpurun_out/r05/traffic_$W.json
  echo "TRAFFIC $W ok"
done
for W in B D; do
  timeout -k 10 400 python -u bench.py --workload $W --no-cpu-baseline > gpurun_out/r05/bench_$W.json 2> gpurun_out/r05/bench_$W.err || exit $?
  echo "BENCH $W ok"
done
