#!/bin/bash
# config C (the driver's invocation), B and D benches without the CPU leg; $1 = tag
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in C B D; do
  S=20; [ $W = C ] || S=10
  timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline --steps $S --warmup 5 > gpurun_out/bench${W}_$T.json 2> gpurun_out/bench${W}_$T.err
  rc=$?; echo "BENCH_$W $rc"; python3 -c "import json,sys; d=json.load(open('gpurun_out/bench${W}_$T.json')); r=d['roofline']; print('$W', round(d['value']/1e6,1), 'M/s', r['avg_launch_us'], 'us/launch', d['engine'])" ; [ $rc -eq 0 ] || exit $rc
done
