#!/bin/bash
# Round-4 GPU cycle: $1 = tag, $2 = pytest selection for the first step (default: the pool tests),
# then the whole -m gpu suite and a config-C bench without the CPU leg.
set -u
T=${1:-x}
SEL=${2:-tests/test_gpu_pools.py}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest $SEL -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/sel_$T.log 2>&1
rc=$?; echo "SEL $rc"; tail -5 gpurun_out/sel_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=25 > gpurun_out/all_$T.log 2>&1
rc=$?; echo "ALL $rc"; tail -30 gpurun_out/all_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/benchC_$T.json 2> gpurun_out/benchC_$T.err
rc=$?; echo "BENCH_C $rc"; cut -c1-300 gpurun_out/benchC_$T.json; exit $rc
