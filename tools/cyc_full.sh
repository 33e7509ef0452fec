#!/bin/bash
# Full measurement cycle: parity, default bench (with the CPU baseline leg), rocprofv3 stats.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_$T.log 2>&1
rc=$?; echo "PYTEST $rc"; tail -2 gpurun_out/t_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo "BENCH $rc"; cat gpurun_out/bench_$T.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python -u bench.py --no-cpu-baseline > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "PROF $rc"; cat gpurun_out/prof_$T/run_kernel_stats.csv | cut -c1-150; exit $rc
