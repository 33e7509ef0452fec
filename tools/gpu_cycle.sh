#!/bin/bash
# One GPU-box cycle: parity tests, bench (no CPU leg), rocprofv3 kernel stats. Tag = $1.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_$T.log 2>&1
rc=$?; echo "PYTEST $rc"; tail -3 gpurun_out/t_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo "BENCH $rc"; cat gpurun_out/bench_$T.json; tail -3 gpurun_out/bench_$T.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "PROF $rc"; exit $rc
