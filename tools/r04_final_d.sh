#!/bin/bash
# Round-4 closing run at head: the whole -m gpu suite, then the driver's bench invocation with
# the CPU leg and the rocprofv3 kernel stats of the same invocation. $1 = tag.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=10 > gpurun_out/all_$T.log 2>&1
rc=$?; echo "ALL $rc"; tail -3 gpurun_out/all_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_$T.json 2> gpurun_out/final_$T.err
rc=$?; echo "BENCH $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "PROF $rc"; exit $rc
