#!/bin/bash
# Quick cycle: GPU parity tests (all), bench C and B without the CPU leg, round timelines.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_$T.log 2>&1
rc=$?; echo "PYTEST $rc"; tail -3 gpurun_out/t_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/benchC_$T.json 2> gpurun_out/benchC_$T.err
rc=$?; echo "BENCH_C $rc"; cut -c1-200 gpurun_out/benchC_$T.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload B --no-cpu-baseline > gpurun_out/benchB_$T.json 2> gpurun_out/benchB_$T.err
rc=$?; echo "BENCH_B $rc"; cut -c1-200 gpurun_out/benchB_$T.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/diag_rounds.py B > gpurun_out/diag_rounds_B_$T.log 2>&1 && tail -1 gpurun_out/diag_rounds_B_$T.log
timeout -k 10 200 python -u tools/diag_rounds.py > gpurun_out/diag_rounds_C_$T.log 2>&1 && tail -1 gpurun_out/diag_rounds_C_$T.log
