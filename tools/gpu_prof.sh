#!/bin/bash
# Profiles of the default bench command for profiles/: kernel-trace stats, then the PMC HBM
# traffic passes (tools/pmc_traffic.sh). Optional first step: extra pytest files ($2).
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${2:-}" ]; then
  timeout -k 10 300 python -u -m pytest $2 -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_$T.log 2>&1
  rc=$?; echo "PYTEST $rc"; tail -4 gpurun_out/t_$T.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python -u bench.py > gpurun_out/prof_bench_$T.json 2> gpurun_out/prof_bench_$T.err
rc=$?; echo "PROF $rc"; cat gpurun_out/prof_bench_$T.json; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_traffic.sh $T C
