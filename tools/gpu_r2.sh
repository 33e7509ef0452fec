#!/bin/bash
# Round-2 GPU cycle: all -m gpu tests, smoke, the default bench (CPU leg + parity). Tag = $1.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_$T.log 2>&1
rc=$?; echo "PYTEST $rc"; tail -4 gpurun_out/t_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; echo "SMOKE $rc"; tail -2 gpurun_out/smoke_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo "BENCH $rc"; cat gpurun_out/bench_$T.json; tail -3 gpurun_out/bench_$T.err; exit $rc
