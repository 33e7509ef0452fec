#!/bin/bash
# Round-end rehearsal on the GPU box: all -m gpu tests, smoke(), the default bench (with its
# CPU leg), rocprofv3 kernel stats of the same bench, then PMC traffic. Tag = $1.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_$T.log 2>&1
rc=$?; echo "PYTEST $rc"; tail -3 gpurun_out/t_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; echo "SMOKE $rc"; tail -3 gpurun_out/smoke_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo "BENCH $rc"; cat gpurun_out/bench_$T.json; tail -3 gpurun_out/bench_$T.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python -u bench.py --no-cpu-baseline > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "PROF $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_traffic.sh $T
