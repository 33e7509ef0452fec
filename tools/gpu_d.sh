#!/bin/bash
# Config D (1M hosts) on one GPU: bench line (no CPU leg) and the 1M-host parity test. Tag = $1.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload D --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/benchD_$T.json 2> gpurun_out/benchD_$T.err
rc=$?; echo "BENCH-D $rc"; cat gpurun_out/benchD_$T.json; tail -3 gpurun_out/benchD_$T.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -v -m gpu -k config_d --timeout 350 --timeout-method thread > gpurun_out/tD_$T.log 2>&1
rc=$?; echo "PYTEST-D $rc"; tail -4 gpurun_out/tD_$T.log; exit $rc
