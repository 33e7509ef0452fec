#!/bin/bash
# APSP: GPU parity tests of the routing table, then build times at V = 1000 and 2000. Tag = $1.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k apsp --timeout 200 --timeout-method thread > gpurun_out/tapsp_$T.log 2>&1
rc=$?; echo "PYTEST $rc"; tail -3 gpurun_out/tapsp_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/apsp_bench.py > gpurun_out/apsp_$T.log 2>&1
rc=$?; echo "APSP $rc"; cat gpurun_out/apsp_$T.log; exit $rc
