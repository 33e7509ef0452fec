#!/bin/bash
# The randomised parity sweep at N cases (default 400) on the GPU box; $1 = tag.
set -u
T=${1:-x}; N=${2:-400}
mkdir -p gpurun_out
export TMPDIR=/tmp SGN_FUZZ_CASES=$N
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/fuzz_$T.log 2>&1
rc=$?; echo "FUZZ $rc"; tail -4 gpurun_out/fuzz_$T.log; exit $rc
