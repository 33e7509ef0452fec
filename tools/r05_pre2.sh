#!/bin/bash
# TGEN second-bucket prefetch: parity of the round kernels, then same-box A/B against HEAD's build.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_xpersist.py tests/test_gpu_fuzz.py > gpurun_out/r05/pre2_tests.log 2>&1 || { tail -30 gpurun_out/r05/pre2_tests.log; exit 1; }
tail -3 gpurun_out/r05/pre2_tests.log
bash tools/ab_lib.sh shadow-gen_amd/libsgn_exp_head.so shadow-gen_amd/libsgn.so C 3 || exit 1
echo DONE
