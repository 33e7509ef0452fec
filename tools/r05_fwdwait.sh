#!/bin/bash
# PERIODIC forwarding lanes wait for the wave's other lanes (experiment build): parity of the
# round kernels with it, then same-box A/B on B and D.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
SGN_LIB=$PWD/shadow-gen_amd/libsgn_exp_fwdwait.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py > gpurun_out/r05/fwdwait_tests.log 2>&1 || { tail -30 gpurun_out/r05/fwdwait_tests.log; exit 1; }
tail -2 gpurun_out/r05/fwdwait_tests.log
for W in B D; do bash tools/ab_lib.sh shadow-gen_amd/libsgn.so shadow-gen_amd/libsgn_exp_fwdwait.so $W 3 || exit 1; done
echo DONE
