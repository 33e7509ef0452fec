#!/bin/bash
# Same-box A/B of the tiled (SoA) hot host line (SGN_SOA build) against the default on B, C, D,
# after the parity suites with the SoA build.
set -u
export TMPDIR=/tmp
SGN_LIB=$PWD/shadow-gen_amd/libsgn_exp_soa.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py > gpurun_out/soa_tests.log 2>&1
rc=$?; tail -2 gpurun_out/soa_tests.log; [ $rc -eq 0 ] || exit $rc
for W in C B D; do
  bash tools/ab_lib.sh shadow-gen_amd/libsgn.so shadow-gen_amd/libsgn_exp_soa.so $W 2 || exit 1
done
