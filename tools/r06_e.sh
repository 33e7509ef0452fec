#!/bin/bash
# Round 6: the next round's first gather in the edge's round trip (TGEN k_rounds): the whole
# -m gpu suite on the product build, then a same-box A/B against SGN_PREGATHER=0 on C.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06/gpu_tests_e.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -n 3 gpurun_out/r06/gpu_tests_e.log
case $rc in 0) ;; *) exit $rc;; esac
bash tools/ab_lib.sh shadow-gen_amd/libsgn.so shadow-gen_amd/libsgn_exp_nopre.so C 3 || exit 1
echo DONE
