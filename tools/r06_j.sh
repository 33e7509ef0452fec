#!/bin/bash
# Round 6: TGEN hosts keep one drained CoDel page (no ring atomics on their chain for it): the
# whole -m gpu suite, then a same-box A/B against the previous build (libsgn_exp_base.so) on C.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06/gpu_tests_j.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -n 3 gpurun_out/r06/gpu_tests_j.log
case $rc in 0) ;; *) exit $rc;; esac
bash tools/ab_lib.sh shadow-gen_amd/libsgn.so shadow-gen_amd/libsgn_exp_base.so C 3 || exit 1
echo DONE
