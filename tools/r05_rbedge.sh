#!/bin/bash
# rb_edge in one round trip: parity of the round kernels, then same-box A/B against HEAD's build.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_xpersist.py > gpurun_out/r05/rbedge_tests.log 2>&1 || { tail -30 gpurun_out/r05/rbedge_tests.log; exit 1; }
tail -3 gpurun_out/r05/rbedge_tests.log
for W in C B D; do
  bash tools/ab_lib.sh shadow-gen_amd/libsgn_exp_head.so shadow-gen_amd/libsgn.so $W 3 || exit 1
done
timeout -k 10 300 python -u tools/xpersist_bench.py --hosts 12500 --shards 1,8 > gpurun_out/r05/rbedge_xb.jsonl 2>&1 || exit 1
cat gpurun_out/r05/rbedge_xb.jsonl | tail -4
echo DONE
