#!/bin/bash
# Round 6: the multi-shard post-message section with its launch constants in LDS — per-workgroup
# timeline (12.5 k and 100 k hosts as 8 shards on one GPU), the rehearsal's per-round times, and
# the multi-shard parity suites.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_xpersist.py tests/test_gpu_rccl.py -x -q -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/xk_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -n 2 gpurun_out/r06/xk_tests.log; [ $rc -eq 0 ] || exit $rc
for n in 12500 100000; do
  timeout -k 10 200 python -u tools/diag_xw.py $n 8 300 C 2>&1 | tail -1 || exit 1
done
timeout -k 10 400 python -u tools/xpersist_bench.py --hosts 12500,100000 --shards 1,8 > gpurun_out/r06/xpersist_xk.jsonl 2>gpurun_out/r06/xpersist_xk.err || exit 1
tail -n 20 gpurun_out/r06/xpersist_xk.jsonl
echo DONE
