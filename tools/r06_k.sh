#!/bin/bash
# Round 6: the persistent multi-shard rehearsal re-measured with round 6's message words (C at
# 12.5k-100k hosts x 1/2/4/8 shards, D at 1M x 1/2/4/8), then the 400-case randomised sweep.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u tools/xpersist_bench.py --hosts 100000,12500,25000,50000 --shards 1,2,4,8 > gpurun_out/r06/xb_C.jsonl 2>&1 || exit $?
timeout -k 10 400 python -u tools/xpersist_bench.py --workload D --hosts 1000000 --shards 1,2,4,8 --rounds 200 --warmup 50 > gpurun_out/r06/xb_D.jsonl 2>&1 || exit $?
echo "XB done"
bash tools/r03_fuzz.sh r06 400
