#!/bin/bash
# Round-5 re-measurements after the train and tile changes: persistent multi-shard rehearsal
# (C and D per shard count) and the keyed PMC traffic of D and B.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u tools/xpersist_bench.py --hosts 100000,12500 --shards 1,2,8 > gpurun_out/r05/xb_C.jsonl 2>&1 || exit $?
timeout -k 10 400 python -u tools/xpersist_bench.py --workload D --hosts 1000000 --shards 1,2,4,8 --rounds 200 --warmup 50 > gpurun_out/r05/xb_D.jsonl 2>&1 || exit $?
timeout -k 10 200 python -u tools/diag_xw.py 12500 8 > gpurun_out/r05/dw.txt 2>&1 || exit $?
for W in D B; do
  bash tools/pmc_traffic.sh r05s_$W $W 10 5 > gpurun_out/r05/traffic2_$W.log 2>&1 || exit 1
  cp gpurun_out/traffic_r05s_$W/summary.json gpurun_out/r05/traffic2_$W.json
done
echo DONE
