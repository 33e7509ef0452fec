#!/bin/bash
# Persistent multi-shard rehearsal after the one-round-trip edge (C and D per shard count) and the
# 8-shard per-workgroup timeline.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u tools/xpersist_bench.py --hosts 100000,12500,25000,50000 --shards 1,2,4,8 > gpurun_out/r05/xb2_C.jsonl 2>&1 || exit $?
timeout -k 10 400 python -u tools/xpersist_bench.py --workload D --hosts 1000000 --shards 1,2,4,8 --rounds 200 --warmup 50 > gpurun_out/r05/xb2_D.jsonl 2>&1 || exit $?
timeout -k 10 200 python -u tools/diag_xw.py 12500 8 > gpurun_out/r05/dw2.txt 2>&1 || exit $?
echo DONE
