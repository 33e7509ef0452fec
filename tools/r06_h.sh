#!/bin/bash
# Round 6: TGEN train-wait threshold (SGN_TRAIN_WAIT 4 / 8 / 16 / 32) on C; hosts per wave for
# the per-GPU round of the strong-scaled N > 1 runs (12.5k / 25k / 50k hosts on one shard).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for i in 1 2; do
  for L in libsgn libsgn_exp_tw4 libsgn_exp_tw16 libsgn_exp_tw32; do
    SGN_LIB=$PWD/shadow-gen_amd/$L.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline --workload C > gpurun_out/r06/tw.json 2>/dev/null || { echo "FAIL $L"; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r06/tw.json').read().strip().splitlines()[-1]); r=d['roofline']
print('C', '$L', round(d['value']/1e9,4), 'G launch us', r['avg_launch_us'])"
  done
done
for H in 64 32 16; do
  SGN_HOSTS_PER_WAVE=$H timeout -k 10 300 python -u tools/xpersist_bench.py --hosts 12500,25000,50000 --shards 1 --rounds 300 --warmup 100 > gpurun_out/r06/hpw_$H.jsonl 2>&1 || exit 1
  echo "HPW $H"; cat gpurun_out/r06/hpw_$H.jsonl
done
echo DONE
