#!/bin/bash
# Round 6: same-box A/B of the multi-shard round with the post-message constants in LDS
# (libsgn_exp_xk.so) against the build before it (libsgn_exp_base.so): config C, 8 shards on one
# GPU at 12.5 k and 100 k hosts, two interleaved passes.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for i in 1 2; do
  for L in base xk; do
    SGN_LIB=$PWD/shadow-gen_amd/libsgn_exp_$L.so timeout -k 10 300 python -u tools/xpersist_bench.py --hosts 12500,100000 --shards 8 > gpurun_out/r06/xk_ab.jsonl 2>/dev/null || { echo "FAIL $L"; exit 1; }
    python -c "
import json
for l in open('gpurun_out/r06/xk_ab.jsonl'):
    d=json.loads(l); print('$L', d['hosts'], d['shards'], d['kernel_us_per_round'])"
  done
done
echo DONE
