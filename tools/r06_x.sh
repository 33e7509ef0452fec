#!/bin/bash
# Round 6 (experiment library with two extra stamps, not parity-relevant): where the multi-shard
# round's post-message phase goes; 12.5 k and 100 k hosts as 8 shards on one GPU.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for n in 12500 100000; do
  SGN_LIB=$PWD/shadow-gen_amd/libsgn_exp_xpost.so timeout -k 10 200 python -u tools/diag_xw_post.py $n 8 300 C 2>&1 | tail -1 || exit 1
  SGN_LIB=$PWD/shadow-gen_amd/libsgn_exp_xpost.so timeout -k 10 200 python -u tools/diag_xw.py $n 8 300 C 2>&1 | tail -1 || exit 1
done
echo DONE
