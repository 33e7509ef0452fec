#!/bin/bash
# Cost experiments: the bench (no CPU leg) with each libsgn variant, configs C and D. Tag = $1.
set -u
T=${1:-x}
export TMPDIR=/tmp
for v in base nodig norng both; do
  if [ $v = base ]; then L=$PWD/shadow-gen_amd/libsgn.so; else L=$PWD/shadow-gen_amd/libsgn_exp_$v.so; fi
  for w in C D; do
    if [ $w = C ]; then A="--steps 10 --warmup 5"; else A="--workload D --steps 2 --warmup 1"; fi
    SGN_LIB=$L timeout -k 10 200 python -u bench.py $A --no-cpu-baseline > gpurun_out/exp_${T}_${v}_$w.json 2>&1 || exit 1
    python -c "import json;d=json.load(open('gpurun_out/exp_${T}_${v}_$w.json'));print('$v $w', round(d['value']/1e6,1), 'M/s launch_us', d['roofline']['avg_launch_us'])"
  done
done
