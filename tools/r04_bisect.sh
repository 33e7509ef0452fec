#!/bin/bash
# Same-box comparison of the bench across staged builds (exp_<rev>/: that revision's bench.py,
# sgn.py and libsgn.so; untracked) and HEAD. $1 = tag, $2 = workload, $3 = steps, then dirs.
set -u
T=$1; W=$2; S=$3; shift 3
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for d in head "$@"; do
    b=bench.py; [ $d = head ] || b=$d/bench.py
    timeout -k 10 200 python -u $b --workload $W --no-cpu-baseline --steps $S --warmup 5 > gpurun_out/bis_${T}_${rep}_${d}_$W.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/bis_${T}_${rep}_${d}_$W.json'));print('$d $W', round(d['value']/1e6,1), 'M/s launch_us', d['roofline']['avg_launch_us'])"
  done
done
