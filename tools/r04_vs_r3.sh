#!/bin/bash
# Same-box A/B of the bench against round 3's final build (exp_r3/: its bench.py, sgn.py and
# libsgn.so, staged from a worktree; not tracked). $1 = tag, $2 = workload, $3 = steps.
set -u
T=${1:-x}; W=${2:-C}; S=${3:-20}
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --steps $S --warmup 5 > gpurun_out/vs_${T}_${rep}_head_$W.json 2>/dev/null || exit 1
  timeout -k 10 200 python -u exp_r3/bench.py --workload $W --no-cpu-baseline --steps $S --warmup 5 > gpurun_out/vs_${T}_${rep}_r3_$W.json 2>/dev/null || exit 1
  for v in head r3; do
    python3 -c "import json;d=json.load(open('gpurun_out/vs_${T}_${rep}_${v}_$W.json'));print('$v $W', round(d['value']/1e6,1), 'M/s launch_us', d['roofline']['avg_launch_us'])"
  done
done
