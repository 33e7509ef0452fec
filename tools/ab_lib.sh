#!/bin/bash
# Same-box A/B of two builds on one workload: bench.py with SGN_LIB=A and =B, interleaved.
# usage: bash tools/ab_lib.sh <libA> <libB> <workload> [reps] [extra bench args]
set -u
A=$1; B=$2; W=$3; N=${4:-2}; shift 4 2>/dev/null; X="$*"
for i in $(seq $N); do
  for L in $A $B; do
    SGN_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline --workload $W $X > gpurun_out/ab_$$.json 2>/dev/null || { echo "FAIL $L"; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab_$$.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$W', '$L', round(d['value']/1e9,4), 'G  ms/step', round(d['ms_per_step'],4), ' launch us', r['avg_launch_us'])"
  done
done
