#!/bin/bash
# Same-box A/B of one build under two environments, interleaved (bench.py, no CPU leg).
# usage: bash tools/ab_env.sh <workload> <reps> "<VAR=val ...|->" "<VAR=val ...>" [extra bench args]
set -u
W=$1; N=$2; A=$3; B=$4; shift 4; X="$*"
for i in $(seq $N); do
  for E in "$A" "$B"; do
    EV=""; [ "$E" != "-" ] && EV="$E"
    env $EV timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline --workload $W $X > gpurun_out/abe_$$.json 2>/dev/null || { echo "FAIL $E"; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/abe_$$.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$W', '$E', round(d['value']/1e9,4), 'G  ms/step', round(d['ms_per_step'],4), ' launch us', r['avg_launch_us'])"
  done
done
