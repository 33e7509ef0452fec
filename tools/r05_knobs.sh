#!/bin/bash
# Re-check of the per-config knobs after round 5's changes (no CPU leg, two interleaved passes):
# hosts per wave for B (default 16), D (64) and C (64), the TGEN train-wait default (8).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
run() {  # workload, env assignment
  env $2 timeout -k 10 200 python -u bench.py --workload $1 --no-cpu-baseline --steps 10 --warmup 5 > gpurun_out/r05/knob.json 2>/dev/null || { echo "FAIL $1 $2"; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r05/knob.json').read().strip().splitlines()[-1])
print('$1', '$2', round(d['value']/1e6,2), 'M', d['roofline']['avg_launch_us'], 'us per launch')"
}
for i in 1 2; do
  for H in 16 8 32; do run B SGN_HOSTS_PER_WAVE=$H; done
  for H in 64 32; do run D SGN_HOSTS_PER_WAVE=$H; done
  for H in 64 32; do run C SGN_HOSTS_PER_WAVE=$H; done
done
echo DONE
