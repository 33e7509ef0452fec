#!/bin/bash
# Experiment: hosts per wave (SGN_HOSTS_PER_WAVE) for configs B and C, no CPU leg.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in B C; do
  for H in 64 32 16; do
    SGN_HOSTS_PER_WAVE=$H timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --steps 5 --warmup 3 > gpurun_out/hpw_${W}_$H.json 2> gpurun_out/hpw_${W}_$H.err
    rc=$?; echo "$W hpw=$H rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/hpw_${W}_$H.json'));print(round(d['value']/1e6,1), d['roofline']['latency_bound']['round_us'], d['engine'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
