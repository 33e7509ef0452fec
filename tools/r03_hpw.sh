#!/bin/bash
# Hosts per wave on small config-C shards (the strong-scaled N > 1 runs: 100k / N hosts per GPU),
# per-round k_execute (the N > 1 path's kernel) and persistent. $1 = tag.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
for H in 12500 25000; do
  for P in 0 1; do
    for HPW in 64 32 16; do
      SGN_PERSISTENT=$P SGN_HOSTS_PER_WAVE=$HPW timeout -k 10 200 python -u bench.py --hosts $H --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/hpw_${T}_${H}_${P}_${HPW}.json 2> gpurun_out/hpw_${T}.err || { tail -3 gpurun_out/hpw_${T}.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/hpw_${T}_${H}_${P}_${HPW}.json'));r=d['roofline'];print('hosts $H persistent $P hpw $HPW', round(d['value']/1e6,1), 'M/s', r['kernel'], 'round_us', r['latency_bound']['round_us'], 'ms/step', round(d['ms_per_step'],3))"
    done
  done
done
