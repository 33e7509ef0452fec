#!/bin/bash
# Round 6: compiler scheduling of engine.hip (device code only) priced on config C: the default,
# -misched=gcn-max-ilp, gcn-max-memory-clause, -O2, schedule-metric-bias=0, no unclustered
# high-register-pressure reschedule; same box, two interleaved passes.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for i in 1 2; do
  for L in libsgn libsgn_exp_ilp libsgn_exp_memc libsgn_exp_o2 libsgn_exp_bias0 libsgn_exp_nounc; do
    SGN_LIB=$PWD/shadow-gen_amd/$L.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline --workload C > gpurun_out/r06/cc.json 2>/dev/null || { echo "FAIL $L"; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r06/cc.json').read().strip().splitlines()[-1]); r=d['roofline']
print('C', '$L', round(d['value']/1e9,4), 'G launch us', r['avg_launch_us'])"
  done
done
echo DONE
