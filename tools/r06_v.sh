#!/bin/bash
# Round 6 (experiment): where bf_front's time goes — the sweep loop capped at 1 / 3 / 6 sweeps
# (results wrong, timing only), kernel stats on the random V = 1000 graph.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
for c in 1 3 6 100; do
  SGN_EXP_BF_CAP=$c timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/c$c -o run --output-format csv -- python3 tools/apsp_bench.py random 1000 > $O/c$c.log 2>&1
  python3 -c "
import csv
for x in csv.DictReader(open('$O/c$c/run_kernel_stats.csv')):
    if 'bf_' in x['Name']: print('cap', $c, x['Name'][:20], x['Calls'], round(float(x['AverageNs'])/1000,1), 'us')"
done
echo DONE
