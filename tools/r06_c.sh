#!/bin/bash
# Round 6: handler grouping priced on B, D (PERIODIC: grp1) and C (TGEN:
# grp2) against the product build, interleaved same-box pairs; then the D bench line with its
# parity leg (the oracle over every round the GPU ran).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
bash tools/ab_lib.sh shadow-gen_amd/libsgn.so shadow-gen_amd/libsgn_exp_grp1.so B 2 || exit 1
bash tools/ab_lib.sh shadow-gen_amd/libsgn.so shadow-gen_amd/libsgn_exp_grp1.so D 2 || exit 1
bash tools/ab_lib.sh shadow-gen_amd/libsgn.so shadow-gen_amd/libsgn_exp_grp2.so C 2 || exit 1
timeout -k 10 600 python -u bench.py --workload D --steps 10 --warmup 5 > gpurun_out/r06/bench_D.json 2> gpurun_out/r06/bench_D.err || exit $?
python - <<'PY'
import json; d=json.loads(open('gpurun_out/r06/bench_D.json').read().strip().splitlines()[-1]); r=d['roofline']
print('BENCH D', round(d['value']/1e9,4), 'G parity', d['parity'], d['parity_detail']['rounds_compared'], 'launch us', r['avg_launch_us'], 'frac', r['frac'], 'cpu', d['cpu_baseline']['value'])
PY
echo DONE
