#!/bin/bash
# The bench (no CPU leg) under environment variants: exp_env.sh <tag> <workload> [VAR=val ...]
set -u
T=$1; W=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
env "$@" timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline > gpurun_out/env_$T.json 2> gpurun_out/env_$T.err || { tail -5 gpurun_out/env_$T.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/env_$T.json'));r=d['roofline'] or {};print('$T', '$*', round(d['value']/1e6,1), 'M/s', r.get('kernel'), 'launch_us', r.get('avg_launch_us'), 'ms/step', round(d['ms_per_step'],3))"
