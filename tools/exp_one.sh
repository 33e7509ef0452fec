#!/bin/bash
# One cost experiment (NOT parity-valid): the bench without its CPU leg on a libsgn variant
# built by shadow-gen_amd/csrc/build_exp.sh. Usage: exp_one.sh <variant> <workload> <tag>
set -u
v=$1; w=${2:-C}; T=${3:-x}; shift 3 || true
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ $v = base ]; then L=$PWD/shadow-gen_amd/libsgn.so; else L=$PWD/shadow-gen_amd/libsgn_exp_$v.so; fi
SGN_LIB=$L timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline "$@" > gpurun_out/exp_${T}_${v}_$w.json 2>&1 || exit 1
python -c "import json;d=json.load(open('gpurun_out/exp_${T}_${v}_$w.json'));print('$v $w', round(d['value']/1e6,1), 'M/s launch_us', d['roofline']['avg_launch_us'])"
