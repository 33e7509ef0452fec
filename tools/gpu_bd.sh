#!/bin/bash
# Configs B and D through bench.py with the CPU baselines. Tag = $1.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --workload B > gpurun_out/benchB_$T.json 2> gpurun_out/benchB_$T.err
rc=$?; echo "BENCH_B $rc"; cat gpurun_out/benchB_$T.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload D --steps 5 --warmup 2 --cpu-budget-s 8 > gpurun_out/benchD_$T.json 2> gpurun_out/benchD_$T.err
rc=$?; echo "BENCH_D $rc"; cat gpurun_out/benchD_$T.json | cut -c1-400; tail -3 gpurun_out/benchD_$T.err; exit $rc
