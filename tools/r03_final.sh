#!/bin/bash
# Round-3 closing measurements at head: the driver's bench invocation (with the CPU leg),
# benches of B and D, rocprofv3 kernel stats of the driver's invocation, keyed PMC traffic of
# C (--steps 20 --warmup 5), B and D (--steps 10 --warmup 5). $1 = tag.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_$T.json 2> gpurun_out/final_$T.err
rc=$?; echo "BENCH $rc"; tail -c 600 gpurun_out/final_$T.json; echo; [ $rc -eq 0 ] || exit $rc
bash tools/r03_bench.sh $T "B D" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "PROF $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_traffic.sh ${T}_C C 20 5 || exit $?
bash tools/pmc_traffic.sh ${T}_B B 10 5 || exit $?
bash tools/pmc_traffic.sh ${T}_D D 10 5 || exit $?
