#!/bin/bash
# Round-3 profiles: counter calibration, rocprofv3 kernel stats of the driver's bench
# invocation, keyed PMC traffic of C (driver's --steps 20 --warmup 5), B and D. $1 = tag.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc_calib.sh $T || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "PROF $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_traffic.sh ${T}_C C 20 5 || exit $?
bash tools/pmc_traffic.sh ${T}_B B 10 5 || exit $?
bash tools/pmc_traffic.sh ${T}_D D 10 5 || exit $?
