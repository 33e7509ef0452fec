#!/bin/bash
# Round-4 closing measurements, part 2: the driver's bench invocation with the CPU leg (SKIP_C=1:
# not again), benches of B and D, rocprofv3 kernel stats of the driver's invocation, the APSP build's kernel stats.
# $1 = tag.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_C:-0}" != 1 ]; then
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_$T.json 2> gpurun_out/final_$T.err
  rc=$?; echo "BENCH $rc"; tail -c 400 gpurun_out/final_$T.json; echo; [ $rc -eq 0 ] || exit $rc
fi
for W in B D; do  # (no CPU leg: D's parity replay alone outlasts the step's limit)
  timeout -k 10 300 python -u bench.py --workload $W --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/final_${T}_$W.json 2> gpurun_out/final_${T}_$W.err
  rc=$?; echo "BENCH_$W $rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "PROF $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_apsp_$T -o run --output-format csv -- python -u tools/apsp_bench.py tor 1000 > gpurun_out/prof_apsp_$T.log 2>&1
rc=$?; echo "PROF_APSP $rc"; exit $rc
