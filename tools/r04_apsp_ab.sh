#!/bin/bash
# APSP: the route tests, then kernel stats of the Tor V = $1 build with the sweep at 16 and 8
# sources per workgroup (SGN_APSP_SWEEP_S); $2 = tag.
set -u
V=${1:-1000}
T=${2:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k apsp -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/apsp_tests_$T.log 2>&1
rc=$?; echo "TESTS $rc"; tail -3 gpurun_out/apsp_tests_$T.log; [ $rc -eq 0 ] || exit $rc
for S in 16 8; do
  export SGN_APSP_SWEEP_S=$S
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_apsp_s${S}_${V}_$T -o run --output-format csv -- python -u tools/apsp_bench.py tor $V > gpurun_out/prof_apsp_s${S}_${V}_$T.log 2>&1
  rc=$?; echo "PROF S=$S rc=$rc"; grep '^{' gpurun_out/prof_apsp_s${S}_${V}_$T.log | cut -c1-260
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('gpurun_out/prof_apsp_s${S}_${V}_$T/**/*kernel_stats.csv', recursive=True)[0])):
    print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['MinNs'])/1e3,1), 'min')"
  [ $rc -eq 0 ] || exit $rc
done
unset SGN_APSP_SWEEP_S
for S in 16 8; do
  timeout -k 10 120 env SGN_APSP_SWEEP_S=$S python -u tools/apsp_bench.py tor $V > gpurun_out/apsp_plain_s${S}_$T.log 2>&1
  rc=$?; echo "PLAIN S=$S rc=$rc"; grep '^{' gpurun_out/apsp_plain_s${S}_$T.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
