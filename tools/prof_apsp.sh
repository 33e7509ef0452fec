#!/bin/bash
# Kernel times of the APSP build (Tor graph, V = $1) under rocprofv3, dense and sweep forms.
set -u
V=${1:-2000}
mkdir -p gpurun_out
export TMPDIR=/tmp
for F in dense sweep; do
  if [ $F = sweep ]; then export SGN_APSP_SWEEP=1; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_apsp_${F}_$V -o run --output-format csv -- python -u tools/apsp_bench.py tor $V > gpurun_out/prof_apsp_${F}_$V.log 2>&1
  rc=$?; echo "PROF $F rc=$rc"; grep '^{' gpurun_out/prof_apsp_${F}_$V.log | cut -c1-200
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('gpurun_out/prof_apsp_${F}_$V/**/*kernel_stats.csv', recursive=True)[0])):
    print('  ', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['MinNs'])/1e3,1), 'min')"
  [ $rc -eq 0 ] || exit $rc
done
