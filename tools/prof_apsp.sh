#!/bin/bash
# Kernel times of the APSP build (Tor graph, V = $1) under rocprofv3.
set -u
V=${1:-2000}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_apsp_$V -o run --output-format csv -- python -u tools/apsp_bench.py tor $V > gpurun_out/prof_apsp_$V.log 2>&1
rc=$?; echo "PROF rc=$rc"; cat gpurun_out/prof_apsp_$V.log; find gpurun_out/prof_apsp_$V -name "*kernel_stats.csv" -exec cut -c1-160 {} \;
exit $rc
