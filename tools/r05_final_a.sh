#!/bin/bash
# Round-5 closing measurements, part 1: the full -m gpu suite, the driver's bench line (default
# arguments, CPU leg included) and its rocprofv3 kernel-trace summary (same command).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r05/gpu_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -3 gpurun_out/r05/gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python -u bench.py > gpurun_out/r05/bench_C.json 2> gpurun_out/r05/bench_C.err || exit $?
tail -c 600 gpurun_out/r05/bench_C.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof_C -o run --output-format csv -- python -u bench.py > gpurun_out/r05/bench_C_prof.json 2> gpurun_out/r05/bench_C_prof.err || exit $?
echo PROF_OK
