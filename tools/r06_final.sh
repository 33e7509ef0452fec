#!/bin/bash
# Round 6 closing measurements on the final build (everything keyed to the
# driver's exact command and to this libsgn build):
#  1. the whole -m gpu suite;
#  2. rocprofv3 --kernel-trace --stats over the driver's command (25 k_rounds launches);
#  3. PMC HBM traffic of k_rounds for the driver's arguments (C, --steps 20 --warmup 5) and for
#     B and D (--steps 10 --warmup 5), one pass per counter, entries carrying the build id;
#  4. the B and D bench lines with their parity legs, then the driver's C line, which now quotes
#     the traffic measured in 3 on this build.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -n 2 $O/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/rocprof_C -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  > $O/rocprof_C_bench.json 2> $O/rocprof_C_bench.err || exit $?
echo "ROCPROF done"
bash tools/pmc_traffic.sh r06C C 20 5 > $O/traffic_C.log 2>&1 || exit $?
cp gpurun_out/traffic_r06C/summary.json $O/traffic_C.json
bash tools/pmc_traffic.sh r06B B 10 5 > $O/traffic_B.log 2>&1 || exit $?
cp gpurun_out/traffic_r06B/summary.json $O/traffic_B.json
bash tools/pmc_traffic.sh r06D D 10 5 > $O/traffic_D.log 2>&1 || exit $?
cp gpurun_out/traffic_r06D/summary.json $O/traffic_D.json
python tools/traffic_merge.py $O/traffic_C.json $O/traffic_B.json $O/traffic_D.json
echo DONE
