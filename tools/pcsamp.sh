#!/bin/bash
# PC sampling of the bench (stochastic, cycles) to see where k_execute's waves stall.
set -u
mkdir -p gpurun_out/pcs
export TMPDIR=/tmp SGN_PERSISTENT=0
timeout -s KILL 200 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 -d gpurun_out/pcs/st -o run --output-format csv -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pcs/st.log 2>&1
rc=$?; echo "STOCH rc=$rc"; tail -5 gpurun_out/pcs/st.log
if [ $rc -ne 0 ]; then
timeout -s KILL 200 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d gpurun_out/pcs/ht -o run --output-format csv -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pcs/ht.log 2>&1
rc=$?; echo "HOSTTRAP rc=$rc"; tail -5 gpurun_out/pcs/ht.log
fi
ls -la gpurun_out/pcs/*/ 2>/dev/null | head
