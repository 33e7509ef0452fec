#!/bin/bash
# Round 6: kernel stats of the sparse APSP build (random graph V = 1000, configs B / D).
set -u
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks -o run --output-format csv -- python3 tools/apsp_bench.py random 1000 > $O/ks.log 2>&1 || exit $?
echo DONE
