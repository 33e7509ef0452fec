#!/bin/bash
# Round-4 closing measurements after the PERIODIC slot / XCD changes: keyed PMC traffic of B and D
# (--steps 10 --warmup 5) and their bench lines (no CPU leg). $1 = tag.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc_traffic.sh ${T}_B B 10 5 > /dev/null || exit $?
bash tools/pmc_traffic.sh ${T}_D D 10 5 > /dev/null || exit $?
echo TRAFFIC_OK
