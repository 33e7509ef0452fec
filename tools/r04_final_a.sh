#!/bin/bash
# Round-4 closing measurements, part 1: keyed PMC traffic of C (--steps 20 --warmup 5), B and D
# (--steps 10 --warmup 5), C's instruction-mix / wait counters, the 400-case parity sweep. $1 = tag.
set -u
T=${1:-x}
bash tools/pmc_traffic.sh ${T}_C C 20 5 > /dev/null || exit $?
bash tools/pmc_traffic.sh ${T}_B B 10 5 > /dev/null || exit $?
bash tools/pmc_traffic.sh ${T}_D D 10 5 > /dev/null || exit $?
echo TRAFFIC_OK
bash tools/r03_pmc_mix.sh ${T}_C C 3 > gpurun_out/pmcmix_${T}_C.txt 2>&1 || exit $?
grep -E "SQ_WAIT_ANY|SQ_WAVE_CYCLES|SQ_ACTIVE_INST_ANY" gpurun_out/pmcmix_${T}_C.txt
bash tools/r03_fuzz.sh ${T} 400
