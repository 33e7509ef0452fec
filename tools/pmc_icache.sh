#!/bin/bash
# Instruction-cache and issue PMC passes over the per-round k_execute (SGN_PERSISTENT=0).
set -u
T=${1:-x}
mkdir -p gpurun_out/pmci_$T
export TMPDIR=/tmp SGN_PERSISTENT=0
ARGS="--steps 2 --warmup 1 --no-cpu-baseline"
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_IFETCH SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex k_execute -d gpurun_out/pmci_$T/p$i -o run --output-format csv -- python -u bench.py $ARGS > gpurun_out/pmci_$T/p$i.log 2>&1
  rc=$?; echo "PASS $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
