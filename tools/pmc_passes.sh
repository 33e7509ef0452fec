#!/bin/bash
# PMC passes over a short bench run (one pass per counter group, each under its own limit).
set -u
T=${1:-x}
mkdir -p gpurun_out/pmc_$T
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_IFETCH" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex k_execute -d gpurun_out/pmc_$T/p$i -o run --output-format csv -- python -u bench.py $ARGS > gpurun_out/pmc_$T/p$i.log 2>&1
  rc=$?; echo "PASS $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
