#!/bin/bash
# Instruction-mix PMC passes over the per-round k_execute (SGN_PERSISTENT=0: one launch per
# round, no persistent-kernel spinning in the counters). One pass per counter group.
set -u
T=${1:-x}
mkdir -p gpurun_out/pmcx_$T
export TMPDIR=/tmp SGN_PERSISTENT=0
ARGS="--steps 2 --warmup 1 --no-cpu-baseline"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_FLAT SQ_INST_LEVEL_SMEM SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_MISC SQ_IFETCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex k_execute -d gpurun_out/pmcx_$T/p$i -o run --output-format csv -- python -u bench.py $ARGS > gpurun_out/pmcx_$T/p$i.log 2>&1
  rc=$?; echo "PASS $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
