#!/bin/bash
# Instruction-mix / wait PMC passes over the persistent round kernel of one bench invocation
# (k_rounds, the product path); one pass per counter group. $1 = tag, $2 = workload, $3 = steps.
set -u
T=${1:-x}; W=${2:-D}; ST=${3:-3}
mkdir -p gpurun_out/pmcm_$T
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex k_rounds -d gpurun_out/pmcm_$T/p$i -o run --output-format csv -- python -u bench.py --workload $W --steps $ST --warmup 1 --no-cpu-baseline > gpurun_out/pmcm_$T/p$i.log 2>&1
  rc=$?; echo "PASS $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python - gpurun_out/pmcm_$T <<'PY'
import csv, glob, sys
d = sys.argv[1]
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    v = {}
    n = set()
    for r in csv.DictReader(open(f)):
        v[r["Counter_Name"]] = v.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        n.add(r["Dispatch_Id"])
    for k in sorted(v):
        print(f"{k:24s} {v[k] / max(len(n), 1):14.4g} per dispatch ({len(n)} dispatches)")
PY
