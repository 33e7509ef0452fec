#!/bin/bash
# APSP kernel times (rocprofv3 kernel stats) at Tor V = $1: the CSR loss sweep (default) and
# the per-arc sweep (SGN_APSP_SWEEP_ARCS=1); then PMC counters of the sweep kernels.
set -u
V=${1:-1000}
T=${2:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
for F in csr arcs; do
  if [ $F = arcs ]; then export SGN_APSP_SWEEP_ARCS=1; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_apsp_${F}_${V}_$T -o run --output-format csv -- python -u tools/apsp_bench.py tor $V > gpurun_out/prof_apsp_${F}_${V}_$T.log 2>&1
  rc=$?; echo "PROF $F rc=$rc"; grep '^{' gpurun_out/prof_apsp_${F}_${V}_$T.log | cut -c1-300
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('gpurun_out/prof_apsp_${F}_${V}_$T/**/*kernel_stats.csv', recursive=True)[0])):
    print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['MinNs'])/1e3,1), 'min')"
  [ $rc -eq 0 ] || exit $rc
done
unset SGN_APSP_SWEEP_ARCS
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_ANY"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_apsp_${N}_$T -o run --output-format csv -- python -u tools/apsp_bench.py tor $V > gpurun_out/pmc_apsp_${N}_$T.log 2>&1
  rc=$?; echo "PMC $N rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - <<PY
import csv,glob,collections
f=glob.glob('gpurun_out/pmc_apsp_${N}_$T/**/*counter_collection.csv', recursive=True)
acc=collections.defaultdict(lambda: collections.defaultdict(float)); calls=collections.Counter()
for r in csv.DictReader(open(f[0])):
    k=r['Kernel_Name'][:40]
    acc[k][r['Counter_Name']]+=float(r['Counter_Value'])
for k,v in acc.items():
    if 'loss' in k or 'sq_pass' in k: print('  ',k,{c:int(x) for c,x in v.items()})
PY
done
