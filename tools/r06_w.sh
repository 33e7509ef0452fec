#!/bin/bash
# Round 6: occupancy of the sparse APSP latency pass (bf_pass, random V = 1000): wave cycles
# against the kernel's cycles.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex bf_pass -d $O/p1 -o run --output-format csv -- python3 tools/apsp_bench.py random 1000 > $O/p1.log 2>&1 || exit $?
python3 - <<'PY'
import csv
r=list(csv.DictReader(open('gpurun_out/r06w/p1/run_counter_collection.csv')))
by={}
for x in r: by.setdefault(x['Dispatch_Id'],{})[x['Counter_Name']]=by.setdefault(x['Dispatch_Id'],{}).get(x['Counter_Name'],0)+float(x['Counter_Value'])
for d,v in sorted(by.items()): print(d, {k: round(vv) for k,vv in v.items()})
PY
echo DONE
