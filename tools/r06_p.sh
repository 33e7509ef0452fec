#!/bin/bash
# Round 6: where the dense loss sweep's time goes — kernel stats of the APSP build (Tor V = 2000),
# then PMC passes of instruction and wait counters over the sweep kernel.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks -o run --output-format csv -- python3 tools/apsp_bench.py tor 2000 > $O/ks.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-include-regex loss_sweep_dense -d $O/pmc1 -o run --output-format csv -- python3 tools/apsp_bench.py tor 2000 > $O/pmc1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex loss_sweep_dense -d $O/pmc2 -o run --output-format csv -- python3 tools/apsp_bench.py tor 2000 > $O/pmc2.log 2>&1 || exit $?
echo DONE
