#!/bin/bash
# Wave diagnostics of the round kernel (diag build): per-wave phases and in-loop load sites.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
SGN_LIB=$PWD/shadow-gen_amd/libsgn_diag.so SGN_PERSISTENT=0 timeout -k 10 200 python -u tools/diag_execute.py > gpurun_out/diag_exec_$T.log 2>&1
echo "DIAG rc=$?"
