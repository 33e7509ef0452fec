#!/bin/bash
# Per-wave phases of configs C and B (diag build, one round per launch). Tag = $1.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
SGN_LIB=$PWD/shadow-gen_amd/libsgn_diag.so SGN_PERSISTENT=0 timeout -k 10 200 python -u tools/diag_execute.py > gpurun_out/diag_exec_C_$T.log 2>&1
echo "EXEC_C rc=$?"; head -12 gpurun_out/diag_exec_C_$T.log
SGN_LIB=$PWD/shadow-gen_amd/libsgn_diag.so SGN_PERSISTENT=0 timeout -k 10 200 python -u tools/diag_execute.py B > gpurun_out/diag_exec_B_$T.log 2>&1
echo "EXEC_B rc=$?"; head -4 gpurun_out/diag_exec_B_$T.log
