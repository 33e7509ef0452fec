#!/bin/bash
# Per-round timeline (persistent kernel) for configs B and C, then per-wave phases of
# config B (diag build, one round per launch). Tag = $1.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/diag_rounds.py B > gpurun_out/diag_rounds_B_$T.log 2>&1
echo "ROUNDS_B rc=$?"; cat gpurun_out/diag_rounds_B_$T.log | tail -3
timeout -k 10 200 python -u tools/diag_rounds.py > gpurun_out/diag_rounds_C_$T.log 2>&1
echo "ROUNDS_C rc=$?"; cat gpurun_out/diag_rounds_C_$T.log | tail -3
SGN_LIB=$PWD/shadow-gen_amd/libsgn_diag.so SGN_PERSISTENT=0 timeout -k 10 200 python -u tools/diag_execute.py B > gpurun_out/diag_exec_B_$T.log 2>&1
echo "EXEC_B rc=$?"; head -40 gpurun_out/diag_exec_B_$T.log
