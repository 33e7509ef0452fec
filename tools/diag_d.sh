#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
SGN_LIB=$PWD/shadow-gen_amd/libsgn_diag.so SGN_PERSISTENT=0 timeout -k 10 300 python -u tools/diag_execute.py D > gpurun_out/diag_exec_D.log 2>&1
echo "DIAG rc=$?"
