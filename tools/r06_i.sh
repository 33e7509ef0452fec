#!/bin/bash
# Round 6: config C census with CoDel-page, token-bucket and delivery timers (diag build).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
SGN_LIB=$PWD/shadow-gen_amd/libsgn_diag.so SGN_PERSISTENT=0 timeout -k 10 200 python -u tools/diag_execute.py > gpurun_out/r06/diag_exec_C3.log 2>&1
echo "EXEC_C rc=$?"
echo DONE
