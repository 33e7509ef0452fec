#!/bin/bash
# Round 6: config C census with long-train combining counters (diag build), and the persistent
# kernel's per-group timeline (SGN_STAMPS=1, product build).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
SGN_LIB=$PWD/shadow-gen_amd/libsgn_diag.so SGN_PERSISTENT=0 timeout -k 10 200 python -u tools/diag_execute.py > gpurun_out/r06/diag_exec_C2.log 2>&1
echo "EXEC_C rc=$?"
timeout -k 10 200 python -u tools/diag_persist.py > gpurun_out/r06/diag_persist_C.log 2>&1
echo "PERSIST rc=$?"
echo DONE
