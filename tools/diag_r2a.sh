set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
SGN_LIB=$PWD/shadow-gen_amd/libsgn_diag.so SGN_PERSISTENT=0 timeout -k 10 200 python -u tools/diag_execute.py > gpurun_out/diag_exec_r2a.log 2>&1
echo "DIAG rc=$?"
timeout -k 10 200 python -u tools/diag_rounds.py > gpurun_out/diag_rounds_r2a.log 2>&1
echo "ROUNDS rc=$?"
