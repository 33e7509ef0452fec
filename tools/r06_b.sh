#!/bin/bash
# Round 6, second GPU call: (1) the system-scope message fences priced one at a time on the
# two-process one-GPU rehearsal (both / release only / acquire only / none); (2) config C's
# section census from the diag build (where the slowest waves' cycles go);
# (3) SQ_WAIT_ANY / SQ_WAVE_CYCLES and the instruction mix of k_rounds at config C.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for rep in 1 2; do
for L in libsgn libsgn_exp_xnoacq libsgn_exp_xnorel libsgn_exp_xnofence; do
  SGN_LIB=$PWD/shadow-gen_amd/$L.so SGN_XPEER_SHARED=1 SGN_GRAPH=0 NCCL_DEBUG=WARN timeout -k 10 300 python -u bench.py --gpus 2 --one-gpu \
    --steps 5 --warmup 2 --no-shard-check > gpurun_out/r06/xfence.json 2> gpurun_out/r06/xfence.err || { echo "FAIL $L"; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r06/xfence.json').read().strip().splitlines()[-1]); r=d['roofline']
print('XPEER C 2 procs', '$L', r['kernel'], 'round us', r['latency_bound']['round_us'], 'launch us', r['avg_launch_us'])"
done
done
SGN_LIB=$PWD/shadow-gen_amd/libsgn_diag.so SGN_PERSISTENT=0 timeout -k 10 200 python -u tools/diag_execute.py > gpurun_out/r06/diag_exec_C.log 2>&1
echo "EXEC_C rc=$?"; head -n 8 gpurun_out/r06/diag_exec_C.log
bash tools/r03_pmc_mix.sh r06c C 3
echo DONE
