#!/bin/bash
# Debug run of the 2-rank one-GPU RCCL rehearsal with the sgn_run batch trace. Tag = $1,
# then env assignments for the ranks (e.g. SGN_GRAPH=0 SGN_XSZ_INIT=16).
set -u
T=${1:-x}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp NCCL_DEBUG=WARN SGN_DEBUG_RUN=1 "$@"
timeout -k 10 100 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29551 bench.py --gpus 2 --steps 2 --warmup 1 --one-gpu --hosts 20000 --rounds-per-step 70 \
  > gpurun_out/dbg_$T.json 2> gpurun_out/dbg_$T.err
rc=$?; echo "DBG $rc"; grep "\[sgn" gpurun_out/dbg_$T.err | tail -30; cat gpurun_out/dbg_$T.json | cut -c1-300; exit $rc
