#!/bin/bash
# The multi-shard RCCL path on a ONE-GPU box: N ranks (default 2) on device 0, each with its
# own NCCL_HOSTID so RCCL accepts them (bench.py --one-gpu); the exchange goes over RCCL's
# socket transport on loopback. Checks the sharded APSP exchange and the round-edge exchange
# bit for bit (bench's shard_check re-runs all hosts unsharded on rank 0). Tag = $1.
set -u
T=${1:-x}; N=${2:-2}; W=${3:-C}; H=${4:-100000}
mkdir -p gpurun_out
export TMPDIR=/tmp NCCL_DEBUG=WARN
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus $N --steps 2 --warmup 1 --one-gpu --workload $W --hosts $H \
  > gpurun_out/rccl1_$T.json 2> gpurun_out/rccl1_$T.err
rc=$?; echo "RCCL1 $rc"; cat gpurun_out/rccl1_$T.json; tail -5 gpurun_out/rccl1_$T.err; exit $rc
