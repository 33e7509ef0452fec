#!/bin/bash
# Round-3 iteration on the GPU box: GPU tests (optionally a -k filter), then short benches.
# $1 = tag, $2 = pytest -k expression ("" = all), $3 = "bench" to run the bench legs.
set -u
T=${1:-x}; K=${2:-}; B=${3:-bench}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread "${KA[@]}" > gpurun_out/t_$T.log 2>&1
rc=$?; echo "PYTEST $rc"; tail -4 gpurun_out/t_$T.log; [ $rc -eq 0 ] || exit $rc
[ "$B" = "bench" ] || exit 0
timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/bC_$T.json 2> gpurun_out/bC_$T.err
rc=$?; echo "BENCH_C $rc"; cat gpurun_out/bC_$T.json | head -c 1500; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline --hosts 50000 > gpurun_out/bC50_$T.json 2> gpurun_out/bC50_$T.err
rc=$?; echo "BENCH_C50 $rc"; [ $rc -eq 0 ] || exit $rc
SGN_PERSISTENT=0 timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline --hosts 50000 > gpurun_out/bC50e_$T.json 2> gpurun_out/bC50e_$T.err
rc=$?; echo "BENCH_C50_EXEC $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --one-gpu > gpurun_out/rccl2_$T.json 2> gpurun_out/rccl2_$T.err
rc=$?; echo "RCCL2 $rc"; tail -3 gpurun_out/rccl2_$T.err; exit $rc
