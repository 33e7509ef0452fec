#!/bin/bash
# Session GPU cycle: chosen -m gpu test files ($2, default all), then the 2-rank RCCL
# rehearsal at 100k hosts per rank (graph-captured rounds). Tag = $1.
set -u
T=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${2:-tests} -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_$T.log 2>&1
rc=$?; echo "PYTEST $rc"; tail -4 gpurun_out/t_$T.log; [ $rc -eq 0 ] || exit $rc
bash tools/rccl_one_gpu.sh $T 2
