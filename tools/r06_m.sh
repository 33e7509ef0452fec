#!/bin/bash
# Round 6: the N = 8 persistent multi-shard path as EIGHT processes on one GPU (IPC-mapped
# uncached inboxes, the census across processes, system-scope message stores), launched the way
# the driver does it (bench.py --gpus 8, no launcher), checked by bench's unsharded shard_check.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
SGN_XPEER_SHARED=1 SGN_GRAPH=0 NCCL_DEBUG=WARN timeout -k 10 400 python -u bench.py --gpus 8 --one-gpu --steps 2 --warmup 1 \
  --rounds-per-step 40 > gpurun_out/r06/xpeer8.json 2> gpurun_out/r06/xpeer8.err
rc=$?; echo "XPEER8 rc=$rc"; tail -n 5 gpurun_out/r06/xpeer8.err
[ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json; d=json.loads(open('gpurun_out/r06/xpeer8.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'parity', d['parity'], d['parity_detail']['hosts_compared'], 'exchange', d['exchange'], 'kernel', d['roofline']['kernel'], 'round us', d['roofline']['latency_bound']['round_us'])
PY
echo DONE
