#!/bin/bash
# Round 6: the dense loss sweep (loss_sweep_dense) — APSP parity tests, then Tor V = 1000 / 2000
# build times: dense S = 32 (default), S = 16, workgroup targets, and the CSR sweep (SGN_APSP_DENSE=0).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config.py -k "apsp or route or graph or gml" -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/apsp_dense_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -n 3 gpurun_out/r06/apsp_dense_tests.log; [ $rc -eq 0 ] || exit $rc
one() {  # $1 label, rest: env assignments
  local lab=$1; shift
  for V in 1000 2000; do
    env "$@" timeout -k 10 120 python -u tools/apsp_bench.py tor $V > gpurun_out/r06/apsp.json 2>gpurun_out/r06/apsp.err || { echo "FAIL $lab"; cat gpurun_out/r06/apsp.err | tail -5; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r06/apsp.json').read().strip().splitlines()[-1])
print('$lab', 'V', $V, 'total', d['total_ms'], 'latency', d['latency_ms'], 'loss', d['loss_ms'], 'multi', d['loss_multi'])"
  done
}
for i in 1 2; do
  one csr SGN_APSP_DENSE=0
  one dense16h2 SGN_APSP_DENSE=1
  one dense16h1 SGN_APSP_DENSE_H=1
  one dense32 SGN_APSP_DENSE_S=32
  one dense16h2_wg4096 SGN_APSP_DENSE_WG=4096
done
echo DONE
