#!/bin/bash
# Round 6: APSP loss sweep arcs in flight per lane (4 / 8 = product / 16, hit lists checked when
# full), Tor V = 1000 and 2000; then the APSP parity tests on the product build.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config.py -k "apsp or route or graph or gml" -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/apsp_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -n 2 gpurun_out/r06/apsp_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for L in libsgn libsgn_exp_q4 libsgn_exp_q16; do
    for V in 1000 2000; do
      SGN_LIB=$PWD/shadow-gen_amd/$L.so timeout -k 10 120 python -u tools/apsp_bench.py tor $V > gpurun_out/r06/apsp.json 2>/dev/null || { echo "FAIL $L"; exit 1; }
      python -c "
import json; d=json.loads(open('gpurun_out/r06/apsp.json').read().strip().splitlines()[-1])
print('$L', 'V', $V, 'total', d['total_ms'], 'latency', d['latency_ms'], 'loss', d['loss_ms'])"
    done
  done
done
echo DONE
