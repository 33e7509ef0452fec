#!/bin/bash
# Round 6: the frontier form of the sparse latency pass (bf_front) against every-arc sweeps
# (SGN_APSP_BF_SWEEP=1) on the B / D graph (random, V = 1000 / 2000), after the APSP parity tests.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config.py -k "apsp or route or graph or gml" -x -q -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/apsp_bffront_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; grep -E "FAIL|Error" gpurun_out/r06/apsp_bffront_tests.log | head; tail -n 2 gpurun_out/r06/apsp_bffront_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for lab in sweep front; do
    for V in 1000 2000; do
      if [ $lab = sweep ]; then E=1; else E=; fi
      SGN_APSP_BF_SWEEP=$E timeout -k 10 120 python -u tools/apsp_bench.py random $V > gpurun_out/r06/apsp.json 2>gpurun_out/r06/apsp.err || { echo "FAIL $lab"; tail -5 gpurun_out/r06/apsp.err; exit 1; }
      python -c "
import json; d=json.loads(open('gpurun_out/r06/apsp.json').read().strip().splitlines()[-1])
print('$lab', 'V', $V, 'arcs', d['arcs'], 'total', d['total_ms'], 'latency', d['latency_ms'], 'loss', d['loss_ms'], 'sweeps', d['latency_passes'])"
    done
  done
done
echo DONE
