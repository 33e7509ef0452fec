#!/bin/bash
# Round 6: the fused first pass (dense tight sweep on the direct arcs = the squaring's first
# pass) — APSP parity suites, then Tor V = 1000 / 2000 build times: fused (default) against the
# unfused dense sweep (SGN_APSP_FUSED=0).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config.py -k "apsp or route or graph or gml" -x -v -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/apsp_fused_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; grep -E "FAIL|ERROR|Error|assert" gpurun_out/r06/apsp_fused_tests.log | head -20; tail -n 2 gpurun_out/r06/apsp_fused_tests.log; [ $rc -eq 0 ] || exit $rc
one() {  # $1 label, rest: env assignments
  local lab=$1; shift
  for V in 1000 2000; do
    env "$@" timeout -k 10 120 python -u tools/apsp_bench.py tor $V > gpurun_out/r06/apsp.json 2>gpurun_out/r06/apsp.err || { echo "FAIL $lab"; tail -5 gpurun_out/r06/apsp.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r06/apsp.json').read().strip().splitlines()[-1])
print('$lab', 'V', $V, 'total', d['total_ms'], 'latency', d['latency_ms'], 'loss', d['loss_ms'], 'passes', d['latency_passes'], d['loss_form'])"
  done
}
for i in 1 2 3; do
  one unfused SGN_APSP_FUSED=0
  one fused SGN_APSP_FUSED=1
  one fused_wg2048 SGN_APSP_DENSE_WG=2048
  one fused_wg8192 SGN_APSP_DENSE_WG=8192
done
echo DONE
