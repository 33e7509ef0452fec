#!/bin/bash
# PERIODIC forwarding wait as a product feature (waves with >= 24 lanes in their loops): the full
# -m gpu suite, then same-box A/B against HEAD's build and the threshold variants.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r05/fwdwait_gpu_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -3 gpurun_out/r05/fwdwait_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
one() {  # workload, lib
  SGN_LIB=$PWD/shadow-gen_amd/$2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline --workload $1 > gpurun_out/r05/fw.json 2>/dev/null || { echo "FAIL $1 $2"; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r05/fw.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$1', '$2', round(d['value']/1e9,4), 'G  ms/step', round(d['ms_per_step'],4), ' launch us', r['avg_launch_us'])"
}
for i in 1 2; do
  for L in libsgn_exp_head.so libsgn.so libsgn_exp_fw8.so libsgn_exp_fw40.so libsgn_exp_fwdwait.so; do one D $L; done
done
for i in 1 2; do for L in libsgn_exp_head.so libsgn.so libsgn_exp_fw8.so; do one B $L; done; done
echo DONE
