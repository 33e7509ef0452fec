#!/bin/bash
# Round 6, first GPU call: the whole -m gpu suite (new: D sharded / steady state, launcher-less
# N-rank bench, refusal fallback), the driver's bench line, and the xGMI message fences priced on
# the two-process one-GPU rehearsal (product build vs the no-fence experiment build).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06/gpu_tests_a.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -n 3 gpurun_out/r06/gpu_tests_a.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/bench_a.json 2> gpurun_out/r06/bench_a.err || exit $?
python - <<'EOF'
import json; d=json.loads(open('gpurun_out/r06/bench_a.json').read().strip().splitlines()[-1]); r=d['roofline']
print('BENCH C', round(d['value']/1e9,4), 'G parity', d['parity'], 'launch us', r['avg_launch_us'], 'frac', r['frac'])
EOF
for L in shadow-gen_amd/libsgn.so shadow-gen_amd/libsgn_exp_xnofence.so shadow-gen_amd/libsgn.so shadow-gen_amd/libsgn_exp_xnofence.so; do
  SGN_LIB=$PWD/$L SGN_XPEER_SHARED=1 SGN_GRAPH=0 NCCL_DEBUG=WARN timeout -k 10 300 python -u bench.py --gpus 2 --one-gpu \
    --steps 5 --warmup 2 --no-shard-check > gpurun_out/r06/xfence.json 2> gpurun_out/r06/xfence.err || { echo "FAIL $L"; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r06/xfence.json').read().strip().splitlines()[-1]); r=d['roofline']
print('XPEER C 2 procs', '$L', r['kernel'], 'round us', r['latency_bound']['round_us'], 'launch us', r['avg_launch_us'])"
done
echo DONE
