set -u
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_all2.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -2 gpurun_out/gpu_all2.log
case $rc in 124|134|137|139) exit $rc;; esac
for W in B D; do
  timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline > gpurun_out/bench2_$W.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/bench2_$W.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$W', round(d['value']/1e9,4), r['avg_launch_us'])"
done
bash tools/ab_lib.sh shadow-gen_amd/libsgn.so shadow-gen_amd/libsgn_exp_rbrel.so C 2
