set -u
for i in 1 2; do
for L in shadow-gen_amd/libsgn.so shadow-gen_amd/libsgn_exp_w0.so shadow-gen_amd/libsgn_exp_w2.so shadow-gen_amd/libsgn_exp_w16.so shadow-gen_amd/libsgn_exp_w40.so; do
  SGN_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/abw.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/abw.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$L', round(d['value']/1e9,4), r['avg_launch_us'])"
done; done
