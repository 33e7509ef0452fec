set -u
export TMPDIR=/tmp
for v in id kind id kind; do
  SGN_HOST_ORDER=$v timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 10 --warmup 5 > gpurun_out/expo_$v.json 2>&1 || exit 1
  python -c "import json;d=json.load(open('gpurun_out/expo_$v.json'));print('$v', round(d['value']/1e6,1), 'M/s', d['roofline']['avg_launch_us'])"
done
