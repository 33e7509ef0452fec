set -u
export TMPDIR=/tmp
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export SGN_BENCH_SORTED=1; else unset SGN_BENCH_SORTED; fi
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 10 --warmup 5 > gpurun_out/exp1_$v.json 2>&1 || exit 1
  python -c "import json;d=json.load(open('gpurun_out/exp1_$v.json'));print('sorted=$v', round(d['value']/1e6,1), 'M/s', d['roofline']['avg_launch_us'], d['packet_events_timed'])"
done
