#!/bin/bash
# Closing D measurements after the PERIODIC forwarding wait: bench line, keyed PMC traffic, the
# B line, and the D multi-shard rehearsal.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u bench.py --workload D --no-cpu-baseline > gpurun_out/r05/bench_D.json 2> gpurun_out/r05/bench_D.err || exit $?
echo "BENCH D ok"
bash tools/pmc_traffic.sh r05f_D D 10 5 > gpurun_out/r05/traffic_D.log 2>&1 || { echo "TRAFFIC D failed"; exit 1; }
cp gpurun_out/traffic_r05f_D/summary.json gpurun_out/r05/traffic_D.json
echo "TRAFFIC D ok"
timeout -k 10 400 python -u bench.py --workload B --no-cpu-baseline > gpurun_out/r05/bench_B.json 2> gpurun_out/r05/bench_B.err || exit $?
echo "BENCH B ok"
timeout -k 10 400 python -u tools/xpersist_bench.py --workload D --hosts 1000000 --shards 1,2,4,8 --rounds 200 --warmup 50 > gpurun_out/r05/xb3_D.jsonl 2>&1 || exit $?
echo DONE
