#!/bin/bash
# Round 6 closing measurements, part 2 (after tools/r06_final.sh on the same build): the B and D
# bench lines with their parity legs, then the driver's C line, which quotes the PMC traffic
# filed for this build (tools/traffic_merge.py over part 1's summaries, run here first).
set -u
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
test -f profiles/round_kernel_traffic.json || exit 1  # (filed from part 1 before this call: gpurun_out does not travel)
timeout -k 10 300 python -u bench.py --workload B --steps 10 --warmup 5 > $O/bench_B.json 2> $O/bench_B.err || exit $?
timeout -k 10 600 python -u bench.py --workload D --steps 10 --warmup 5 > $O/bench_D.json 2> $O/bench_D.err || exit $?
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_C_driver_args.json 2> $O/bench_C.err || exit $?
python - <<'EOF'
import json
for w in ("B", "D", "C_driver_args"):
    d = json.loads(open(f"gpurun_out/r06f/bench_{w}.json").read().strip().splitlines()[-1]); r = d["roofline"]
    print(w, round(d["value"] / 1e9, 4), "G parity", d["parity"], "frac", r["frac"], "traffic", r["traffic"], r.get("traffic_note"), "launch us", r["avg_launch_us"])
EOF
echo DONE
