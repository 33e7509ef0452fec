#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per access of the engine's access widths (tools/pmc_calib.hip); $1 = tag.
set -u
T=${1:-x}
mkdir -p gpurun_out/calib_$T
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c -d gpurun_out/calib_$T/$c -o run --output-format csv -- ./tools/pmc_calib > gpurun_out/calib_$T/$c.log 2>&1
  rc=$?; echo "CALIB $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python - gpurun_out/calib_$T <<'PY'
import csv, glob, json, sys
d = sys.argv[1]
names = ["ld_dev 8B", "load 16B", "record 32B", "line 8x16B", "st_dev 8B", "store 16B", "st_dev record 32B"]
req = [8, 16, 32, 16, 8, 16, 32]
n = 1 << 22
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{d}/{c}/**/*counter_collection.csv", recursive=True)[0]
    v = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == c and r["Kernel_Name"].startswith("k("):
            v[int(r["Dispatch_Id"])] = v.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    out[c] = [v[k] for k in sorted(v)][-7:]
res = []
for i, nm in enumerate(names):
    fb = out["FETCH_SIZE"][i] * 1024 / n
    wb = out["WRITE_SIZE"][i] * 1024 / n
    res.append({"access": nm, "requested_B": req[i], "fetch_B_per_access": round(fb, 2), "write_B_per_access": round(wb, 2)})
    print(f"{nm:18s} requested {req[i]:3d} B  FETCH_SIZE {fb:7.2f} B/access  WRITE_SIZE {wb:7.2f} B/access")
json.dump(res, open(f"{d}/calib.json", "w"), indent=1)
PY
