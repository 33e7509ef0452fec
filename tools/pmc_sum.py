"""Sums PMC counters per dispatch over rocprofv3 --pmc output directories (argv[1:])."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f:
        print(d, "no data")
        continue
    acc = collections.defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(f[0])):
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
    print(d, "dispatches", len(disp))
    for k, v in sorted(acc.items()):
        print(f"  {k}: {v / len(disp):.5g} per dispatch")
