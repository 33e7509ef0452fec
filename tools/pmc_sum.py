"""Per-dispatch averages of the counters a PMC pass directory holds (tools/pmc_exec.sh)."""
import collections, csv, glob, sys

d = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:20s} {c:24s} n={len(v):5d} mean={sum(v) / len(v):14.1f}")
