"""Summarise a rocprofv3 --kernel-trace --stats CSV directory (run_kernel_stats.csv)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for x in rows:
    print(f"{x['Name'][:44]:44s} calls={int(x['Calls']):6d} total_ms={float(x['TotalDurationNs'])/1e6:9.2f} "
          f"avg_us={float(x['AverageNs'])/1e3:9.2f} min_us={float(x['MinNs'])/1e3:8.2f} "
          f"max_us={float(x['MaxNs'])/1e3:9.2f} pct={float(x['Percentage']):6.2f}")
