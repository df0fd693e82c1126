"""Summarise a rocprofv3 kernel_stats.csv: name, calls, avg us, total ms, %."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    n = r["Name"]
    n = n[:70]
    print(f"{n:72s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:10.2f}us {float(r['TotalDurationNs'])/1e6:9.2f}ms {float(r['Percentage']):6.2f}%")
