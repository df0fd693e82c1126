"""Average every PMC counter of the dispatches whose kernel name contains a substring.

  pmc_avg.py DIR KERNEL_SUBSTRING
"""
import collections
import csv
import glob
import os
import sys

d, sub = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if sub in row.get("Kernel_Name", ""):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:32s} n={len(v):4d} avg={sum(v) / len(v):.4g}")
