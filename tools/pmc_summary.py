"""Summarise rocprofv3 --pmc CSVs per kernel: mean counter value per dispatch."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "?")
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, ctrs in acc.items():
    if "synth" in k:
        continue
    print(f"== {k}")
    for name in sorted(ctrs):
        v = ctrs[name]
        print(f"  {name:32s} mean {sum(v)/len(v):16.1f}   (n={len(v)})")
