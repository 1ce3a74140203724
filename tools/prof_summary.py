#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 --kernel-trace CSV.

Prints, per kernel, the mean over all dispatches and over the last K
dispatches (bench.py's timed steps come after its warmup launches, so the
last --steps dispatches are the ones its HIP-event kernel_ms averages)."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last", type=int, default=100)
a = ap.parse_args()
d = collections.defaultdict(list)
with open(a.trace) as f:
    for row in csv.DictReader(f):
        d[row["Kernel_Name"]].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
for k, v in d.items():
    v.sort()
    durs = [x for _, x in v]
    tail = durs[-a.last:]
    print(f"{k}\n  calls {len(durs)}  mean_all_us {sum(durs) / len(durs) / 1e3:.1f}  "
          f"mean_last{len(tail)}_us {sum(tail) / len(tail) / 1e3:.1f}  min_us {min(durs) / 1e3:.1f}  max_us {max(durs) / 1e3:.1f}")
