#!/usr/bin/env python3
"""Per-wave-step instruction table of the ragged fold vs the strided-chain
kernel from tools/pmc_insts.sh's rocprofv3 CSVs.  A wave step is one
16-byte-per-lane load = one 128-byte line of each of the 8 packets of a
group.  Headline: 1 M x 4096 B -> 4 M wave steps.  C4 mix: the fold's
steps are the line counts of its (>= 2-line) packets / 8, from bench.py's
own length vector (packed back to back, so a packet's line count follows
from its offset)."""
import collections
import csv
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def counters(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def fold_steps_mix():
    import bench

    lens = np.random.default_rng(bench.SEED).choice(np.array(bench.MIX_SIZES, np.uint64), size=4 << 20)
    offs = np.zeros(len(lens), np.uint64)
    offs[1:] = np.cumsum(lens[:-1])
    L = ((offs & 127) + lens - 4 + 127) // 128
    big = L >= 2
    groups_lines = 0
    for l in np.unique(L[big]):  # groups of 8 equal-L packets, padded
        n = int((L == l).sum())
        groups_lines += ((n + 7) // 8) * int(l)
    return groups_lines, int(L[big].sum()), int((~big).sum())


def main():
    out = sys.argv[1]
    res = {}
    for wl, kname in (("headline", "icrc_sck_kernel"), ("mix", "icrc_rsck_kernel")):
        c = collections.defaultdict(list)
        for p in glob.glob(os.path.join(out, wl + "_p*")):
            for k, ctr in counters(p).items():
                if kname in k:
                    for n, v in ctr.items():
                        c[n] += v
        if not c:
            continue
        steps = (1 << 20) * 32 / 8 if wl == "headline" else fold_steps_mix()[0]
        res[wl] = {n: (sum(v) / len(v)) / steps for n, v in c.items()}
        res[wl]["_steps"] = steps
    names = sorted(set().union(*[set(r) for r in res.values()]) - {"_steps"})
    print(f"{'per wave step (8 lines of 128 B)':34s} " + " ".join(f"{w:>14s}" for w in res))
    print(f"{'wave steps per launch':34s} " + " ".join(f"{res[w]['_steps']:14.0f}" for w in res))
    for n in names:
        print(f"{n:34s} " + " ".join(f"{res[w].get(n, float('nan')):14.2f}" for w in res))
    if "mix" in res:
        g, lines, small = fold_steps_mix()
        print(f"\nmix: {lines} lines in >= 2-line packets, {g} wave steps incl. group padding, {small} one-line packets")


if __name__ == "__main__":
    main()
