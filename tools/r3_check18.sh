#!/bin/bash
# Session 18: PMC traffic records for C1 (64 B, quad) and C2 (1024 B, SCK); half-line fetch microbench (time + FETCH_SIZE).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3s18}; mkdir -p "$OUT"
timeout -k 10 60 ./tools/microbench/half_line > "$OUT/half_line.txt" 2>&1 || exit 2
cat "$OUT/half_line.txt"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/hl_pmc" -o run -- ./tools/microbench/half_line > "$OUT/hl_pmc.log" 2>&1 || exit 3
python3 - "$OUT/hl_pmc" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if row["Counter_Name"] == "FETCH_SIZE":
            d[row["Kernel_Name"].split("(")[0]].append(float(row["Counter_Value"]))
for k, v in d.items():
    print(k, "FETCH_SIZE KiB mean", sum(v) / len(v), "x2 / 2 GiB =", 2 * sum(v) / len(v) * 1024 / 2**31)
PY
timeout -k 10 280 python3 tools/pmc_traffic.py --size 64 --out "$OUT/pmc_traffic_64.json" --scratch "$OUT/pmc" > "$OUT/pmc64.log" 2>&1 || exit 4
timeout -k 10 280 python3 tools/pmc_traffic.py --size 1024 --out "$OUT/pmc_traffic_1024.json" --scratch "$OUT/pmc" > "$OUT/pmc1024.log" 2>&1 || exit 5
for f in "$OUT"/pmc_traffic_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['traffic_over_algorithmic'], d['kernels'])"; done
