#!/bin/bash
# Session 37: C4's bimodal step time -- 6 bench processes, each under rocprofv3 --kernel-trace,
# to see which pass differs between the fast and the slow mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3s37}; mkdir -p "$OUT"
for r in 1 2 3 4 5 6; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/p$r" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --mix > "$OUT/b$r.json" 2> "$OUT/b$r.err" || exit 3
  python3 - "$OUT/b$r.json" "$OUT/p$r/run_kernel_trace.csv" <<'PY'
import csv, json, sys, collections
d = json.load(open(sys.argv[1]))
k = collections.defaultdict(list)
for row in csv.DictReader(open(sys.argv[2])):
    k[row["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1]].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
out = []
for name in ("rsck_bucket", "icrc_rsck_kernel", "icrc_rsmall_kernel", "rsck_gather"):
    v = sorted(k[name])[-20:]
    out.append(f"{name} {sum(e - s for s, e in v) / len(v) / 1e3:.1f}")
# step span: first bucket start to last gather end over the last 20 steps, / 20
b = sorted(k["rsck_bucket"])[-20:]; g = sorted(k["rsck_gather"])[-20:]
print(f"ms/step {d['ms_per_step']:.4f} kernel {d['roofline']['kernel_ms']:.4f} | " + " | ".join(out) + f" | span/step {(g[-1][1] - b[0][0]) / 20 / 1e3:.1f} us")
PY
done
