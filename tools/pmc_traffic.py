#!/usr/bin/env python3
"""Measure HBM traffic per ICRC launch with rocprofv3 PMC counters.

Runs bench.py under two separate `rocprofv3 --pmc` passes (FETCH_SIZE, then
WRITE_SIZE: they do not fit one pass on gfx950), averages the streaming
kernel's per-dispatch values and applies the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE counts exactly half of
the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is taken as reported (4 B per packet, small).  Both are in KiB.

Writes gpurun_out/pmc_traffic.json; copied into profiles/pmc_traffic.json it is
what bench.py reports as roofline.traffic when the workload matches.  Usage (on the GPU box):
    python3 tools/pmc_traffic.py [--out profiles/pmc_traffic.json]
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pass(counter, outdir):
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", outdir, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "1", "--no-cpu"]
    subprocess.run(cmd, check=True, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), timeout=600,
                   stdout=subprocess.DEVNULL)
    vals, names = [], set()
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                if "icrc_sck_kernel" in k and row["Counter_Name"] == counter:  # the headline kernel only
                    vals.append(float(row["Counter_Value"]))
                    names.add(k)
    if not vals:
        raise SystemExit(f"no {counter} rows for the icrc kernel")
    return sum(vals) / len(vals), len(vals), names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc_traffic.json"))
    ap.add_argument("--scratch", default=os.path.join(ROOT, "gpurun_out", "pmc_traffic"))
    a = ap.parse_args()
    a.out, a.scratch = os.path.abspath(a.out), os.path.abspath(a.scratch)
    fetch_kib, nf, kernels = run_pass("FETCH_SIZE", os.path.join(a.scratch, "fetch"))
    write_kib, nw, _ = run_pass("WRITE_SIZE", os.path.join(a.scratch, "write"))
    count, size = 1 << 20, 4096
    hbm = 2.0 * fetch_kib * 1024 + write_kib * 1024
    alg = count * size + 4 * count
    sys.path.insert(0, ROOT)
    import bench

    res = {"size": size, "count": count, "dispatches": [nf, nw], "kernel_src": bench.kernel_source_hash(),
           "kernels": sorted(kernels),
           "FETCH_SIZE_KiB": fetch_kib, "WRITE_SIZE_KiB": write_kib,
           "correction": "FETCH_SIZE x2 (gfx950 wide-streaming read undercount, MI355X_MICROARCH.md §HBM)",
           "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": hbm / alg}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
