#!/usr/bin/env python3
"""Measure HBM traffic per ICRC launch with rocprofv3 PMC counters.

Runs bench.py under two separate `rocprofv3 --pmc` passes (FETCH_SIZE, then
WRITE_SIZE: they do not fit one pass on gfx950), averages each kernel's
per-dispatch values and applies the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE counts exactly half of
the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is taken as reported.  Both are in KiB.

  (default)  the headline: 1 M x 4096 B, icrc_sck_kernel -> profiles/pmc_traffic.json
  --size N   1 M x N B back to back (64: the quad kernel, C1; 1024 / 2048:
             the SCK, C2) -> profiles/pmc_traffic_N.json
  --mix      C4: the ragged pipeline's four kernels (bucket, fold, one-line,
             gather) summed per step -> profiles/pmc_traffic_mix.json.  The
             bucket pass reads its 12 descriptor bytes per packet once, so its
             doubled FETCH_SIZE against that byte count is reported as a check
             of the x2 correction on scattered traffic
             ("bucket_pass_fetch_over_descriptors").
  --l3-offset O --stride S
             a framed NIC ring: 1 M slots of S bytes, the L3 packet at O in
             each (S - O bytes) -> profiles/pmc_traffic_ringO_S.json
  --count N  packets on the (one) GPU instead of the BASELINE count (1 M, or
             4 M with --mix): C3's 16 GiB batch (--count 4194304) and the
             8-GPU shard stand-ins; the record's name carries N
             (bench.traffic_record).

Copied into profiles/, the file is what bench.py reports as roofline.traffic
when the workload and the kernel sources match (bench.kernel_source_hash).
Usage (on the GPU box):  python3 tools/pmc_traffic.py [--mix | --size N] [--out F]
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pass(counter, outdir, bench_args, match):
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", outdir, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "1", "--no-cpu", "--no-side"] + bench_args
    subprocess.run(cmd, check=True, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), timeout=600,
                   stdout=subprocess.DEVNULL)
    per = {}
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                key = next((m for m in match if m in k), None)
                if key and row["Counter_Name"] == counter:
                    per.setdefault(key, []).append(float(row["Counter_Value"]))
    if not per:
        raise SystemExit(f"no {counter} rows for {match}")
    return {k: (sum(v) / len(v), len(v)) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mix", action="store_true")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--count", type=int, default=None)
    ap.add_argument("--l3-offset", type=int, default=0)
    ap.add_argument("--stride", type=int, default=None)
    ap.add_argument("--slot-lengths", default=None, help="LO:HI: a ring with a length per slot (bench.py's flag)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--scratch", default=os.path.join(ROOT, "gpurun_out", "pmc_traffic"))
    a = ap.parse_args()
    sys.path.insert(0, ROOT)
    import bench

    std = (4 << 20) if a.mix else (1 << 20)
    count = a.count or std
    sl = tuple(int(x) for x in a.slot_lengths.split(":")) if a.slot_lengths else None
    rec = bench.traffic_record(a.mix, a.size, count, a.l3_offset, a.stride, sl)
    if rec is None:
        raise SystemExit(f"no traffic record is kept for --size {a.size}")
    name, srcs, match = rec
    a.out = os.path.abspath(a.out or os.path.join(ROOT, "gpurun_out", name))
    a.scratch = os.path.abspath(a.scratch + ("_mix" if a.mix else f"_{a.size}") + f"_{count}_{a.l3_offset}")
    bench_args = (["--mix"] if a.mix else ["--size", str(a.size)]) + ["--count", str(count)]
    if a.l3_offset or sl:
        bench_args += ["--l3-offset", str(a.l3_offset), "--stride", str(a.stride or a.size)]
    if sl:
        bench_args += ["--slot-lengths", a.slot_lengths]
    fetch = run_pass("FETCH_SIZE", os.path.join(a.scratch, "fetch"), bench_args, match)
    write = run_pass("WRITE_SIZE", os.path.join(a.scratch, "write"), bench_args, match)
    if a.mix:
        import numpy as np

        lens = np.random.default_rng(bench.SEED).choice(np.array(bench.MIX_SIZES, np.uint32), size=count)
        alg = int(lens.sum(dtype=np.uint64)) + 16 * count
        src, size = bench.kernel_source_hash(srcs), "mix"
    elif sl:  # the packets' bytes + 4 written + 4 of length read per slot
        size = a.size
        bargs = bench.parse(bench_args)
        _, _, lens = bench.shard_plan(bargs, 1)
        alg = int(lens.sum(dtype="uint64")) + 8 * count
        src = bench.kernel_source_hash(srcs)
    elif a.l3_offset:
        size = a.size
        alg = count * ((a.stride or a.size) - a.l3_offset) + 4 * count
        src = bench.kernel_source_hash(srcs)
    else:
        size = a.size
        alg = count * size + 4 * count
        src = bench.kernel_source_hash(srcs)
    kernels = {k: {"FETCH_SIZE_KiB": fetch.get(k, (0.0, 0))[0], "WRITE_SIZE_KiB": write.get(k, (0.0, 0))[0],
                   "dispatches": [fetch.get(k, (0, 0))[1], write.get(k, (0, 0))[1]]} for k in match}
    hbm = sum(2.0 * v["FETCH_SIZE_KiB"] * 1024 + v["WRITE_SIZE_KiB"] * 1024 for v in kernels.values())
    res = {"size": size, "count": count, "kernel_src": src, "kernels": kernels,
           **({"l3_offset": a.l3_offset, "stride": a.stride or a.size} if a.l3_offset or sl else {}),
           **({"slot_lengths": list(sl)} if sl else {}),
           "correction": "FETCH_SIZE x2 (gfx950 wide-streaming read undercount, MI355X_MICROARCH.md §HBM)",
           "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": hbm / alg}
    if a.mix and kernels.get("rsck_bucket", {}).get("dispatches", [0])[0]:  # (the three-pass pipeline ran)
        cp = kernels["rsck_bucket"]["FETCH_SIZE_KiB"] * 2 * 1024
        res["bucket_pass_fetch_over_descriptors"] = cp / (12.0 * count)
        res["fold_fetch_over_its_lines"] = None  # filled by tools/pmc_summary.py when the line count is known
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
