#!/usr/bin/env python3
"""One line per bench process of tools/c4_modes.sh: step and kernel time, the
ragged pipeline's per-pass times (--pass-times), and the GPU state read by
amd-smi in the same process right before and after the timed steps (mean gfx
clock over the XCDs, memory and fabric clocks, socket power, hotspot / HBM
temperature).

    python tools/c4_modes_summary.py gpurun_out/<tag>/run_*.json
"""
import json
import sys


def state(st):
    if not isinstance(st, dict) or "data" not in st:
        return "n/a"
    g = st["data"]["gpu_data"][0]
    clk = g.get("clock", {})
    gfx = [v["clk"]["value"] for k, v in clk.items() if k.startswith("gfx_") and isinstance(v.get("clk"), dict)]
    mem = clk.get("mem_0", {}).get("clk", {}).get("value", "n/a")
    fclk = clk.get("fclk_0", {}).get("clk", {}).get("value", "n/a")
    pw = g.get("power", {}).get("socket_power", {}).get("value", "n/a")
    t = g.get("temperature", {})
    hot = t.get("hotspot", {}).get("value", "n/a") if isinstance(t.get("hotspot"), dict) else "n/a"
    hbm = t.get("mem", {}).get("value", "n/a") if isinstance(t.get("mem"), dict) else "n/a"
    g_mean = f"{sum(gfx) / len(gfx):.0f}" if gfx else "n/a"
    g_rng = f"{min(gfx)}-{max(gfx)}" if gfx else "n/a"
    return f"gfx {g_mean} MHz ({g_rng}) mem {mem} fclk {fclk} MHz {pw} W hot {hot} C hbm {hbm} C"


def main(paths):
    for p in paths:
        d = json.load(open(p))
        pm = d.get("pass_ms") or {}
        passes = " ".join(f"{k} {v * 1e3:.1f}" for k, v in pm.items())
        print(f"{p}: ms/step {d['ms_per_step']:.4f} kernel {d['roofline']['kernel_ms']:.4f} | passes (us) {passes} "
              f"| before: {state(d.get('gpu_state_before'))} | after: {state(d.get('gpu_state_after'))}")


if __name__ == "__main__":
    main(sys.argv[1:])
