#!/bin/bash
# C4's bimodal step time: N separate bench processes, each recording where its
# batch, descriptors and ragged workspace landed (RICRC_DEBUG=1) next to its
# step time, to see whether the mode follows placement.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-c4_modes}; mkdir -p $O
for r in $(seq 1 ${RUNS:-8}); do
  RICRC_DEBUG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --mix ${ARGS:-} > $O/run_$r.json 2> $O/run_$r.err || exit 3
  python3 - "$O/run_$r.json" "$O/run_$r.err" <<'PY'
import json, re, sys
d = json.load(open(sys.argv[1])); e = open(sys.argv[2]).read()
buf = re.search(r"buf (0x[0-9a-f]+) offs (0x[0-9a-f]+) lens (0x[0-9a-f]+)", e)
ws = re.findall(r"ragged workspace (0x[0-9a-f]+)", e)
b, o, l = (int(x, 16) for x in buf.groups())
w = int(ws[-1], 16) if ws else 0
print(f"ms/step {d['ms_per_step']:.4f} kernel {d['roofline']['kernel_ms']:.4f} | buf {b:#x} (mod 2M {b % (2<<20):#x}, mod 1G {b % (1<<30):#x}) "
      f"offs {o:#x} lens {l:#x} ws {w:#x} (mod 2M {w % (2<<20):#x})")
PY
done
