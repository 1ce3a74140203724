#!/bin/bash
# Build the "prev" side of the same-box A/B tools from a commit (default HEAD):
# tools/ab/libroceicrc_prev.so and tools/microbench/rsck_abl_prev.  Runs here
# (build container), not on the GPU box.
set -eu
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
cd "$ROOT"
for f in $(git ls-files roce-test_amd/csrc include); do mkdir -p "$T/$(dirname "$f")"; git show "$REV:$f" > "$T/$f"; done
mkdir -p "$T/roce-test_amd/roce_icrc" "$T/tools/microbench" tools/ab
make -s -C "$T/roce-test_amd/csrc" -j8 > /dev/null
cp "$T/roce-test_amd/roce_icrc/libroceicrc.so" tools/ab/libroceicrc_prev.so
cp tools/microbench/rsck_abl.hip "$T/tools/microbench/"
(cd "$T/tools/microbench" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 rsck_abl.hip -o "$ROOT/tools/microbench/rsck_abl_prev" 2>&1 | grep -v unused || true)
rm -rf "$T"
echo "prev = $(git rev-parse --short "$REV")"
