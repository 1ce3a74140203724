#!/bin/bash
# Snapshot the working tree (or a git revision) into tools/ab/<name>/ and
# build its library in place, for tools/ab_multi.sh:
#   bash tools/ab_snap.sh va            working tree
#   bash tools/ab_snap.sh prev HEAD     a revision
set -eu
cd "$(dirname "$0")/.."
d=tools/ab/$1; rm -rf "$d"; mkdir -p "$d/tools"
if [ -n "${2:-}" ]; then
  git archive "$2" roce-test_amd bench.py oracle include __graft_entry__.py tools/ring_bench.py | tar -x -C "$d"
else
  cp -r roce-test_amd bench.py oracle include __graft_entry__.py "$d"; cp tools/ring_bench.py "$d/tools"
fi
rm -rf "$d"/roce-test_amd/csrc/obj "$d"/roce-test_amd/roce_icrc/*.so
make -s -j8 -C "$d/roce-test_amd/csrc" > /dev/null
make -s -C "$d/oracle" > /dev/null
