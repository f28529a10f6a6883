#!/bin/bash
# GPU round 2: pager test, vmem bench (config 5), suite (all ai-benchmark tests).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))"; tail -n 4 "$OUT/$name.log" | cut -c1-1500
  return $rc
}
step build 600 python -c "import __graft_entry__ as g; g.build()" || exit 1
step pytest_pager 600 python -m pytest tests/test_pager.py -m gpu -q -p no:cacheprovider; rc=$?; [ $rc -le 1 ] || exit $rc
step vmem 900 python -m vgpu.bench.vmem --spill-gib 8 --budget-gib 8 --tokens 16 || exit 1
step suite 1500 python -m vgpu.bench.suite --steps 10 --warmup 3 --timeout 600 || exit 1
exit 0
