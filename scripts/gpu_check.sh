#!/bin/bash
# One GPU-box session: build in-tree, GPU tests, short bench.  Every GPU step
# has its own time limit; the script stops at the first fault/abort/timeout.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out
STAGE=${1:-all}

step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))"
  tail -n 25 "$OUT/$name.log"
  return $rc
}

ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

step build 600 python -c "import __graft_entry__ as g; g.build()" || exit 1
rocminfo > "$OUT/rocminfo.txt" 2>&1 || true

if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider
  rc=$?; ok_or_testfail $rc || exit $rc
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  step bench 900 python bench.py --steps 20 --warmup 5
  rc=$?; [ $rc -eq 0 ] || exit $rc
  grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"
fi
exit 0
