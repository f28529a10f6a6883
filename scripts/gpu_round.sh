#!/bin/bash
# Full GPU validation: build, GPU tests, default bench, kernel-trace profile.
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
  echo "=== $name rc=$rc ($(date +%T))"; tail -n 6 "$OUT/$name.log"
  return $rc
}
step build 600 python -c "import __graft_entry__ as g; g.build()" || exit 1
step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider; rc=$?; [ $rc -le 1 ] || exit $rc
step smoke 600 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 900 python bench.py || exit 1
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
step rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_default/%pid% -o run -- python3 bench.py --steps 20 --warmup 5 --no-cap-probe
exit 0
