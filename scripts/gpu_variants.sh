#!/bin/bash
# Bench variants + a kernel-trace profile of the flagship config.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out
run() {  # run <name> <secs> <args...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" python bench.py "$@" > "$OUT/v_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep '^{' "$OUT/v_$name.log" | tail -1
  return $rc
}
python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || exit 1
run exclusive 600 --pods 1 --no-shim --gpucores 100 --gpumem 0 --steps 30 --warmup 5 --no-cap-probe || exit 1
run shared2_nomask 600 --pods 2 --no-shim --steps 30 --warmup 5 --no-cap-probe || exit 1
run shared2 600 --pods 2 --steps 30 --warmup 5 --no-cap-probe || exit 1
run shared4 600 --pods 4 --gpucores 25 --gpumem 70000 --steps 30 --warmup 5 --no-cap-probe || exit 1
run shared2_nograph 600 --pods 2 --steps 30 --warmup 5 --no-cap-probe --no-graph || exit 1
echo "=== rocprof ($(date +%T))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shared2 -o run -- python3 bench.py --pods 2 --steps 20 --warmup 5 --no-cap-probe > $OUT/prof_shared2.log 2>&1
echo "=== rocprof rc=$?"
exit 0
