#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out
run() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/v_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep '^{' "$OUT/v_$name.log" | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['per_pod_images_s'])" 2>/dev/null
  return $rc
}
python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_gpu_fused.py -q -x -p no:cacheprovider > $OUT/pytest_fused.log 2>&1; rc=$?; tail -3 $OUT/pytest_fused.log; [ $rc -le 1 ] || exit 1
B="python bench.py --steps 30 --warmup 5 --no-cap-probe"
run e_q1_nograph 400 $B --pods 1 --no-shim --gpucores 100 --gpumem 0 --no-graph || exit 1
run e_q4_nograph 400 $B --pods 1 --no-shim --gpucores 100 --gpumem 0 --no-graph --hw-queues 0 || exit 1
run e_q1_graph 400 $B --pods 1 --no-shim --gpucores 100 --gpumem 0 || exit 1
run e_q1_nofuse 400 $B --pods 1 --no-shim --gpucores 100 --gpumem 0 --no-fused || exit 1
run p2_q1_graph 400 $B --pods 2 || exit 1
run p2_q1_nograph 400 $B --pods 2 --no-graph || exit 1
run p2_q2_nograph 400 $B --pods 2 --no-graph --hw-queues 2 || exit 1
run p2_nomask_q1 400 $B --pods 2 --no-shim || exit 1
run p4_q1_graph 400 $B --pods 4 --gpucores 25 --gpumem 70000 || exit 1
run p4_q1_nograph 400 $B --pods 4 --gpucores 25 --gpumem 70000 --no-graph || exit 1
exit 0
