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
timeout -k 10 300 python -m vgpu.bench.convbench > $OUT/convbench.log 2>&1; echo "convbench rc=$?"
timeout -k 10 400 python -m vgpu.bench.convbench --find > $OUT/convbench_find.log 2>&1; echo "convbench find rc=$?"
B="python bench.py --steps 30 --warmup 5 --no-cap-probe --no-graph"
GPU_MAX_HW_QUEUES=1 run p2_m50_q1 300 $B --pods 2 || exit 1
GPU_MAX_HW_QUEUES=1 run p4_m25_q1 300 $B --pods 4 --gpucores 25 --gpumem 70000 || exit 1
GPU_MAX_HW_QUEUES=1 run p2_nomask_q1 300 $B --pods 2 --no-shim || exit 1
GPU_MAX_HW_QUEUES=2 run p4_m25_q2 300 $B --pods 4 --gpucores 25 --gpumem 70000 || exit 1
run p1_m25 300 $B --pods 1 --gpucores 25 --gpumem 70000 || exit 1
run p1_excl_find 600 $B --pods 1 --no-shim --gpucores 100 --gpumem 0 --find || exit 1
exit 0
