#!/bin/bash
# A/B: one pod's batch as forked micro-batches inside its hipGraph (VGPU_POD_SPLIT),
# against the default, interleaved so box drift hits both arms.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 300 "$@" > "$OUT/split_$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' "$OUT/split_$name.log" | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
B="python bench.py --steps 30 --warmup 10 --no-cap-probe"
for r in 1 2; do
  run base_$r $B || exit 1
  VGPU_POD_SPLIT=2 run s2q1_$r $B || exit 1
  VGPU_POD_SPLIT=2 run s2q2_$r $B --hw-queues 2 || exit 1
  run baseq2_$r $B --hw-queues 2 || exit 1
  VGPU_POD_SPLIT=2 run s2q4_$r $B --hw-queues 4 || exit 1
done
run excl $B --pods 1 --gpucores 100 --gpumem 0 || exit 1
VGPU_POD_SPLIT=2 run excl_s2q2 $B --pods 1 --gpucores 100 --gpumem 0 --hw-queues 2 || exit 1
exit 0
