#!/bin/bash
# A/B: conv tile grid-fill threshold sized for the pod's CUs, interleaved.
#   default  = CUs derived from VGPU_DEVICE_CU_LIMIT_0 (128 for a 50 % pod), threshold 1.5 x CUs
#   c256     = VGPU_CONV_CUS=256 (the chip-wide threshold 384; previous behaviour ~ 512)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 300 "$@" > "$OUT/cus_$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' "$OUT/cus_$name.log" | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
B="python bench.py --steps 30 --warmup 10 --no-cap-probe"
E="$B --pods 1 --gpucores 100 --gpumem 0"
for r in 1 2; do
  run flag_$r $B || exit 1
  VGPU_CONV_CUS=256 run flag_c256_$r $B || exit 1
  run excl_$r $E || exit 1
  VGPU_CONV_CUS=342 run excl_old_$r $E || exit 1
  VGPU_CONV_CUS=128 run excl_c128_$r $E || exit 1
done
exit 0
