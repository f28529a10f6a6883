#!/bin/bash
# Native weight gradient: numerics tests, per-layer timing vs MIOpen, training step A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad or train" > $OUT/wgrad_pytest.log 2>&1
rc=$?; tail -12 $OUT/wgrad_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m vgpu.bench.convtrain > $OUT/wgrad_convtrain.jsonl 2>$OUT/wgrad_convtrain.err || { tail -5 $OUT/wgrad_convtrain.err; exit 1; }
tail -1 $OUT/wgrad_convtrain.jsonl
run() {
  local name=$1; shift
  timeout -k 10 300 "$@" > "$OUT/wgrad_$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' "$OUT/wgrad_$name.log" | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
T="python bench.py --workload 1.2 --steps 20 --warmup 5 --no-cap-probe --pods 1 --gpucores 100 --gpumem 0"
for r in 1 2; do
  run nat_$r $T || exit 1
  VGPU_CONV_WGRAD=0 run mio_$r $T || exit 1
  VGPU_CONV_WGRAD=all run all_$r $T || exit 1
done
exit 0
