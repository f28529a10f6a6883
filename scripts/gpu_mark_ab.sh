#!/bin/bash
# Limiter marker density A/B on 4 x 25 % temporal pods: marker per launch vs every 500 us.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/markab; mkdir -p $O; export TMPDIR=/tmp
one() {  # one <tag> <workload> [env...]
  local tag=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --no-cap-probe --steps 40 --warmup 5 --workload $w --pods 4 --gpucores 25 --gpumem 70000 --cu-share temporal > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; return 1; }
  grep '^{' $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["per_pod_images_s"])' $tag
}
for w in 1.1 2.2; do
  one w${w}_m0 $w VGPU_LIMITER_MARK_US=0 || exit 1
  one w${w}_m500 $w VGPU_LIMITER_MARK_US=500 || exit 1
  one w${w}_m5000 $w VGPU_LIMITER_MARK_US=5000 || exit 1
done
