#!/bin/bash
# 4 x 25 % pods: unenforced time sharing (no shim) vs the temporal limiter, its
# dry-run (markers + charging, no waiting) and sparse markers.
#   WL="4.2 1.1" bash scripts/gpu_weak_ab.sh
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/weak; mkdir -p $O; export TMPDIR=/tmp
one() {  # one <tag> <workload> <bench args...>
  local tag=$1 w=$2; shift 2
  timeout -k 10 300 python bench.py --no-cap-probe --steps 40 --warmup 5 --workload $w --pods 4 --gpucores 25 --gpumem 70000 "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; return 1; }
  grep '^{' $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["per_pod_images_s"])' $tag
}
for w in ${WL:-4.2 1.1}; do
  one w${w}_noshim $w --no-shim || exit 1
  one w${w}_temporal $w --cu-share temporal || exit 1
  VGPU_LIMITER_DRYRUN=1 one w${w}_dryrun $w --cu-share temporal || exit 1
  VGPU_LIMITER_MARK_US=100 one w${w}_sparse100 $w --cu-share temporal || exit 1
done
