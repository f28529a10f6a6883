#!/bin/bash
# Temporal limiter on the flagship: lone 25 % / 50 % pods vs exclusive (120 steps).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/t25; mkdir -p $O; export TMPDIR=/tmp
one() {  # one <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cap-probe --steps 150 "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; return 1; }
  grep '^{' $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["per_pod_images_s"])' $tag
}
one excl --pods 1 --gpucores 100 --gpumem 0 || exit 1
VGPU_LOG_LEVEL=4 one t25 --pods 1 --gpucores 25 --cu-share temporal || exit 1
grep "limiter dev" $O/t25.log | tail -4
one t50 --pods 1 --gpucores 50 --cu-share temporal || exit 1
one t4x25 --pods 4 --gpucores 25 --gpumem 72000 --cu-share temporal || exit 1
