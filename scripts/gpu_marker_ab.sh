#!/bin/bash
# Does the limiter's per-launch marker event cost throughput? exclusive vs a 99 % temporal pod.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/marker; mkdir -p $O; export TMPDIR=/tmp
one() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cap-probe --steps 150 "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; return 1; }
  grep '^{' $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["per_pod_images_s"])' $tag
}
one excl --pods 1 --gpucores 100 --gpumem 0 || exit 1
one t99 --pods 1 --gpucores 99 --cu-share temporal || exit 1
VGPU_LIMITER_QUANTUM_MS=20 one t25q20 --pods 1 --gpucores 25 --cu-share temporal || exit 1
one excl_nograph --pods 1 --gpucores 100 --gpumem 0 --no-graph || exit 1
one t99_nograph --pods 1 --gpucores 99 --cu-share temporal --no-graph || exit 1
