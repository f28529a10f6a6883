#!/bin/bash
# A/B of compute-share enforcement with 4 x 25 % pods (and 3 x 33 %): one mask
# per pod, temporal token bucket only, masks shared by pod pairs.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/cushare
mkdir -p $O
run() {  # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cap-probe "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  echo "$tag $(grep '^{' $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["per_pod_images_s"])')"
}
for rep in 1 2; do
  run p4_mask_$rep     --pods 4 --gpucores 25 --gpumem 72000
  run p4_temporal_$rep --pods 4 --gpucores 25 --gpumem 72000 --cu-share temporal
  run p4_group2_$rep   --pods 4 --gpucores 25 --gpumem 72000 --cu-share group2
  run p4_group2i_$rep  --pods 4 --gpucores 25 --gpumem 72000 --cu-share group2i
done
run p3_temporal --pods 3 --gpucores 33 --gpumem 96000 --cu-share temporal
run p2_temporal --pods 2 --gpucores 50 --gpumem 144000 --cu-share temporal
run p4_train_mask --pods 4 --gpucores 25 --gpumem 72000 --workload 1.2 --steps 10 --warmup 3
run p4_train_temporal --pods 4 --gpucores 25 --gpumem 72000 --workload 1.2 --steps 10 --warmup 3 --cu-share temporal
