#!/bin/bash
# Why do 4 x 25 % pods lose to the exclusive GPU?  Same-box comparisons:
# 2 x 25 % (masks, half the GPU idle), 3 x 33 %, 4 pods unmasked (time-shared
# CUs), 4 x 25 % with the runtime's default HW queues, 4 x 25 % baseline.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/p4diag
mkdir -p $O
run() {  # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cap-probe "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  echo "$tag $(grep '^{' $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["per_pod_images_s"])')"
}
run p4_m25      --pods 4 --gpucores 25 --gpumem 72000
run p2_m25      --pods 2 --gpucores 25 --gpumem 72000
run p3_m33      --pods 3 --gpucores 33 --gpumem 96000
run p4_nomask   --pods 4 --gpucores 100 --gpumem 72000
run p4_m25_q0   --pods 4 --gpucores 25 --gpumem 72000 --hw-queues 0
run p4_m25_nog  --pods 4 --gpucores 25 --gpumem 72000 --no-graph
run p1_m25      --pods 1 --gpucores 25 --gpumem 72000
