#!/bin/bash
# Temporal limiter (open-loop workgroup-rate share) on MI355X: lone pods at
# 25 % / 50 %, then 4 x 25 % and 2 x 50 % sharing, against CU masks.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/temporal2
mkdir -p $O
run() {  # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cap-probe "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  echo "$tag $(grep '^{' $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["per_pod_images_s"])')"
}
run p1_excl --pods 1 --gpucores 100 --gpumem 0 --steps 400
run p1_t25_long --pods 1 --gpucores 25 --gpumem 72000 --cu-share temporal --steps 2000 --warmup 20
run p1_t50 --pods 1 --gpucores 50 --gpumem 144000 --cu-share temporal --steps 800
run p1_t25 --pods 1 --gpucores 25 --gpumem 72000 --cu-share temporal --steps 500
run p4_t25 --pods 4 --gpucores 25 --gpumem 72000 --cu-share temporal --steps 300

run p2_t50 --pods 2 --gpucores 50 --gpumem 144000 --cu-share temporal --steps 600

