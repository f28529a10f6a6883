#!/bin/bash
# Flagship (2 pods x 50 %, ResNet-V2-50 b=50 inference): share policy A/B, alternated.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/flag; mkdir -p $O; export TMPDIR=/tmp
one() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; return 1; }
  grep '^{' $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["per_pod_images_s"], d["vram_cap"][0]["accuracy"] if d["vram_cap"] else None)' $tag
}
for i in 1 2; do
  one hybrid$i || exit 1
  one temporal$i --cu-share temporal || exit 1
done
one temporal_long --cu-share temporal --steps 200 || exit 1
one hybrid_long --steps 200 || exit 1
