#!/bin/bash
# Each pod process owns 2 compute queues (the HIP queue + a small ROCr-internal
# one, not created through hsa_queue_create) and 1 SDMA queue.  Which ROCr
# setting removes the internal compute queue, and does 4 x 25 % speed up?
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/queues2
mkdir -p $O
try() {  # try <tag> [VAR=value]
  local tag=$1; shift
  ( sleep 13; for p in /sys/class/kfd/kfd/proc/*; do
      [ -d $p/queues ] || continue
      for q in $p/queues/*; do echo "$(basename $p) $(cat $q/gpuid 2>/dev/null) $(cat $q/type 2>/dev/null) $(cat $q/size 2>/dev/null)"; done
    done ) > $O/$tag.q 2>&1 &
  env "$@" timeout -k 10 300 python bench.py --no-cap-probe --pods 4 --gpucores 25 --gpumem 72000 --steps 1200 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; wait; return 0; }
  wait
  local v; v=$(grep '^{' $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_pod_images_s"])')
  echo "$tag $v | compute-queue sizes of GPU 17010 procs: $(awk '$2==17010 && $3==0 {print $4}' $O/$tag.q | sort | uniq -c | tr '\n' ' ')"
}
try base
try noreclaim HSA_NO_SCRATCH_RECLAIM=1
try noasync HSA_ENABLE_SCRATCH_ASYNC_RECLAIM=0
try nopcs HSA_DISABLE_PC_SAMPLING=1
try codma HSA_CO_DMACOPY_SIZE=1099511627776
try nosdma HSA_ENABLE_SDMA=0
