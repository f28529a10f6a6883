#!/bin/bash
# what chaining a graph into one line (the shim's workaround for
# multi-branch graphs under GPU_MAX_HW_QUEUES=1) costs on a branchy graph -- the
# N=1 DDP pod, whose whole step (backward with the bucketed all-reduce on a side
# stream, SGD) is one hipGraph -- at 1 and at 4 HW queues, under the shim and
# without it.
#   [BUCKET=4] bash scripts/chain_graph_ab.sh > gpurun_out/chain_graph_ab.log
# (BUCKET=4: ~25 buckets, each all-reduce a side-stream branch of the graph
# overlapping the rest of the backward)
set -u
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD
SHIM=$(python3 -c "from vgpu.native import shim_path; print(shim_path())")
BUCKET=${BUCKET:-64}
run() {
  local tag=$1 q=$2 pre=$3; shift 3
  local port=$((29500 + RANDOM % 2000))
  local out
  out=$(env GPU_MAX_HW_QUEUES=$q ${pre:+LD_PRELOAD=$pre} VGPU_DEVICE_MEMORY_LIMIT_0=64g "$@" \
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 \
    --master-port=$port -m vgpu.parallel.ddp --workload 1.2 --steps 60 --warmup 5 --batch 16 --size 160 --bucket-mb $BUCKET 2>/dev/null \
    | grep '^{' | tail -1)
  local rc=$?
  echo "$tag $out"
  return $rc
}
run shim_q1 1 "$SHIM" || exit 1
run shim_q4 4 "$SHIM" || exit 1
run noshim_q1 1 "" || exit 1
run noshim_q4 4 "" || exit 1
run shim_q1_again 1 "$SHIM" || exit 1
