#!/bin/bash
# A/B of HIP runtime knobs on a launch-bound replayed training step (4.2,
# DeepLab-v3 b=1): each variant is its own pod process, 30 timed replays.
#   bash scripts/graph_env_ab.sh [workload] > gpurun_out/graph_env_ab.log
set -u
cd "$(dirname "$0")/.."
W=${1:-4.2}
run() {
  local tag=$1; shift
  local out
  out=$(env "$@" timeout -k 10 200 python3 -m vgpu.bench.pod --workload $W --steps 30 --warmup 5 --graph --no-wait 2>/dev/null | grep DONE)
  local rc=$?
  echo "$tag $out"
  return $rc
}
run base VGPU_AB=0 || exit 1
run devkernarg HIP_FORCE_DEV_KERNARG=1 || exit 1
run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
run pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
run batch8 DEBUG_HIP_GRAPH_BATCH_SIZE=8 || exit 1
run batch64 DEBUG_HIP_GRAPH_BATCH_SIZE=64 || exit 1
run wgrad_launch12 VGPU_WGRAD_LAUNCH_US=12 || exit 1
run wgrad_launch30 VGPU_WGRAD_LAUNCH_US=30 || exit 1
run dw_wgrad_v1 VGPU_DW_WGRAD=1 || exit 1
run base2 VGPU_AB=0 || exit 1
