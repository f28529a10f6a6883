#!/bin/bash
# One VGG-16 training pod under the vgpu-vmem knobs with the shim's INFO log:
# which managed ranges are promoted / demoted, and when.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/vmem_log
mkdir -p $O
export TMPDIR=/tmp
A="--workload ${T:-3.2} --pods 1 --gpucores 0 --gpumem 230000 --oversubscribe --memory-scaling 1.8 --steps 30 --warmup 10 --no-cap-probe"
VGPU_LOG_LEVEL=4 timeout -k 10 300 python3 bench.py $A > $O/out.log 2> $O/err.log || exit 1
grep -c "vmem:" $O/err.log; grep "vmem:" $O/err.log | head -60; grep '^{' $O/out.log | cut -c1-200
