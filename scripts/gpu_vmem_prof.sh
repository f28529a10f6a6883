#!/bin/bash
# Kernel trace of one VGG-16 pod under the vgpu-vmem knobs: managed-by-default
# ranges vs plain allocations (is the cost on the GPU or between launches?).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/vmem_prof
mkdir -p $O
export TMPDIR=/tmp
A="--workload ${T:-3.2} --pods 1 --gpucores 0 --gpumem 230000 --oversubscribe --memory-scaling 1.8 --steps 30 --warmup 10 --no-cap-probe"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/default/%pid%" -o run -- python3 bench.py $A > $O/default.log 2>&1 || exit 1
VGPU_VMEM_MANAGED_MIN_MB=-1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/plain/%pid%" -o run -- python3 bench.py $A > $O/plain.log 2>&1 || exit 1
python3 scripts/prof_summary.py $O/default > $O/default_summary.txt 2>&1
python3 scripts/prof_summary.py $O/plain > $O/plain_summary.txt 2>&1
grep '^{' $O/default.log $O/plain.log
