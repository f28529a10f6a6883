#!/bin/bash
# VGG-16 under the vgpu-vmem scenario: managed-by-default ranges (default) vs
# plain hipMalloc until the budget is exceeded (VGPU_VMEM_MANAGED_MIN_MB=-1).
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash scripts/gpu_vmem_ab.sh'
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/vmem_ab
mkdir -p $O
export TMPDIR=/tmp
VGPU_SUITE_LOGDIR=$O/default timeout -k 10 400 python -u -m vgpu.bench.suite --tests ${TESTS:-3.1,3.2} \
  --scenarios vgpu-vmem --steps 40 --warmup 10 --timeout 150 > $O/default.log 2>&1 || exit $?
VGPU_VMEM_MANAGED_MIN_MB=-1 VGPU_SUITE_LOGDIR=$O/plain timeout -k 10 400 python -u -m vgpu.bench.suite \
  --tests ${TESTS:-3.1,3.2} --scenarios vgpu-vmem --steps 40 --warmup 10 --timeout 150 > $O/plain.log 2>&1 || exit $?
grep SUITE $O/default.log $O/plain.log
