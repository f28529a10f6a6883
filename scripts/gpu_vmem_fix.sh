#!/bin/bash
# After the host-copy fix: the shim's GPU tests, then the vgpu-vmem column of
# the suite (2 pods, cap 230000 MiB, memory scaling 1.8, managed by default).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/vmem_fix
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_shim.py -x -q --timeout 120 --timeout-method thread > $O/pytest_shim.log 2>&1 || { tail -30 $O/pytest_shim.log; exit 1; }
tail -2 $O/pytest_shim.log
timeout -k 10 900 python -u -m vgpu.bench.suite --scenarios vgpu-vmem --steps 40 --warmup 10 --timeout 150 > $O/suite_vmem.log 2>&1 || exit $?
grep SUITE $O/suite_vmem.log | cut -c1-160
