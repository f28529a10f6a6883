#!/bin/bash
# Transparent virtual device memory on MI355X: the probe (diagnostics on
# stderr), the GPU test, then the Llama-3-8B neighbour-leaves A/B (pager vs
# zero-copy), with a shim trace of the migrations.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/vmem; mkdir -p $O/trace; export TMPDIR=/tmp
VGPU_DEVICE_MEMORY_LIMIT_0=400000m VGPU_OVERSUBSCRIBE=true VGPU_LOG_LEVEL=3 LD_PRELOAD="$PWD/vgpu/_lib/libvgpu.so ${LD_PRELOAD:-}" \
  timeout -k 10 120 python -u -m vgpu.bench.probes vmem 4 30 > $O/probe.log 2>&1
rc=$?; tail -5 $O/probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_shim.py -k vmem -x -v -s --timeout 280 --timeout-method thread \
  > $O/pytest_vmem.log 2>&1 || { tail -30 $O/pytest_vmem.log; exit 1; }
tail -3 $O/pytest_vmem.log
[ "${1:-}" = "probe" ] && exit 0
VGPU_TRACE=$PWD/$O/trace timeout -k 10 600 python -u -m vgpu.bench.vmem --part-c --leave-gib 8 --tokens 16 --windows 8 \
  > $O/part_c.log 2>&1 || { tail -30 $O/part_c.log; exit 1; }
grep VMEM_C_RUN $O/part_c.log | cut -c1-1500
