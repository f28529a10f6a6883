#!/bin/bash
# Shim event trace of a lone 25 % temporal pod and a 99 % pod: per-marker GPU busy
# intervals (gpu_time events) and throttle waits.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/t25trace; rm -rf $O; mkdir -p $O/t25 $O/t99; export TMPDIR=/tmp
VGPU_TRACE=$PWD/$O/t25 timeout -k 10 300 python bench.py --no-cap-probe --steps 150 --pods 1 --gpucores 25 --cu-share temporal > $O/t25.log 2>&1 || exit 1
VGPU_TRACE=$PWD/$O/t99 timeout -k 10 300 python bench.py --no-cap-probe --steps 150 --pods 1 --gpucores 99 --cu-share temporal > $O/t99.log 2>&1 || exit 1
grep -h '^{' $O/t25.log $O/t99.log | cut -c1-100
ls -la $O/t25 $O/t99
