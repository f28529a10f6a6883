#!/bin/bash
# Round-3 GPU session D: conv numerics, in-process A/B of the conv23 tail
# pipeline against the previous build (vgpu/_lib/libvgpu_conv_ab.so), the GPU
# test tier, then the headline bench.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r3d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/conv_tests.log 2>&1
rc=$?; tail -3 $O/conv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m vgpu.bench.convab --other vgpu/_lib/libvgpu_conv_ab.so > $O/convab.log 2>&1
rc=$?; grep -E "tail|total" $O/convab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
