#!/bin/bash
# Round-3 GPU session E: conv numerics, in-process A/B against the round-start
# conv build (vgpu/_lib/libvgpu_conv_ab.so), then the headline bench.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r3e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fused.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/conv_tests.log 2>&1
rc=$?; tail -3 $O/conv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m vgpu.bench.convab --other vgpu/_lib/libvgpu_conv_ab.so > $O/convab.log 2>&1
rc=$?; cat $O/convab.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
