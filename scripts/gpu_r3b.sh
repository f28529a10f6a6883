#!/bin/bash
# Round-3 GPU session B: cap tests (hipMallocAsync backend, RCCL under
# contention), then the 4 x 25 % suite under the temporal and the adaptive
# ("auto") share policies against exclusive.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r3b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_caps.py -x -v -s --timeout 600 --timeout-method thread \
  -p no:cacheprovider > $O/caps.log 2>&1
rc=$?; tail -8 $O/caps.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 2400 python -u -m vgpu.bench.suite --scenarios ${SCEN:-exclusive,vgpu-cu25-temporal,vgpu-cu25-auto} \
  --steps ${STEPS:-40} --warmup ${WARM:-10} --timeout 600 > $O/suite.log 2>&1 || exit $?
tail -16 $O/suite.log
exit 0
