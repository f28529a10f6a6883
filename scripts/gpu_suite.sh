#!/bin/bash
# The ai-benchmark suite on one MI355X: SCEN scenarios (default: exclusive and
# 4 x 25 % under the device plugin's default share policy), STEPS timed steps.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash scripts/gpu_suite.sh'
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/suite
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m vgpu.bench.suite --scenarios ${SCEN:-exclusive,vgpu-cu25} \
  --steps ${STEPS:-40} --warmup ${WARM:-10} --timeout 300 > $O/${NAME:-suite}.log 2>&1 || exit $?
tail -14 $O/${NAME:-suite}.log
