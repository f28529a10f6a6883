#!/bin/bash
# ai-benchmark suite, 4 x 25 % under the share policies vs exclusive.
#   bash scripts/gpu_suite_r2.sh [scenarios] [tests]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
SC=${1:-exclusive,vgpu-cu25,vgpu-cu25-temporal,vgpu-cu25-mask}
T=${2:-}
timeout -k 10 1100 python -u -m vgpu.bench.suite --steps 40 --warmup 5 --timeout 300 --scenarios $SC ${T:+--tests $T} \
  > gpurun_out/suite_r2.log 2>&1
rc=$?
tail -16 gpurun_out/suite_r2.log
exit $rc
