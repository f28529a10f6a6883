#!/bin/bash
# Full GPU pass: tests, smoke, flagship bench, ai-benchmark suite, virtual memory.
set -u
cd "$(dirname "$0")/.."
bash scripts/gpu_session.sh tests,smoke,bench || exit $?
bash scripts/gpu_session.sh "python -m vgpu.bench.suite --steps 10 --warmup 3 --timeout 600 > gpurun_out/suite.log 2>&1" || exit $?
bash scripts/gpu_session.sh "python -m vgpu.bench.vmem --spill-gib 8 --budget-gib 8 --tokens 16 > gpurun_out/vmem.log 2>&1" || exit $?
exit 0
