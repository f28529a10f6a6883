#!/bin/bash
# ai-benchmark suite refresh (subset of tests given as $1), 3 scenarios each.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -m vgpu.bench.suite --tests "$1" --steps 10 --warmup 3 --timeout 300 > gpurun_out/suite_$2.log 2>&1
rc=$?; grep -E "^SUITE|^\|" gpurun_out/suite_$2.log | tail -40; exit $rc
