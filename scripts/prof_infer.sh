#!/bin/bash
# Kernel trace of one inference pod (ai-benchmark test $1, exclusive GPU, hipGraph step).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof_infer_${1/./_}
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 -m vgpu.bench.pod --workload $1 --steps 6 --warmup 3 --graph --no-wait > $OUT/log 2>&1
rc=$?; tail -1 $OUT/log; exit $rc
