#!/bin/bash
# Round-3 GPU session C: GPU test tier, then the headline bench (default auto
# share policy) on the rebuilt tree.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r3c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
