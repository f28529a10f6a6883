#!/bin/bash
# Round-3 GPU session G: conv numerics (incl. the fused stem + pool), stem A/B,
# headline bench.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r3g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q -k stem --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/conv_tests.log 2>&1
rc=$?; tail -3 $O/conv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 env PYTHONPATH=. python -u scripts/stem_ab.py > $O/stem_ab.json 2>$O/stem_ab.err; rc=$?; cat $O/stem_ab.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
