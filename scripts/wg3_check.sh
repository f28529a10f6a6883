#!/bin/bash
# Weight-gradient numerics only (quick GPU check).
cd "$(dirname "$0")/.."; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad" > gpurun_out/wg3.log 2>&1; rc=$?
tail -15 gpurun_out/wg3.log; exit $rc
