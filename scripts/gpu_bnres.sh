#!/bin/bash
# BN fused-shortcut-gradient tests + training A/B (counters + fused add vs before).
set -u
cd "$(dirname "$0")/.."; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/bnres_pytest.log 2>&1
rc=$?; tail -6 gpurun_out/bnres_pytest.log; [ $rc -eq 0 ] || exit $rc
for w in 1.2 2.2; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cap-probe --pods 1 --gpucores 100 --gpumem 0 > gpurun_out/bnres_$w.log 2>&1 || exit 1
  echo "$w $(grep '^{' gpurun_out/bnres_$w.log | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])")"
done
exit 0
