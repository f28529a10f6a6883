#!/bin/bash
# Round-2 conv/GEMM check: big-tile numerics, GEMM ceiling table (hipBLASLt vs
# native 128x128 vs 256x256), flagship bench, and a rocprofv3 kernel-trace of
# the flagship for profiles/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/conv_r2; rm -rf $O; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_conv.py -k "big_tile or matches_fp32" -x -q --timeout 150 \
  --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/gemm_ceiling.py > $O/gemm_ceiling.jsonl 2>&1 || { tail -5 $O/gemm_ceiling.jsonl; exit 1; }
grep '^{' $O/gemm_ceiling.jsonl | cut -c1-260
for i in 1 2; do
  timeout -k 10 240 python bench.py > $O/bench$i.log 2>&1 || { tail -5 $O/bench$i.log; exit 1; }
  grep '^{' $O/bench$i.log | cut -c1-160
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/%pid% -o run -- python3 bench.py --steps 20 --warmup 5 --no-cap-probe > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 scripts/prof_summary.py $O/prof > $O/prof_summary.md 2>&1; head -30 $O/prof_summary.md
