#!/bin/bash
# Round-3 GPU session J: GPU test tier on the final kernels, then the PMC
# passes + kernel trace of the exclusive flagship forward.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r3j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_flagship.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_flagship --last 88 > $O/pmc_summary.md 2>&1; tail -25 $O/pmc_summary.md
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
