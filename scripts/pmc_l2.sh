#!/bin/bash
# L2 traffic of the flagship forward per kernel family: one rocprofv3 PMC pass
# (TCC requests / hits / misses, one TCC block budget) next to a kernel trace.
#   bash scripts/pmc_l2.sh && python3 scripts/pmc_l2.py gpurun_out/pmc_l2
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_l2
rm -rf $OUT; mkdir -p $OUT
POD="python3 -m vgpu.bench.pod --workload 1.1 --steps 2 --warmup 1 --no-wait"
timeout -s KILL 180 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/p1 -o run -- $POD > $OUT/p1.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p1.log; exit $rc; }
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- $POD > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
