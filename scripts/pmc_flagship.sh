#!/bin/bash
# PMC passes over the flagship forward (ResNet-V2-50 b=50 346², native convs,
# one exclusive pod, eager so every dispatch is its own row), one rocprofv3 run
# per counter group, plus a kernel-trace run for per-dispatch time.  Summary:
#   python scripts/pmc_summary.py gpurun_out/pmc_flagship
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_flagship
rm -rf $OUT; mkdir -p $OUT
POD="python3 -m vgpu.bench.pod --workload 1.1 --steps 2 --warmup 1 --no-wait"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $POD > $OUT/p$i.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
echo "=== trace"
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- $POD > $OUT/trace.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/trace.log; exit $rc; }
exit 0
