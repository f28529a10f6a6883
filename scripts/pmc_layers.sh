#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over selected conv layers.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
L=${1:-s1b1.conv3,s3b1.conv3,s3b2.conv2,s3b2.conv1}
OUT=gpurun_out/pmc
rm -rf $OUT; mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 scripts/convnative.py --only "$L" --no-miopen --iters 3 > $OUT/p$i.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
exit 0
