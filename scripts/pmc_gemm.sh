#!/bin/bash
# PMC passes over the 256x256-tile GEMM probe (scripts/gemm_probe.py).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONPATH=$PWD
OUT=gpurun_out/pmc_gemm; rm -rf $OUT; mkdir -p $OUT
MODE=${1:-1}
P="python3 scripts/gemm_probe.py $MODE 65536 1024 1024 10"
timeout -k 10 120 $P > $OUT/plain.log 2>&1; cat $OUT/plain.log | grep GEMM
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $P > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("gpurun_out/pmc_gemm/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "conv" not in r.get("Kernel_Name", ""):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:.4g}  (per dispatch {tot[k] / max(n[k], 1):.4g})")
g = tot.get("GRBM_GUI_ACTIVE", 0) / max(n["GRBM_GUI_ACTIVE"], 1)
if g:
    per = lambda c: tot.get(c, 0) / max(n[c], 1)
    print("MFMA busy", per("SQ_VALU_MFMA_BUSY_CYCLES") / (4 * 256 * g / 8) if g else None)
    wc = per("SQ_WAVE_CYCLES")
    print("wait_any/wave", per("SQ_WAIT_ANY") / wc, "wait_inst_any/wave", per("SQ_WAIT_INST_ANY") / wc,
          "active/wave", per("SQ_ACTIVE_INST_ANY") / wc)
PY
