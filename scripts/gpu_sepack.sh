#!/bin/bash
# A/B: CU masks spread over every shader engine (default) vs packed onto whole
# shader engines (VGPU_CU_PACK=se).  Census of one 25 % mask of each kind, then
# interleaved flagship runs at 2 x 50 % and 4 x 25 %.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sepack
O=gpurun_out/sepack
census() {  # census <pack>
  local m
  m=$(python -c "from vgpu.device.cualloc import *; print(hex(alloc_cu_mask(0, 25, MI355X, '$1')))")
  VGPU_CU_MASK_0=$m timeout -k 10 120 python -c "
import json, os, subprocess, sys
from vgpu.native import preload_env
env = preload_env(dict(os.environ))
r = subprocess.run([sys.executable, '-m', 'vgpu.bench.probes', 'census', '4096', '200000'], env=env,
                   capture_output=True, text=True, timeout=100)
print([l for l in r.stdout.splitlines() if l.startswith('PROBE')][-1])
" > $O/census_$1.log 2>&1 || return 1
  echo "census $1: $(cut -c1-400 $O/census_$1.log)"
}
census spread && census se || exit 1
for rep in 1 2; do
  for cfg in "2 50 144000" "4 25 72000"; do
    set -- $cfg
    for pack in spread se; do
      tag=p$1_${pack}_$rep
      VGPU_CU_PACK=$pack timeout -k 10 300 python bench.py --pods $1 --gpucores $2 --gpumem $3 --no-cap-probe \
        > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
      echo "$tag $(grep '^{' $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["per_pod_images_s"])')"
    done
  done
done
