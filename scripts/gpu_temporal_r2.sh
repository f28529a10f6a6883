#!/bin/bash
# Temporal (GPU-time token bucket + fair-share board) vs exclusive on one MI355X.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/temporal
mkdir -p $O
export TMPDIR=/tmp
run() {  # run <tag> <secs> <bench args...>
  local tag=$1 secs=$2; shift 2
  timeout -k 10 $secs python bench.py --no-cap-probe "$@" > $O/$tag.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; tail -5 $O/$tag.log; return $rc; fi
  grep '^{' $O/$tag.log | tail -1 > $O/$tag.json
  python - "$tag" "$O/$tag.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(sys.argv[1], d["value"], d["per_pod_images_s"], d["config"]["enforcement"])
PY
}
timeout -k 10 120 env LD_PRELOAD=$PWD/vgpu/_lib/libvgpu.so VGPU_DEVICE_MEMORY_LIMIT_0=8g VGPU_LOG_LEVEL=3 python scripts/hostpid_probe.py > $O/hostpid.log 2>&1; echo "hostpid rc=$?"; tail -3 $O/hostpid.log
run excl 300 --pods 1 --gpucores 100 --gpumem 0 || exit 1
run t1x25 400 --pods 1 --gpucores 25 --cu-share temporal || exit 1
run t1x50 400 --pods 1 --gpucores 50 --cu-share temporal || exit 1
run t2x50 400 --pods 2 --gpucores 50 --cu-share temporal || exit 1
run t4x25 400 --pods 4 --gpucores 25 --gpumem 72000 --cu-share temporal || exit 1
run m4x25 400 --pods 4 --gpucores 25 --gpumem 72000 --cu-share mask || exit 1
