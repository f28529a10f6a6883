#!/bin/bash
# Does the temporal limiter (no CU mask) hold a lone pod to its share?
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/temporal
mkdir -p $O
ls /sys/class/kfd/kfd/proc/ > $O/kfd_proc.txt 2>&1
run() {  # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cap-probe "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  echo "$tag $(grep '^{' $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["per_pod_images_s"])')"
}
run p1_excl --pods 1 --gpucores 100 --gpumem 0
run p1_t50 --pods 1 --gpucores 50 --gpumem 144000 --cu-share temporal --steps 100
run p1_t25 --pods 1 --gpucores 25 --gpumem 72000 --cu-share temporal --steps 100
run p1_m25 --pods 1 --gpucores 25 --gpumem 72000 --steps 100
timeout -k 10 300 python - <<'PY' > $O/busy.log 2>&1 || { tail -5 $O/busy.log; exit 1; }
import json, os, subprocess, sys
from vgpu.native import preload_env
def probe(env_extra, preload=True):
    env = dict(os.environ)
    if preload:
        env = preload_env(env)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-m", "vgpu.bench.probes", "busy", "16384", "4000", "40"], env=env,
                       capture_output=True, text=True, timeout=200)
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("PROBE ")][-1][6:])
full = probe({}, preload=False)
print("full", full)
for pct in (50, 25):
    r = probe({"VGPU_DEVICE_CU_LIMIT_0": str(pct), "VGPU_CU_MASK_FROM_LIMIT": "false"})
    print(pct, r, "ratio", r["median_s"] / full["median_s"])
PY
cat $O/busy.log
