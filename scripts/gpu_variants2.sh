#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out
run() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" python bench.py "$@" > "$OUT/v_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep '^{' "$OUT/v_$name.log" | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['per_pod_images_s'])"
  return $rc
}
python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || exit 1
run p1_m50_graph 600 --pods 1 --gpucores 50 --steps 30 --warmup 5 --no-cap-probe || exit 1
run p1_m50_nograph 600 --pods 1 --gpucores 50 --steps 30 --warmup 5 --no-cap-probe --no-graph || exit 1
run p1_excl_nograph 600 --pods 1 --no-shim --gpucores 100 --gpumem 0 --steps 30 --warmup 5 --no-cap-probe --no-graph || exit 1
run p1_shim100_graph 600 --pods 1 --gpucores 100 --steps 30 --warmup 5 --no-cap-probe || exit 1
run p2_nomask_nograph 600 --pods 2 --no-shim --steps 30 --warmup 5 --no-cap-probe --no-graph || exit 1
run p4_m25_nograph 600 --pods 4 --gpucores 25 --gpumem 70000 --steps 30 --warmup 5 --no-cap-probe --no-graph || exit 1
run p4_nomask_nograph 600 --pods 4 --no-shim --gpucores 25 --gpumem 70000 --steps 30 --warmup 5 --no-cap-probe --no-graph || exit 1
for cfg in graph nograph; do
  extra=""; [ $cfg = nograph ] && extra="--no-graph"
  echo "=== rocprof $cfg ($(date +%T))"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_p1_$cfg/%pid% -o run -- python3 bench.py --pods 1 --gpucores 50 --steps 10 --warmup 3 --no-cap-probe $extra > $OUT/prof_p1_$cfg.log 2>&1
  echo "=== rocprof rc=$?"
done
exit 0
