#!/bin/bash
# One GPU-box session: GPU tests, smoke, flagship bench, per-layer conv bench and a
# rocprofv3 kernel trace of the flagship.  Every GPU step has its own time limit;
# the script stops at the first fault/abort/timeout.  .so files are built here
# (CPU container) and travel with the tree.
#
#   bash scripts/gpu_session.sh tests,smoke,bench,conv,prof     (default)
# stages: tests smoke bench excl conv halo prof pmc shim suite vmem limiter-prof ddp1
# (A/B comparisons of bench.py flags and env knobs: scripts/bench_ab.py recipes;
# results worth keeping are copied into profiles/.)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))"
  tail -n ${TAILN:-6} "$OUT/$name.log" | cut -c1-600
  return $rc
}
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
n=0
# Stages are comma-separated; an argument containing newlines is split on
# newlines instead (custom commands that need commas of their own).
if [[ "${1:-}" == *$'\n'* ]]; then
  mapfile -t STAGES <<< "$1"
else
  IFS=, read -ra STAGES <<< "${1:-tests,smoke,bench,conv,prof}"
fi
for s in "${STAGES[@]}"; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
           rc=$?; ok_or_testfail $rc || exit $rc ;;
    smoke) step smoke 600 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench) step bench 900 python bench.py || exit 1
           grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json" ;;
    excl)  step bench_excl 600 python bench.py --pods 1 --gpucores 100 --gpumem 0 --no-cap-probe || exit 1 ;;
    conv)  step convnative 600 python scripts/convnative.py || exit 1 ;;
    prof)  step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_native/%pid%" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cap-probe || exit 1 ;;
    shim) step pytest_shim 900 python -u -m pytest tests/test_gpu_shim.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider
          rc=$?; ok_or_testfail $rc || exit $rc ;;
    halo) step convknob_halo 300 python scripts/convknob.py --knob halo --extra || exit 1 ;;
    pmc)  step pmc 900 bash scripts/pmc_flagship.sh || exit 1
          step pmc_summary 60 python scripts/pmc_summary.py gpurun_out/pmc_flagship --last 88 || exit 1 ;;
    suite) step suite 2400 python -u -m vgpu.bench.suite --scenarios "${SCEN:-exclusive,vgpu,vgpu-cu25}" \
             --steps "${STEPS:-20}" --warmup "${WARM:-5}" --timeout 600 || exit 1 ;;
    vmem) step pytest_vmem 600 python -u -m pytest tests/test_gpu_shim.py -x -v --timeout 300 --timeout-method thread \
            -p no:cacheprovider -k "vmem or oversub or spill or suspend"
          rc=$?; ok_or_testfail $rc || exit $rc
          step vmem_bench 900 python -u -m vgpu.bench.vmem || exit 1 ;;
    # the temporal limiter of a lone 25 % pod, plain and under rocprofv3 (isolation check)
    limiter-prof) B="bench.py --pods 1 --gpucores 25 --cu-share temporal --core-policy force --seconds 4 --warmup 10 --no-cap-probe"
          step limiter_plain 300 python3 -u $B || exit 1
          step limiter_traced 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/limiter_trace/%pid%" -o run -- python3 $B || exit 1 ;;
    ddp1) step ddp1 900 python -u bench.py --pod-gpus 1 --steps 10 --warmup 3 || exit 1 ;;
    *) n=$((n+1)); step "cmd$n" 900 bash -c "$s" || exit 1 ;;
  esac
done
exit 0
