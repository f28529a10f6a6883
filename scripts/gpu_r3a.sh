#!/bin/bash
# Round-3 GPU session A: new GPU tests (caps, RCCL under contention, weighted
# shares), the vmem model switch with its migration trace, then the flagship.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r3a
export TMPDIR=/tmp
O=gpurun_out/r3a
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))"
  tail -n 5 "$O/$name.log" | cut -c1-400
  return $rc
}
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
run caps 900 python -u -m pytest tests/test_gpu_caps.py -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider
rc=$?; ok_or_testfail $rc || exit $rc
run weighted 600 python -u -m pytest tests/test_gpu_temporal.py -x -v -s -k weighted --timeout 500 --timeout-method thread -p no:cacheprovider
rc=$?; ok_or_testfail $rc || exit $rc
mkdir -p $O/trace
run part_d 900 env VGPU_TRACE=$O/trace VGPU_VMEM_LOG_DIR=$O python -u -m vgpu.bench.vmem --part-d --budget-gib 22 --tokens 16 --windows 6 || exit $?
python -m vgpu.monitor.trace $O/trace/part_d > $O/trace_summary_d.json 2>&1
run bench 600 python bench.py || exit $?
exit 0
