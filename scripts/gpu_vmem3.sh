#!/bin/bash
# Virtual device memory v3 on one MI355X: shim GPU tests, then the model-switch
# (part D) and hot-set-beyond-budget (part E) Llama-3-8B graph-decode runs.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/vmem3
export TMPDIR=/tmp VGPU_VMEM_LOG_DIR=gpurun_out/vmem3 VGPU_LOG_LEVEL=${VGPU_LOG_LEVEL:-4}
STAGES=${1:-tests,d,e}
for s in ${STAGES//,/ }; do
  case $s in
    tests) timeout -k 10 600 python -u -m pytest tests/test_gpu_shim.py -x -v --timeout 300 --timeout-method thread \
             -p no:cacheprovider -k "vmem or oversub or spill" > gpurun_out/vmem3/pytest.log 2>&1
           rc=$?; tail -5 gpurun_out/vmem3/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc ;;
    d) VGPU_TRACE=gpurun_out/vmem3/trace timeout -k 10 900 python -u -m vgpu.bench.vmem --part-d \
         --budget-gib ${BUDGET_D:-22} --tokens 16 --windows ${WIN:-6} > gpurun_out/vmem3/part_d.log 2>&1 || exit $?
       python -m vgpu.monitor.trace gpurun_out/vmem3/trace/part_d > gpurun_out/vmem3/trace_summary_d.json 2>&1
       tail -c 3000 gpurun_out/vmem3/part_d.log ;;
    caps) timeout -k 10 900 python -u -m pytest tests/test_gpu_caps.py tests/test_gpu_shim.py -x -v --timeout 600 \
            --timeout-method thread -p no:cacheprovider > gpurun_out/vmem3/pytest_caps.log 2>&1
          rc=$?; tail -8 gpurun_out/vmem3/pytest_caps.log; [ $rc -eq 0 ] || exit $rc ;;
    e) timeout -k 10 600 python -u -m vgpu.bench.vmem --part-e --budget-gib ${BUDGET_E:-11.5} --tokens 16 \
         --windows 4 > gpurun_out/vmem3/part_e.log 2>&1 || exit $?
       tail -c 2000 gpurun_out/vmem3/part_e.log ;;
  esac
done
exit 0
