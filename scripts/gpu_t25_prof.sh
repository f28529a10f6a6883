#!/bin/bash
# Kernel trace of a lone 25 % temporal pod (per-kernel durations under the limiter).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/t25prof; mkdir -p $O; export TMPDIR=/tmp
VGPU_LOG_LEVEL=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t25/%pid% -o run -- python3 bench.py --no-cap-probe --steps 60 --pods 1 --gpucores 25 --cu-share temporal > $O/t25.log 2>&1 || exit 1
grep -h '^{' $O/t25.log | cut -c1-120
grep -c "limiter dev" $O/t25.log; grep "limiter dev\|board\|capture" $O/t25.log | tail -5
