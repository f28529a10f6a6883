#!/bin/bash
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/evprobe2; mkdir -p $O; export TMPDIR=/tmp; export PYTHONPATH=$PWD
export VGPU_LOG_LEVEL=${VGPU_LOG_LEVEL:-4}
B="bench.py --pods 1 --gpucores 25 --cu-share temporal --core-policy force --seconds 4 --warmup 10 --no-cap-probe ${EXTRA:-}"
timeout -k 10 200 python3 -u $B > $O/q_plain.json 2> $O/q_plain.err || { tail -5 $O/q_plain.err; exit 1; }
echo "plain: $(grep -o '"value": [0-9.]*' $O/q_plain.json)"; grep "limiter dev" $O/q_plain.err | tail -8
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/qtrace/%pid% -o run -- python3 $B > $O/q_traced.json 2> $O/q_traced.err || { tail -5 $O/q_traced.err; exit 1; }
echo "traced: $(grep -o '"value": [0-9.]*' $O/q_traced.json)"; grep "limiter dev" $O/q_traced.err | tail -8
grep -i "vgpu.*\(warn\|err\|board\|pool\|limiter\)" $O/q_traced.err | grep -v "limiter dev" | head -12
