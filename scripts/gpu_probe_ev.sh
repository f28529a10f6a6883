#!/bin/bash
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/evprobe; mkdir -p $O; export TMPDIR=/tmp; export PYTHONPATH=$PWD
timeout -k 10 120 python -u scripts/graph_event_probe.py > $O/plain.json 2> $O/plain.err || { tail -5 $O/plain.err; exit 1; }
cat $O/plain.json
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 scripts/graph_event_probe.py > $O/traced.json 2> $O/traced.err || { tail -5 $O/traced.err; exit 1; }
grep '^{' $O/traced.json
B="bench.py --pods 1 --gpucores 25 --cu-share temporal --core-policy force --steps 30 --warmup 10 --no-cap-probe"
timeout -k 10 200 python -u $B > $O/q_plain.json 2> $O/q_plain.err || { tail -5 $O/q_plain.err; exit 1; }
echo "plain: $(grep -o '"value": [0-9.]*' $O/q_plain.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/qtrace/%pid% -o run -- python3 $B > $O/q_traced.json 2> $O/q_traced.err || { tail -5 $O/q_traced.err; exit 1; }
echo "traced: $(grep -o '"value": [0-9.]*' $O/q_traced.json)"
