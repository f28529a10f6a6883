#!/bin/bash
# The limiter under rocprofv3 with the shim's own event trace: launches seen,
# throttle waits and GPU time charged, plain vs traced (graph replays).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/evprobe3; rm -rf $O; mkdir -p $O/tp $O/tt; export TMPDIR=/tmp; export PYTHONPATH=$PWD
export VGPU_LOG_LEVEL=2
B="bench.py --pods 1 --gpucores 25 --cu-share temporal --core-policy force --seconds 4 --warmup 10 --no-cap-probe"
VGPU_TRACE=$PWD/$O/tp timeout -k 10 200 python3 -u $B > $O/plain.json 2> $O/plain.err || { tail -5 $O/plain.err; exit 1; }
VGPU_TRACE=$PWD/$O/tt timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/k/%pid% -o run -- python3 $B > $O/traced.json 2> $O/traced.err || { tail -5 $O/traced.err; exit 1; }
for m in tp tt; do
  echo "== $m $(grep -o '"value": [0-9.]*' $O/$([ $m = tp ] && echo plain || echo traced).json)"
  for f in $O/$m/*; do python3 -c "
import sys, collections
from vgpu.monitor.trace import read
h, ev = read(sys.argv[1])
c = collections.Counter(e['type'] for e in ev)
gt = [e for e in ev if e['type'] == 'gpu_time']
th = [e for e in ev if e['type'] == 'throttle']
span = (ev[-1]['t_ns'] - ev[0]['t_ns']) / 1e9 if ev else 0
print(dict(c), 'span_s', round(span, 2), 'charged_s', round(sum(e['a'] for e in gt) / 1e9, 3),
      'busy_s', round(sum(e['b'] for e in gt) / 1e9, 3), 'throttle_s', round(sum(e['a'] for e in th) / 1e9, 3))
" $f; done
done
