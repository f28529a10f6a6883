#!/bin/bash
# rocprofv3 kernel traces of every ai-benchmark test, exclusive (one pod, no
# shim, hipGraph as in the suite), then the dispatch-size summary.
set -u
cd "$(dirname "$0")/.."
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/ksize
mkdir -p $O
for t in ${TESTS:-1.1 1.2 2.1 2.2 3.1 3.2 4.1 4.2 5.1 5.2}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/$t -o run -- \
    python3 -m vgpu.bench.pod --workload $t --steps 6 --warmup 3 --no-wait --graph --find > $O/$t.log 2>&1
  rc=$?; echo "$t rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/kernel_sizes.py $O > $O/summary.json && cat $O/summary.json
find $O -name "*.csv" -delete  # traces are large; the summary is what we keep
