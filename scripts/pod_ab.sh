#!/bin/bash
# One workload's pod (exclusive, hipGraph) under env variants, alternating:
#   bash scripts/pod_ab.sh <workload> "TAG1 ENV=V ..." "TAG2 ENV=V ..." ...
set -u
cd "$(dirname "$0")/.."
W=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    tag=${v%% *}; envs=${v#* }; [ "$envs" = "$v" ] && envs=""
    out=$(env $envs timeout -k 10 200 python3 -m vgpu.bench.pod --workload $W --steps 30 --warmup 5 --graph --no-wait 2>/dev/null | grep DONE) || { echo "$tag FAILED"; exit 1; }
    echo "$tag rep$rep $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()[5:]); print(round(d["throughput"],1), round(d["ms_per_step"],3))')"
  done
done
