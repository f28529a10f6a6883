#!/bin/bash
# Which KFD queues does each pod process own while 4 pods run (type, size)?
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/queues
mkdir -p $O
( sleep 14; for p in /sys/class/kfd/kfd/proc/*; do
    [ -d $p/queues ] || continue
    for q in $p/queues/*; do
      echo "$(basename $p) q$(basename $q): $(for f in $q/*; do echo -n "$(basename $f)=$(cat $f 2>/dev/null | head -c 40) "; done)"
    done
  done ) > $O/kfd_queues.txt 2>&1 &
timeout -k 10 300 python bench.py --no-cap-probe --pods 4 --gpucores 25 --gpumem 72000 --steps 2000 > $O/p4.log 2>&1 || { tail -5 $O/p4.log; exit 1; }
wait
grep -o '"pid": [0-9]*' $O/p4.log | tr '\n' ' '; echo
cat $O/kfd_queues.txt | head -60
