set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abcus
for i in 1 2; do
  for v in default 256 192; do
    if [ $v = default ]; then
      timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cap-probe > gpurun_out/abcus/${v}_$i.json 2>/dev/null || exit 1
    else
      VGPU_CONV_CUS=$v timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cap-probe > gpurun_out/abcus/${v}_$i.json 2>/dev/null || exit 1
    fi
    echo "$v $i $(grep -o '"value": [0-9.]*' gpurun_out/abcus/${v}_$i.json)"
  done
done
