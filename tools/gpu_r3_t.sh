#!/bin/bash
# GPU-box: one-GPU strong-scaling prediction (render-only) of the C4 and C5 cubemaps.
# usage: tools/gpu_r3_t.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3t}
mkdir -p gpurun_out
for m in face cube; do
  timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode $m --out gpurun_out/${TAG}_scale_c4_$m.jsonl > gpurun_out/${TAG}_scale_c4_$m.log 2>&1
  rc=$?; echo "scale c4 $m rc=$rc"; grep '^{' gpurun_out/${TAG}_scale_c4_$m.log | cut -c1-330
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 700 python -u tools/cube_shard_time.py C5 --mode cube --out gpurun_out/${TAG}_scale_c5_cube.jsonl > gpurun_out/${TAG}_scale_c5_cube.log 2>&1
rc=$?; echo "scale c5 cube rc=$rc"; grep '^{' gpurun_out/${TAG}_scale_c5_cube.log | cut -c1-330
exit $rc
