#!/bin/bash
# GPU-box: cube job vs face loop after the per-frame grid-hint rates: render/readback split,
# then N = 1 / 8 shares of both. usage: tools/gpu_r3_p.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3p}
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/cube_face_split.py > gpurun_out/${TAG}_split.log 2>&1
rc=$?; echo "split rc=$rc"; tail -1 gpurun_out/${TAG}_split.log
[ $rc -ne 0 ] && exit $rc
for m in cube face; do
  timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode $m --gpus 1,8 > gpurun_out/${TAG}_${m}.log 2>&1
  rc=$?; echo "c4 $m rc=$rc"; grep '^{' gpurun_out/${TAG}_${m}.log | cut -c1-330
  [ $rc -ne 0 ] && exit $rc
done
exit 0
