#!/bin/bash
# GPU-box: C4 cubemap batch-capacity sweep, cube job and face loop, at N = 1 and N = 8 shares
# (tools/cube_shard_time.py). usage: tools/gpu_r3_l.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3l}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for cap in 0 33554432 16777216; do
  for m in cube face; do
    timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode $m --gpus 1,8 --capacity $cap > gpurun_out/${TAG}_${m}_$cap.log 2>&1
    rc=$?; echo "c4 $m cap=$cap rc=$rc"; grep '^{' gpurun_out/${TAG}_${m}_$cap.log | cut -c1-150
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
