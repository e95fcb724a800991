#!/bin/bash
# GPU-box: spatial-split BVH (YRT_SBVH=1) vs the default on C5 (one view, 64 spp) and C3.
# usage: tools/gpu_r3_v.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3v}
mkdir -p gpurun_out
for sb in 0 1 0 1; do
  YRT_SBVH=$sb timeout -k 10 300 python -u tools/c5_profile.py --spp 64 --views 2 > gpurun_out/${TAG}_c5_$sb.log 2>&1
  rc=$?; echo "c5 sbvh=$sb rc=$rc $(grep '^{' gpurun_out/${TAG}_c5_$sb.log | cut -c1-120)"
  [ $rc -ne 0 ] && exit $rc
done
for sb in 0 1; do
  YRT_SBVH=$sb timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --capture 0 > gpurun_out/${TAG}_c3_$sb.json 2> gpurun_out/${TAG}_c3_$sb.err
  rc=$?; echo "c3 sbvh=$sb rc=$rc $(cut -c1-200 gpurun_out/${TAG}_c3_$sb.json)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
