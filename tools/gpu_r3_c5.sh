#!/bin/bash
# GPU-box: C5 (one FPR view pair at 64 spp, tools/c5_profile.py) and the C3 bench per variant
# (lib_variants/old, new), alternating, on one box.
# usage: tools/gpu_r3_c5.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3c5}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in old new old new; do
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u tools/c5_profile.py --spp 64 --views 2 > gpurun_out/${TAG}_c5_$v.log 2>&1
  rc=$?; echo "c5 $v rc=$rc $(grep '^{' gpurun_out/${TAG}_c5_$v.log | cut -c1-160)"
  [ $rc -ne 0 ] && exit $rc
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c3_$v.json 2> gpurun_out/${TAG}_c3_$v.err
  rc=$?; echo "c3 $v rc=$rc $(cut -c100-200 gpurun_out/${TAG}_c3_$v.json)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
