#!/bin/bash
# GPU-box: stereo raygen without the identity-factor products, branch-free acos, fastdiv index
# math (new) vs HEAD (old): GPU suite on new, then C4 cube job and C3 frame per variant, twice.
# usage: tools/gpu_r3_y.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3y}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && exit $rc
for v in old new old new; do
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1 > gpurun_out/${TAG}_c4_$v.log 2>&1
  rc=$?; echo "c4 $v rc=$rc $(grep '^{' gpurun_out/${TAG}_c4_$v.log | cut -c1-130)"
  [ $rc -ne 0 ] && exit $rc
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c3_$v.json 2> gpurun_out/${TAG}_c3_$v.err
  rc=$?; echo "c3 $v rc=$rc $(cut -c100-200 gpurun_out/${TAG}_c3_$v.json)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
