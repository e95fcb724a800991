#!/bin/bash
# GPU-box: 48-byte index shade records (tsidx) vs the 96-byte records (new): C3 kernel stats
# twice, C5 one view at 64 spp and the C4 cube per variant, then the C3 PMC passes of tsidx.
# usage: tools/gpu_r3_x.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3x}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_kstats.sh ${TAG}a || exit $?
bash tools/gpu_kstats.sh ${TAG}b || exit $?
for v in new tsidx new tsidx; do
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u tools/c5_profile.py --spp 64 --views 2 > gpurun_out/${TAG}_c5_$v.log 2>&1
  rc=$?; echo "c5 $v rc=$rc $(grep '^{' gpurun_out/${TAG}_c5_$v.log | cut -c1-110)"
  [ $rc -ne 0 ] && exit $rc
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1 > gpurun_out/${TAG}_c4_$v.log 2>&1
  rc=$?; echo "c4 $v rc=$rc $(grep '^{' gpurun_out/${TAG}_c4_$v.log | cut -c1-130)"
  [ $rc -ne 0 ] && exit $rc
done
YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/tsidx bash tools/gpu_pmc.sh ${TAG}_tsidx || exit $?
exit 0
