#!/bin/bash
# GPU-box: any-hit refill A/B (C3 kernel stats per variant), any-hit lane utilization of the
# profile builds, then rocprof kernel statistics + PMC passes of C5 and C4 (profiles/r03).
# usage: tools/gpu_r3_i.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3i}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
bash tools/gpu_kstats.sh ${TAG} || exit $?
for v in prof_any prof_any_pf16 prof_any_pf24; do
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 200 python -u tools/trace_profile.py 1024 > gpurun_out/${TAG}_$v.txt 2>&1
  rc=$?; echo "== $v rc=$rc"; tail -4 gpurun_out/${TAG}_$v.txt
  [ $rc -ne 0 ] && exit $rc
done
bash tools/gpu_profile_cmd.sh c5_${TAG} tools/c5_profile.py --spp 64 || exit $?
bash tools/gpu_profile_cmd.sh c4_${TAG} tools/cube_shard_time.py C4 --mode cube --gpus 1 || exit $?
exit 0
