#!/bin/bash
# GPU-box: the GPU suite on the default build (all failures listed), then per-kernel stats of
# the default bench for every variant (box-factor and geometry-record A/B) and the C4 cube.
# usage: tools/gpu_r3_f.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3f}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_pytest.log | tail -8
[ $rc -ge 2 ] && exit $rc
bash tools/gpu_kstats.sh ${TAG} || exit $?
for v in r36 r12; do
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1 > gpurun_out/${TAG}_c4_$v.log 2>&1
  rc=$?; echo "c4 cube $v rc=$rc"; grep '^{' gpurun_out/${TAG}_c4_$v.log | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
done
exit 0
