#!/bin/bash
# GPU-box: GPU suite (default build), C3 kernel stats per variant, C4 cube per variant, C5
# render-only (face loop and cube job) on the default build and cube job on the old variant.
# usage: tools/gpu_r3_h.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3h}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_pytest.log | tail -8
[ $rc -ge 2 ] && exit $rc
bash tools/gpu_kstats.sh ${TAG} || exit $?
for v in old new; do
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1 > gpurun_out/${TAG}_c4_$v.log 2>&1
  rc=$?; echo "c4 cube $v rc=$rc"; grep '^{' gpurun_out/${TAG}_c4_$v.log | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u tools/c5_bench.py --no-startrt --no-cpu --out gpurun_out/${TAG}_c5_new.json > gpurun_out/${TAG}_c5_new.log 2>&1
rc=$?; echo "c5 new rc=$rc"; tail -2 gpurun_out/${TAG}_c5_new.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/old timeout -k 10 300 python -u tools/c5_bench.py --no-startrt --no-cpu --no-face --out gpurun_out/${TAG}_c5_old.json > gpurun_out/${TAG}_c5_old.log 2>&1
rc=$?; echo "c5 old rc=$rc"; tail -1 gpurun_out/${TAG}_c5_old.log | cut -c1-400
exit 0
