#!/bin/bash
# GPU-box: GPU suite on the default build and on one variant, then per-kernel stats of every
# variant under lib_variants with one lane (kernels do not overlap) and with the default two.
# usage: tools/gpu_ab.sh <tag> <variant-for-parity>
export TMPDIR=/tmp
TAG=${1:-ab}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}_default.log 2>&1
rc=$?; echo "pytest default rc=$rc"; tail -n 3 gpurun_out/pytest_${TAG}_default.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$2" ]; then
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$2 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}_$2.log 2>&1
  rc=$?; echo "pytest $2 rc=$rc"; tail -n 3 gpurun_out/pytest_${TAG}_$2.log
  [ $rc -ne 0 ] && exit $rc
fi
YRT_LANES=1 bash tools/gpu_kstats.sh ${TAG}1 || exit $?
bash tools/gpu_kstats.sh ${TAG}2 || exit $?
exit 0
