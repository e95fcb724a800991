#!/bin/bash
# GPU-box: the round's evidence for HEAD in one call — GPU suite, smoke(), default bench line
# (with the CPU baseline), the same command under rocprofv3 kernel stats, then the PMC passes.
# usage: tools/gpu_final.sh <tag>
export TMPDIR=/tmp
TAG=${1:-final}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 3 gpurun_out/smoke_$TAG.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_bench.sh $TAG || exit $?
bash tools/gpu_pmc.sh $TAG || exit $?
exit 0
