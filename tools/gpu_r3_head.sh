#!/bin/bash
# GPU-box: HEAD check after a container restore — GPU suite, smoke(), default bench line.
# usage: tools/gpu_r3_head.sh <tag>
export TMPDIR=/tmp
TAG=${1:-head}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 3 gpurun_out/smoke_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench_$TAG.json
exit $rc
