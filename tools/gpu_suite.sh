#!/bin/bash
# GPU-box: GPU suite and smoke() on the working tree, the default bench line, and the N=2
# gloo rehearsal of bench.py (two ranks on this one GPU).
# usage: tools/gpu_suite.sh <tag>
export TMPDIR=/tmp
TAG=${1:-suite}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/bench_$TAG.json
[ $rc -ne 0 ] && exit $rc
YRT_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_n2_$TAG.json 2> gpurun_out/bench_n2_$TAG.err
rc=$?; echo "n2 rc=$rc"; grep "^{" gpurun_out/bench_n2_$TAG.json | cut -c1-200
exit $rc
