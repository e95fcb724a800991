#!/bin/bash
# GPU-box, round-3 evidence part B: the C4 cubemap strong-scaling prediction (one GPU, every
# rank's share), the C5 cube job render-only at 1024 spp, and every BASELINE config with the CPU
# restatement beside it.
# usage: tools/gpu_configs.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3f}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube > gpurun_out/c4shard_$TAG.log 2>&1
rc=$?; echo "c4 shard rc=$rc"; grep '^{' gpurun_out/c4shard_$TAG.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/c5_bench.py --no-face --no-startrt --no-cpu --out gpurun_out/c5_$TAG.json > gpurun_out/c5_$TAG.log 2>&1
rc=$?; echo "c5 rc=$rc"; tail -n 3 gpurun_out/c5_$TAG.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/configs_bench.py > gpurun_out/configs_$TAG.txt 2>&1
rc=$?; echo "configs rc=$rc"; cut -c1-200 gpurun_out/configs_$TAG.txt
exit $rc
