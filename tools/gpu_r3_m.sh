#!/bin/bash
# GPU-box: C4 cube job vs face loop at N = 1 / 8 shares (per-frame grid hints), the same with
# one lane, and the N = 2 gloo rehearsal of bench.py (stereo cubemap + gather check).
# usage: tools/gpu_r3_m.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3m}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for m in cube face; do
  timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode $m --gpus 1,8 > gpurun_out/${TAG}_${m}.log 2>&1
  rc=$?; echo "c4 $m rc=$rc"; grep '^{' gpurun_out/${TAG}_${m}.log | cut -c1-150
  [ $rc -ne 0 ] && exit $rc
  YRT_LANES=1 timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode $m --gpus 1 > gpurun_out/${TAG}_${m}_l1.log 2>&1
  rc=$?; echo "c4 $m one lane rc=$rc"; grep '^{' gpurun_out/${TAG}_${m}_l1.log | cut -c1-150
  [ $rc -ne 0 ] && exit $rc
done
YRT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_n2_gloo.json 2> gpurun_out/${TAG}_n2_gloo.err
rc=$?; echo "bench n2 gloo rc=$rc"; tail -c 1500 gpurun_out/${TAG}_n2_gloo.json
exit $rc
