#!/bin/bash
# GPU-box: trace-grid rays-per-wave A/B (C3 kernel stats, C4 cube per variant), then the
# one-GPU strong-scaling prediction of the C4 and C5 cubemaps (tools/cube_shard_time.py).
# usage: tools/gpu_r3_k.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3k}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
bash tools/gpu_kstats.sh ${TAG} || exit $?
for v in new rpa1k rpa4k rpc1k rpc4k; do
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1 > gpurun_out/${TAG}_c4_$v.log 2>&1
  rc=$?; echo "c4 cube $v rc=$rc"; grep '^{' gpurun_out/${TAG}_c4_$v.log | cut -c1-160
  [ $rc -ne 0 ] && exit $rc
done
for m in face cube; do
  timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode $m --out gpurun_out/${TAG}_scale_c4_$m.jsonl > gpurun_out/${TAG}_scale_c4_$m.log 2>&1
  rc=$?; echo "scale c4 $m rc=$rc"; grep '^{' gpurun_out/${TAG}_scale_c4_$m.log | cut -c1-220
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python -u tools/cube_shard_time.py C5 --mode cube --out gpurun_out/${TAG}_scale_c5_cube.jsonl > gpurun_out/${TAG}_scale_c5_cube.log 2>&1
rc=$?; echo "scale c5 cube rc=$rc"; grep '^{' gpurun_out/${TAG}_scale_c5_cube.log | cut -c1-220
exit $rc
