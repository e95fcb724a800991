#!/bin/bash
# GPU-box: the GPU suite on the default build, per-kernel stats of the default bench for the
# variants under lib_variants, the C4 cube per variant (and with every light in the direct
# loop), and the kernel trace of the default build's C4 cube. usage: tools/gpu_r3_g.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3g}
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
YRT_ALL_DIRECT_LIGHTS=1 timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1 > gpurun_out/${TAG}_c4_alldirect.log 2>&1
rc=$?; echo "c4 cube all-direct rc=$rc"; grep '^{' gpurun_out/${TAG}_c4_alldirect.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_k_cube -o run -- \
  python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 1 > $R/gpurun_out/${TAG}_k_cube.log 2>&1
rc=$?; cd $R; echo "kstats cube rc=$rc"; python3 tools/kstats_csv.py gpurun_out/${TAG}_k_cube 8
exit 0
