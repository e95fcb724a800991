#!/bin/bash
# GPU-box: GPU suite on the working tree, then rocprofv3 kernel stats of the C4 cube job
# (tools/cube_shard_time.py) and the C3 bench per variant (lib_variants/old = HEAD, new =
# working tree), back to back on one box.
# usage: tools/gpu_r3_z.sh <tag> [skip-tests]
export TMPDIR=/tmp
TAG=${1:-r3z}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
if [ "$2" != "skip-tests" ]; then
  cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu_$TAG.log
  [ $rc -ne 0 ] && exit $rc
fi
for v in old new; do
  cd /tmp && YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/gpurun_out/ks_${TAG}_$v -o run -- python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 1 > $R/gpurun_out/ks_${TAG}_$v.log 2>&1
  rc=$?
  echo "== C4 $v rc=$rc $(grep '^{' $R/gpurun_out/ks_${TAG}_$v.log | cut -c60-130)"
  [ $rc -ne 0 ] && exit $rc
  python3 $R/tools/kstats_csv.py $R/gpurun_out/ks_${TAG}_$v 5
done
for v in old new old new; do
  cd /tmp && YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 1 > $R/gpurun_out/c4_${TAG}_$v.log 2>&1
  rc=$?; echo "C4 $v rc=$rc $(grep '^{' $R/gpurun_out/c4_${TAG}_$v.log | cut -c60-130)"
  [ $rc -ne 0 ] && exit $rc
  cd $R && YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c3_${TAG}_$v.json 2> gpurun_out/c3_${TAG}_$v.err
  rc=$?; echo "C3 $v rc=$rc $(cut -c100-200 gpurun_out/c3_${TAG}_$v.json)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
