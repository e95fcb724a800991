#!/bin/bash
# GPU-box: C5 per-path debug of the full-spp band mismatch (pixel 1081,772 sample 191 of scene
# camera 2), the sample-scene tests, then kernel statistics of one C4 cubemap as 12 face
# renders and as one cube job (cube-vs-face time split). usage: tools/gpu_r3_e.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3e}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/pathdbg timeout -k 10 300 python -u tools/c5_path_debug.py 2 1081 772 191 \
  > gpurun_out/${TAG}_path.log 2>&1
rc=$?; echo "path debug rc=$rc"; cut -c1-400 gpurun_out/${TAG}_path.log | tail -14
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_samples.py -m gpu -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_pytest.log | tail -5
[ $rc -ge 2 ] && exit $rc
for m in face cube; do
  cd /tmp && timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_k_$m -o run -- \
    python3 $R/tools/cube_shard_time.py C4 --mode $m --gpus 1 > $R/gpurun_out/${TAG}_k_$m.log 2>&1
  rc=$?; cd $R; echo "kstats $m rc=$rc"; grep '^{' gpurun_out/${TAG}_k_$m.log | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
  python3 tools/kstats_csv.py gpurun_out/${TAG}_k_$m 8
done
for m in face cube; do
  YRT_NO_GRID_HINTS=1 timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode $m --gpus 1 > gpurun_out/${TAG}_nohint_$m.log 2>&1
  rc=$?; echo "no-hints $m rc=$rc"; grep '^{' gpurun_out/${TAG}_nohint_$m.log | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
done
exit 0
