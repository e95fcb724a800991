#!/bin/bash
# GPU-box: per-kernel statistics of one C4 cubemap as a cube job and as a face loop, one lane
# (kernels do not overlap, so durations are the kernels' own). usage: tools/gpu_r3_n.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3n}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for m in cube face; do
  cd /tmp && YRT_LANES=1 timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_k_$m -o run -- \
    python3 $R/tools/cube_shard_time.py C4 --mode $m --gpus 1 > $R/gpurun_out/${TAG}_k_$m.log 2>&1
  rc=$?; cd $R; echo "kstats $m rc=$rc"; grep '^{' gpurun_out/${TAG}_k_$m.log | cut -c1-150
  [ $rc -ne 0 ] && exit $rc
  python3 tools/kstats_csv.py gpurun_out/${TAG}_k_$m 8
done
exit 0
