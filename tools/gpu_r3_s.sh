#!/bin/bash
# GPU-box: kernel trace of rank 0's N = 8 share of the C4 cubemap (cube job), to see where the
# strong-scaling overhead goes. usage: tools/gpu_r3_s.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3s}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_k8 -o run -- \
  python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 8 --ranks 0 > $R/gpurun_out/${TAG}_k8.log 2>&1
rc=$?; cd $R; echo "kstats rc=$rc"; grep '^{' gpurun_out/${TAG}_k8.log | cut -c1-200
python3 tools/kstats_csv.py gpurun_out/${TAG}_k8 8
exit $rc
