#!/bin/bash
# GPU-box: C3 kernel stats per variant (any-hit refill threshold / LDS ring, 128-byte shade
# records), then rocprof kernel statistics + PMC passes of C5 and C4. usage: tools/gpu_r3_j.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3j}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
bash tools/gpu_kstats.sh ${TAG} || exit $?
bash tools/gpu_profile_cmd.sh c5_${TAG} tools/c5_profile.py --spp 64 || exit $?
bash tools/gpu_profile_cmd.sh c4_${TAG} tools/cube_shard_time.py C4 --mode cube --gpus 1 || exit $?
exit 0
