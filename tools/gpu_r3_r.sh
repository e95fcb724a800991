#!/bin/bash
# GPU-box: C3 kernel stats per variant (nearest-first child order), twice each (box noise).
# usage: tools/gpu_r3_r.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3r}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_kstats.sh ${TAG}a || exit $?
bash tools/gpu_kstats.sh ${TAG}b || exit $?
exit 0
