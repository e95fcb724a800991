#!/bin/bash
# GPU-box: rocprofv3 kernel statistics and PMC passes (one run per counter group, kernel trace
# only, each under its own time limit) of an arbitrary python workload, then tools/pmc_json.py.
# usage: tools/gpu_profile_cmd.sh <tag> <script.py> [args...]
#   -> gpurun_out/kstats_<tag>/ (kernel_stats.csv), gpurun_out/pmc_<tag>/pmc.json
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
R=$GRAFT_REPO_ROOT
# the workload runs from /tmp: make a relative script path absolute
S=$1; shift
case $S in /*) ;; *) S=$R/$S;; esac
set -- "$S" "$@"
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kstats_$TAG -o run -- \
   python3 "$@" > $R/gpurun_out/kstats_$TAG.log 2>&1
rc=$?; echo "kstats rc=$rc"; tail -2 $R/gpurun_out/kstats_$TAG.log; [ $rc -ne 0 ] && exit $rc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
     python3 "$@" > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
cd $R && python3 tools/pmc_json.py $OUT $OUT/pmc.json > /dev/null && echo "pmc.json written"
