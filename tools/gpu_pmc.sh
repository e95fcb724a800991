#!/bin/bash
# GPU-box: PMC counter passes of the bench workload (one rocprofv3 run per counter group,
# kernel trace only, each under its own time limit) + the VALU calibration kernel, then
# tools/pmc_json.py -> gpurun_out/pmc_<tag>/pmc.json (copy to profiles/pmc_c3.json).
# usage: tools/gpu_pmc.sh <tag> ["<bench args>"]
set -o pipefail
export TMPDIR=/tmp
# one frame, no warm-up: the depth-0 kernels the steady state uses on C3 (camera rays mostly hit,
# so Device::render_shard picks k_raygen + the queued trace once it has measured that)
export YRT_PRIMARY=${YRT_PRIMARY:-0}
# one lane: the per-dispatch counts must describe the batches of the bench's one-lane roofline
# frame (with three lanes a C3 frame splits into 6 batches instead of 4; the counters are
# collected with kernels serialized either way)
export YRT_LANES=${YRT_LANES:-1}
TAG=${1:-dev}
ARGS=${2:-""}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
# VALU lane utilization: thread-cycles of VALU work per VALU instruction cycle, if
# this rocprofv3 lists the counter on gfx950 (rocprofv3 -L), normalized by the calibration
# kernel's (every lane active) in tools/pmc_json.py
LANE=""
cd /tmp && timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -q "SQ_THREAD_CYCLES_VALU" $OUT/counters.txt && LANE="SQ_THREAD_CYCLES_VALU"
echo "lane counter: ${LANE:-none listed}"
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum" ${LANE:+"$LANE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"}; do
  i=$((i+1))
  cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
     python3 $R/bench.py --steps 1 --warmup 0 --capture 0 --no-cpu-baseline $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
cd /tmp && timeout -k 10 -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT $LANE \
   --output-format csv -d $OUT/calib -o run -- $R/tools/valu_calib > $OUT/calib.log 2>&1
rc=$?; echo "calib rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/calib.log; exit $rc; }
cd $R && python3 tools/pmc_json.py $OUT $OUT/pmc.json > /dev/null && echo "pmc.json written"
