#!/bin/bash
# GPU-box: PMC counter passes (one rocprofv3 run per counter group, kernel trace only)
# on a reduced bench frame; summaries go to gpurun_out/pmc_<tag>/.
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-dev}
ARGS=${2:-"--size 1024 --spp 16 --steps 1 --warmup 0 --no-cpu-baseline --capture 256"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
     python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; fi
  [ $rc -ge 124 ] && exit $rc
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT > $OUT/summary.txt; cat $OUT/summary.txt
exit 0
