#!/bin/bash
# GPU-box: SIMD-utilization counters of the traversal (YRT_PROFILE variant) + SQ PMC pass
# on the reduced C3 frame. Output under gpurun_out/diag_<tag>/.
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-dev}
OUT=$GRAFT_REPO_ROOT/gpurun_out/diag_$TAG
mkdir -p $OUT
YRT_LIB_DIR=$GRAFT_REPO_ROOT/yulio-raytracer_amd/lib_variants/prof timeout -k 10 120 python tools/trace_profile.py 1024 > $OUT/trace_profile.txt 2>&1
rc=$?; echo "trace_profile rc=$rc"; cat $OUT/trace_profile.txt | tail -6
[ $rc -ne 0 ] && exit $rc
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
     python3 $GRAFT_REPO_ROOT/bench.py --size 1024 --spp 16 --steps 1 --warmup 0 --no-cpu-baseline --capture 256 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py $OUT > $OUT/summary.txt; cat $OUT/summary.txt
