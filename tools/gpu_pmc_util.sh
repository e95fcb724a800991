#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_util
mkdir -p $OUT
i=0
for grp in "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU" "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32" "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
     python3 $GRAFT_REPO_ROOT/bench.py --size 1024 --spp 16 --steps 1 --warmup 0 --no-cpu-baseline --capture 256 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; fi
  [ $rc -ge 124 ] && exit $rc
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT > $OUT/summary.txt; cat $OUT/summary.txt
