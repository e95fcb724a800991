#!/bin/bash
# GPU-box: lane 0's stream at the greatest priority (YRT_LANE_PRIORITY=1) vs default: C3 bench,
# C4 cube job, C5 at 64 spp, two rounds on one box.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for round in 1 2; do
  for p in 0 1; do
    if [ $p = 1 ]; then export YRT_LANE_PRIORITY=1; else unset YRT_LANE_PRIORITY; fi
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prio_c3_$p.json 2> gpurun_out/prio_c3_$p.err
    rc=$?; echo "C3 prio=$p rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/prio_c3_$p.json')); print(d['ms_per_step'], 'ms')" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
    timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1 > gpurun_out/prio_c4_$p.log 2>&1
    rc=$?; echo "C4 prio=$p rc=$rc $(grep '^{' gpurun_out/prio_c4_$p.log | cut -c95-125)"
    [ $rc -ne 0 ] && exit $rc
    timeout -k 10 300 python -u tools/c5_profile.py --spp 64 --views 2 > gpurun_out/prio_c5_$p.log 2>&1
    rc=$?; echo "C5 prio=$p rc=$rc $(grep '^{' gpurun_out/prio_c5_$p.log | cut -c40-90)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
