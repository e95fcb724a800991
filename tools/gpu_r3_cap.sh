#!/bin/bash
# GPU-box: C3 bench over batch capacities and lane counts (same box), two rounds.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for round in 1 2; do
  for cfg in "2 0" "2 50331648" "2 100663296" "2 134217728" "3 0" "3 50331648"; do
    set -- $cfg
    YRT_LANES=$1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --capacity $2 > gpurun_out/cap_$1_$2.json 2> gpurun_out/cap_$1_$2.err
    rc=$?; echo "lanes $1 cap $2 rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/cap_$1_$2.json')); print(d['ms_per_step'], 'ms', d['value'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
