#!/bin/bash
# GPU-box: lanes x batch-capacity sweep of the default bench (no CPU baseline), same box
mkdir -p gpurun_out
for cfg in "2 0" "3 0" "2 50331648" "2 100663296" "3 50331648" "2 0"; do
  set -- $cfg
  extra=""; [ "$2" != "0" ] && extra="--capacity $2"
  YRT_LANES=$1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --capture 0 $extra > gpurun_out/lanes_$1_$2.json 2> gpurun_out/lanes_$1_$2.err
  rc=$?
  echo "lanes=$1 cap=$2 rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/lanes_$1_$2.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
