#!/bin/bash
# GPU-box: HBM traffic per kernel dispatch for the default bench workload, from separate
# rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE; MI355X_MICROARCH.md §HBM).
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=$GRAFT_REPO_ROOT/gpurun_out/traffic_$TAG
mkdir -p $OUT
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  cd /tmp && timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d $OUT/p$i -o run -- \
     python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --capture 512 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $c rc=$rc"; tail -2 $OUT/p$i.log
  [ $rc -ne 0 ] && exit $rc
done
python3 $GRAFT_REPO_ROOT/tools/traffic_json.py $OUT > $OUT/traffic.json && cat $OUT/traffic.json
