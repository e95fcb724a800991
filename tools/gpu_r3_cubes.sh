#!/bin/bash
# GPU-box: round-3 cube-job check: new tests, the GPU suite, the default bench, and the C4
# strong-scaling prediction (per-face loop vs one job per cube). usage: tools/gpu_r3_cubes.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3b}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cubes.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_cubes.log 2>&1
rc=$?; echo "cube tests rc=$rc"; tail -n 4 gpurun_out/${TAG}_cubes.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_cubes.py > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/${TAG}_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json | cut -c1-400
[ $rc -ne 0 ] && exit $rc
for m in face cube; do
  timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode $m --out gpurun_out/${TAG}_c4_$m.jsonl > gpurun_out/${TAG}_c4_$m.log 2>&1
  rc=$?; echo "c4 $m rc=$rc"; grep '^{' gpurun_out/${TAG}_c4_$m.log | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
done
exit 0
