#!/bin/bash
# GPU-box: C5 full-spp parity debugging, then the GPU suite (all failures listed), the default
# bench and the C4 cube strong-scaling prediction. usage: tools/gpu_r3_dbg.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3c}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/c5_pixel_debug.py 2 760 16 4 > gpurun_out/${TAG}_c5dbg.log 2>&1
rc=$?; echo "c5 debug rc=$rc"; cut -c1-600 gpurun_out/${TAG}_c5dbg.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_pytest.log | tail -8
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/${TAG}_bench.json
[ $rc -ne 0 ] && exit $rc
for m in face cube; do
  timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode $m --out gpurun_out/${TAG}_c4_$m.jsonl > gpurun_out/${TAG}_c4_$m.log 2>&1
  rc=$?; echo "c4 $m rc=$rc"; grep '^{' gpurun_out/${TAG}_c4_$m.log | cut -c1-220
  [ $rc -ne 0 ] && exit $rc
done
exit 0
