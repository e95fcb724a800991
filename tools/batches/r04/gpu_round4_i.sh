# round-4 batch I: batches dealt to the first lane with room (default) against lanes in turn
# (YRT_LANE_ORDER=rr), one and two batches ahead: C4 N = 1, 2, 3, 4, 8 rank shares and C3
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "batch_capacity or fused_primary or tile_shards" --timeout 200 --timeout-method thread > gpurun_out/pytest_r4i.log 2>&1 || { tail -20 gpurun_out/pytest_r4i.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_r4i.log
for cfg in "dyn|" "dyn_pd2|YRT_PEND_DEPTH=2" "rr|YRT_LANE_ORDER=rr" "dyn2|"; do
  IFS='|' read -r tag envs <<< "$cfg"
  env $envs timeout -k 10 240 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,2,3,4,8 > gpurun_out/c4i_$tag.log 2>&1 || exit $?
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --capture 0 > gpurun_out/c3i_$tag.json 2> gpurun_out/c3i_$tag.err || exit $?
  echo "$tag [$envs] C3 $(python3 -c "import json; d=json.load(open('gpurun_out/c3i_$tag.json')); print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step')")"
  grep '^{' gpurun_out/c4i_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  C4 N=%d max %.1f ms mean %.1f eff %s' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
done
