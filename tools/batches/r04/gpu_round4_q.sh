# round-4 batch Q: 1.5x batches for shards of 9-16 batches per lane (C4 N = 4) on top of the 2x
# rule — invariance tests, C4 N = 1, 2, 4, 8 and C3 against YRT_BATCH_GROW=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cubes.py tests/test_gpu_parity.py -m gpu -q -k "batch_grow or batch_capacity" --timeout 200 --timeout-method thread > gpurun_out/pytest_r4q.log 2>&1 || { tail -20 gpurun_out/pytest_r4q.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_r4q.log
for cfg in "grow|" "nogrow|YRT_BATCH_GROW=0" "grow_again|"; do
  IFS='|' read -r tag envs <<< "$cfg"
  env $envs timeout -k 10 240 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,2,4,8 > gpurun_out/c4q_$tag.log 2>&1 || exit $?
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --capture 0 > gpurun_out/c3q_$tag.json 2> gpurun_out/c3q_$tag.err || exit $?
  echo "$tag [$envs] C3 $(python3 -c "import json; d=json.load(open('gpurun_out/c3q_$tag.json')); print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step')")"
  grep '^{' gpurun_out/c4q_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  C4 N=%d max %.1f ms mean %.1f eff %s' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
done
