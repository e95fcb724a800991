# round-4 batch M: larger batches for shards of 5-8 batches per lane (default) against
# YRT_BATCH_GROW=0 — the invariance test, C4 N = 1, 2, 4, 8 rank shares and C3
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cubes.py tests/test_gpu_parity.py -m gpu -q -k "batch_grow or batch_capacity or tile_shards or shards_compose" --timeout 200 --timeout-method thread > gpurun_out/pytest_r4m.log 2>&1 || { tail -20 gpurun_out/pytest_r4m.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_r4m.log
for cfg in "grow|" "nogrow|YRT_BATCH_GROW=0" "grow_again|"; do
  IFS='|' read -r tag envs <<< "$cfg"
  env $envs timeout -k 10 240 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,2,4,8 > gpurun_out/c4m_$tag.log 2>&1 || exit $?
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --capture 0 > gpurun_out/c3m_$tag.json 2> gpurun_out/c3m_$tag.err || exit $?
  echo "$tag [$envs] C3 $(python3 -c "import json; d=json.load(open('gpurun_out/c3m_$tag.json')); print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step')")"
  grep '^{' gpurun_out/c4m_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  C4 N=%d max %.1f ms mean %.1f eff %s' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
done
