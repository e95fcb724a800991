# round-4 batch K: with full grids (hints off): lanes one / two batches ahead and the batch
# capacity (64 M / 96 M / 128 M paths): C4 N = 1, 2, 4, 8 rank shares and C3
mkdir -p gpurun_out
for cfg in "def||" "pd2|YRT_PEND_DEPTH=2|" "c96|YRT_LANES=2|--capacity 100663296" "c128|YRT_LANES=2|--capacity 134217728" "def_again||"; do
  IFS='|' read -r tag envs args <<< "$cfg"
  env $envs timeout -k 10 240 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,2,4,8 $args > gpurun_out/c4k_$tag.log 2>&1 || exit $?
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --capture 0 $args > gpurun_out/c3k_$tag.json 2> gpurun_out/c3k_$tag.err || exit $?
  echo "$tag [$envs $args] C3 $(python3 -c "import json; d=json.load(open('gpurun_out/c3k_$tag.json')); print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step')")"
  grep '^{' gpurun_out/c4k_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  C4 N=%d max %.1f ms mean %.1f eff %s' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
done
