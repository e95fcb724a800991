# round-4 batch J: grid-size hint pad (queue entries added to every hinted grid) against the
# hints' under-sizing at N = 2 / 3: C4 N = 1, 2, 3, 8 rank shares and C3
mkdir -p gpurun_out
for cfg in "p64k|YRT_GRID_HINTS=1" "p256k|YRT_GRID_HINTS=1 YRT_HINT_PAD=262144" "p512k|YRT_GRID_HINTS=1 YRT_HINT_PAD=524288" "p1m|YRT_GRID_HINTS=1 YRT_HINT_PAD=1048576" "nohint|" "p64k_again|YRT_GRID_HINTS=1"; do
  IFS='|' read -r tag envs <<< "$cfg"
  env $envs timeout -k 10 240 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,2,3,8 > gpurun_out/c4j_$tag.log 2>&1 || exit $?
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --capture 0 > gpurun_out/c3j_$tag.json 2> gpurun_out/c3j_$tag.err || exit $?
  echo "$tag [$envs] C3 $(python3 -c "import json; d=json.load(open('gpurun_out/c3j_$tag.json')); print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step')")"
  grep '^{' gpurun_out/c4j_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  C4 N=%d max %.1f ms mean %.1f eff %s' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
done
