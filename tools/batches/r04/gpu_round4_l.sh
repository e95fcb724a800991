# round-4 batch L: the end-of-job tail with full grids — tapered last batch round (YRT_TAPER=1)
# at 64 M and 96 M paths per batch: C4 N = 1, 4, 8 rank shares
mkdir -p gpurun_out
for cfg in "def||" "taper|YRT_TAPER=1|" "c96|YRT_LANES=2|--capacity 100663296" "c96taper|YRT_TAPER=1|--capacity 100663296" "def_again||"; do
  IFS='|' read -r tag envs args <<< "$cfg"
  env $envs timeout -k 10 240 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,4,8 $args > gpurun_out/c4l_$tag.log 2>&1 || exit $?
  echo "$tag [$envs $args]"
  grep '^{' gpurun_out/c4l_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  C4 N=%d max %.1f ms mean %.1f eff %s' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
done
