# round-4 batch H: why the C4 N = 2 rank share runs at 0.91 efficiency (N = 4: 0.98) — N = 1..4
# with the default build, without the fused depth 0, and with the lanes two batches ahead
mkdir -p gpurun_out
for cfg in "def|" "noprim|YRT_PRIMARY=0" "pd2|YRT_PEND_DEPTH=2" "def2|"; do
  IFS='|' read -r tag envs <<< "$cfg"
  env $envs timeout -k 10 200 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,2,3,4 > gpurun_out/c4h_$tag.log 2>&1 || exit $?
  echo "$tag [$envs]"; grep '^{' gpurun_out/c4h_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  N=%d max %.1f ms mean %.1f eff %s' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
done
