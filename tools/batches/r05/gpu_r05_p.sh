# round-5 batch P: C3 rank shares at N = 8 on one GPU (tools/cube_shard_time.py C3 --gpus 1,8)
# for batch capacities 64 M (default: one batch per lane), 8 M, 4 M paths and 3 / 4 lanes
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # tag, env..., args
  local tag=$1; shift

  timeout -k 10 300 env $ENVS python -u tools/cube_shard_time.py C3 --gpus 1,8 $ARGS > gpurun_out/c3p_$tag.txt 2>&1 || { tail -5 gpurun_out/c3p_$tag.txt; exit 1; }
  grep '^{' gpurun_out/c3p_$tag.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$tag N=%d max %.1f mean %.1f eff %.3f' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
}
ENVS="" ARGS="" run def
ENVS="" ARGS="--capacity 8388608" run cap8m
ENVS="" ARGS="--capacity 4194304" run cap4m
ENVS="YRT_LANES=3" ARGS="" run lanes3
ENVS="YRT_LANES=4" ARGS="" run lanes4
ENVS="YRT_LANES=4" ARGS="--capacity 8388608" run lanes4cap8m
ENVS="" ARGS="" run defb
