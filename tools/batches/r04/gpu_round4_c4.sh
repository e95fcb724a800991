mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,8 > gpurun_out/c4_$tag.log 2>&1 || return $?
  echo "$tag [$*]"; grep '^{' gpurun_out/c4_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  N=%d max %.1f ms mean %.1f eff %s' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
}
run eager YRT_EAGER_READBACK=1 || exit $?
run def YRT_HINT_PAD=65536 || exit $?
run pad4k YRT_HINT_PAD=4096 || exit $?
run pad1k YRT_HINT_PAD=1024 || exit $?
run def2 YRT_HINT_PAD=65536 || exit $?
