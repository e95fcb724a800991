# round-4 C4 per-batch fixed cost: a kernel timeline of one N=8 rank share (rocprofv3 kernel
# trace, read by tools/c4_timeline.py), and lane-count / batch-capacity sweeps of the share
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c4trace -o run -- \
  python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 8 --ranks 0 > $R/gpurun_out/c4trace.log 2>&1 || exit $?
cd $R && python3 tools/c4_timeline.py gpurun_out/c4trace || exit $?
run() {  # tag, args, env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u tools/cube_shard_time.py C4 --mode cube $args > gpurun_out/c4b_$tag.log 2>&1 || return $?
  echo "$tag [$args $*]"; grep '^{' gpurun_out/c4b_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  N=%d max %.1f ms mean %.1f eff %s' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
}
run l2 "--gpus 1,8" YRT_LANES=2 || exit $?
run l3 "--gpus 1,8" YRT_LANES=3 || exit $?
run l4 "--gpus 1,8" YRT_LANES=4 || exit $?
run c32 "--gpus 1,8 --capacity 33554432" YRT_LANES=2 || exit $?
run c32l4 "--gpus 1,8 --capacity 33554432" YRT_LANES=4 || exit $?
