#!/bin/bash
# GPU-box: full default bench line, then the same command under rocprofv3 kernel trace.
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.err
rc=$?; echo "rocprof rc=$rc"; cat $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json
find $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -name "*stats*" | head
exit $rc
