#!/bin/bash
# GPU-box, round-3 evidence part A: GPU suite, smoke(), the C3 PMC passes (-> pmc.json, which the
# bench line's roofline reads), the default bench line with the CPU baseline, and the same
# command under rocprofv3 kernel stats.
# usage: tools/gpu_r3_finalA.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3f}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke_$TAG.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_pmc.sh $TAG || exit $?
cp gpurun_out/pmc_$TAG/pmc.json profiles/pmc_c3.json
cd $R && timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/bench_$TAG.json
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof_$TAG.json 2> $R/gpurun_out/bench_prof_$TAG.err
rc=$?; echo "rocprof rc=$rc"; cut -c1-200 $R/gpurun_out/bench_prof_$TAG.json
[ $rc -ne 0 ] && exit $rc
python3 $R/tools/kstats_csv.py $R/gpurun_out/prof_$TAG 6
exit 0
