#!/bin/bash
# GPU-box: PMC passes of the C3 bench workload (-> pmc.json), then the default bench line reading
# it, and the same command under rocprofv3 kernel stats (tree already through the GPU suite).
# usage: tools/gpu_evidence_c3.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r3p}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/gpu_pmc.sh $TAG || exit $?
cp gpurun_out/pmc_$TAG/pmc.json profiles/pmc_c3.json
cd $R && timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/bench_$TAG.json
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof_$TAG.json 2> $R/gpurun_out/bench_prof_$TAG.err
rc=$?; echo "rocprof rc=$rc"; cut -c1-200 $R/gpurun_out/bench_prof_$TAG.json
[ $rc -ne 0 ] && exit $rc
python3 $R/tools/kstats_csv.py $R/gpurun_out/prof_$TAG 6
exit 0
