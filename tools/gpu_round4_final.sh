# round-4 end-state evidence, part 1: a same-box A/B of the depth-0 choice and the round-3 build,
# the GPU suite, PMC passes of the C3 bench workload (-> profiles/pmc_c3.json), the default bench
# line reading them and its rocprof split (part 2: tools/gpu_round4_final2.sh)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r4f}
bash tools/gpu_ab_cfg.sh ${T}ab "auto|-|" "never|-|YRT_PRIMARY=0" "r3|r3|" || exit $?
timeout -k 10 480 python -u -m pytest tests -m gpu -q --maxfail=12 --timeout 200 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_$T.log | tail -n 14
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_pmc.sh $T || exit $?
mkdir -p profiles && cp gpurun_out/pmc_$T/pmc.json profiles/pmc_c3.json
timeout -k 10 400 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit $?
cut -c1-240 gpurun_out/bench_$T.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$T -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof_$T.json 2> $R/gpurun_out/bench_prof_$T.err || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_$T 6
