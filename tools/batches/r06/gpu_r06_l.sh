# round-6 batch L (end state, part 1): GPU suite, smoke, PMC passes of the bench workload (kept
# as profiles/pmc_c3.json, which the bench line reads), the default bench line (with the CPU
# port), rocprof of the same command (four lanes) and of one lane, the YRT_PROFILE lane counters.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06l.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r06l.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r06l.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r06l.log 2>&1 || { tail -20 gpurun_out/smoke_r06l.log; exit 1; }
tail -1 gpurun_out/smoke_r06l.log
bash tools/gpu_pmc.sh r06l || exit $?
cp gpurun_out/pmc_r06l/pmc.json profiles/pmc_c3.json
timeout -k 10 600 python bench.py > gpurun_out/bench_r06l.json 2> gpurun_out/bench_r06l.err || { tail -20 gpurun_out/bench_r06l.err; exit 1; }
cut -c1-300 gpurun_out/bench_r06l.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06l -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof_r06l.json 2>&1 || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_r06l 6 | tee gpurun_out/kstats_bench_r06l.txt
cd /tmp && YRT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_l1_r06l -o run -- \
  python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/bench_prof_l1_r06l.json 2>&1 || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_l1_r06l 5 | tee gpurun_out/kstats_l1_r06l.txt
YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/prof timeout -k 10 120 python tools/trace_profile.py 1024 > gpurun_out/trace_profile_r06l.txt 2>&1 || exit $?
cat gpurun_out/trace_profile_r06l.txt
