# round-6 batch B: the default build after batch A (rcpps by the float route + one corrected
# entry, rsqrtps arithmetic, no hit geometry id, quantized any-hit nodes). GPU suite; same-box A/B
# against the round-5 reciprocals (ieee) twice; PMC passes of the bench workload (with the VALU
# lane-utilization counter if rocprofv3 lists it); the -DYRT_PROFILE build's traversal lane
# counters; the default bench line under rocprofv3 --kernel-trace --stats.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06b.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r06b.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r06b.log
bash tools/gpu_ab_cfg.sh r06b "head|-|" "ieee|ieee|" "head2|-|" "ieee2|ieee|" || exit $?
bash tools/gpu_pmc.sh r06b || exit $?
YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/prof timeout -k 10 120 python tools/trace_profile.py 1024 > gpurun_out/trace_profile_r06b.txt 2>&1 || exit $?
cat gpurun_out/trace_profile_r06b.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench_r06b -o run -- \
  python3 $R/bench.py > $R/gpurun_out/bench_r06b.json 2> $R/gpurun_out/bench_r06b.err || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_bench_r06b 8 > gpurun_out/kstats_bench_r06b.txt 2>&1; head -8 gpurun_out/kstats_bench_r06b.txt
python3 -c "import json; d=json.load(open('gpurun_out/bench_r06b.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
