# round-5 batch K: end-state evidence of the round-5 tree — GPU suite, smoke, PMC passes of the
# bench workload (-> profiles/pmc_c3.json, read by the bench line's roofline), the default bench
# line, the rocprof split of the same command (two lanes) and of one lane, every BASELINE config
# (tools/configs_bench.py), C4 strong-scaling prediction, C5 at its own size with the CPU port.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r05k.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r05k.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r05k.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05k.log 2>&1 || { tail -20 gpurun_out/smoke_r05k.log; exit 1; }
tail -2 gpurun_out/smoke_r05k.log
bash tools/gpu_pmc.sh final_r05k || exit $?
cp gpurun_out/pmc_final_r05k/pmc.json profiles/pmc_c3.json
timeout -k 10 600 python bench.py > gpurun_out/bench_r05k.json 2> gpurun_out/bench_r05k.err || { tail -20 gpurun_out/bench_r05k.err; exit 1; }
cut -c1-400 gpurun_out/bench_r05k.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r05k -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof_r05k.json 2>&1 || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_r05k 8
cd /tmp && YRT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_l1_r05k -o run -- \
  python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/bench_prof_l1_r05k.json 2>&1 || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_l1_r05k 6
timeout -k 10 600 python -u tools/configs_bench.py > gpurun_out/configs_r05k.txt 2>&1 || { tail -20 gpurun_out/configs_r05k.txt; exit 1; }
tail -6 gpurun_out/configs_r05k.txt | cut -c1-300
timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube > gpurun_out/scaling_prediction_c4_r05k.txt 2>&1 || exit $?
tail -4 gpurun_out/scaling_prediction_c4_r05k.txt | cut -c1-300
timeout -k 10 600 python tools/c5_bench.py --no-face --no-startrt --out gpurun_out/c5_render_r05k.json > gpurun_out/c5_render_r05k.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/c5_render_r05k.json')); print('C5', d['render_cube_job'], d['cpu_baseline'])" | cut -c1-500
