# round-6 batch C: the tree after batches A and B (reference reciprocals, quantized any-hit nodes, lane-utilization PMC) — GPU suite, smoke, the default bench line (with the CPU
# port), rocprof of the same command (four lanes) and of one lane, every BASELINE config, C3 / C4
# strong-scaling predictions on one GPU, C5 at its own size with the CPU port
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06c.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r06c.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r06c.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r06c.log 2>&1 || { tail -20 gpurun_out/smoke_r06c.log; exit 1; }
tail -1 gpurun_out/smoke_r06c.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r06c.json 2> gpurun_out/bench_r06c.err || { tail -20 gpurun_out/bench_r06c.err; exit 1; }
cut -c1-300 gpurun_out/bench_r06c.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06c -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof_r06c.json 2>&1 || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_r06c 6
cd /tmp && YRT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_l1_r06c -o run -- \
  python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/bench_prof_l1_r06c.json 2>&1 || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_l1_r06c 4
timeout -k 10 600 python -u tools/configs_bench.py > gpurun_out/configs_r06c.txt 2>&1 || { tail -20 gpurun_out/configs_r06c.txt; exit 1; }
tail -4 gpurun_out/configs_r06c.txt | cut -c1-200
timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube > gpurun_out/scaling_prediction_c4_r06c.txt 2>&1 || exit $?
grep '^{' gpurun_out/scaling_prediction_c4_r06c.txt | cut -c1-110
timeout -k 10 300 python -u tools/cube_shard_time.py C3 > gpurun_out/scaling_prediction_c3_r06c.txt 2>&1 || exit $?
grep '^{' gpurun_out/scaling_prediction_c3_r06c.txt | cut -c1-110
timeout -k 10 600 python tools/c5_bench.py --no-face --no-startrt --out gpurun_out/c5_render_r06c.json > gpurun_out/c5_render_r06c.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/c5_render_r06c.json')); print('C5', d['render_cube_job'], d['cpu_baseline'])" | cut -c1-400
