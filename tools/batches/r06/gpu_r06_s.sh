# round-6 batch S (final): three lanes by default (batch R). GPU suite, smoke, the default bench
# line with the CPU port, rocprof of the same command and of one lane, C5 1024 spp with the CPU
# port, C3 / C4 rank-share predictions.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06s.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r06s.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r06s.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r06s.log 2>&1 || { tail -20 gpurun_out/smoke_r06s.log; exit 1; }
tail -1 gpurun_out/smoke_r06s.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r06s.json 2> gpurun_out/bench_r06s.err || { tail -20 gpurun_out/bench_r06s.err; exit 1; }
cut -c1-300 gpurun_out/bench_r06s.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06s -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof_r06s.json 2>&1 || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_r06s 6 | tee gpurun_out/kstats_bench_r06s.txt
cd /tmp && YRT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_l1_r06s -o run -- \
  python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/bench_prof_l1_r06s.json 2>&1 || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_l1_r06s 5 | tee gpurun_out/kstats_l1_r06s.txt
timeout -k 10 600 python tools/c5_bench.py --no-face --no-startrt --out gpurun_out/c5_render_r06s.json > gpurun_out/c5_render_r06s.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/c5_render_r06s.json')); print('C5', d['render_cube_job'], d['cpu_baseline'])" | cut -c1-400
timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube > gpurun_out/scaling_prediction_c4_r06s.txt 2>&1 || exit $?
grep '^{' gpurun_out/scaling_prediction_c4_r06s.txt | cut -c1-200
timeout -k 10 300 python -u tools/cube_shard_time.py C3 > gpurun_out/scaling_prediction_c3_r06s.txt 2>&1 || exit $?
grep '^{' gpurun_out/scaling_prediction_c3_r06s.txt | cut -c1-200
