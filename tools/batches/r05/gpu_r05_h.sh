# round-5 batch H: the shading order (launch_shade_order: counting sort of the live queue slots
# by a bin of the hit triangle id before k_shade at depth >= 1, in place of batch G's radix sort
# over the queue's capacity). GPU suite on the new tree, same-box A/B against queue order
# (YRT_SHADE_ORDER=0) and the bin-count / first-depth variants, rocprof of both orders.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r05h.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r05h.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r05h.log
bash tools/gpu_ab_cfg.sh r05h "order|-|" "queue|-|YRT_SHADE_ORDER=0" "od0|od0|" "b512|b512|" "b8k|b8k|" \
  "orderb|-|" "queueb|-|YRT_SHADE_ORDER=0" || exit $?
for v in order queue; do
  envs=""; [ $v = queue ] && envs="YRT_SHADE_ORDER=0"
  cd /tmp && env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_h_$v -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 --capture 0 > $R/gpurun_out/bench_prof_h_$v.json 2>&1 || exit $?
  cd $R && python3 tools/kstats_csv.py gpurun_out/prof_h_$v 12 > gpurun_out/kstats_h_$v.txt 2>&1; head -9 gpurun_out/kstats_h_$v.txt
  cd /tmp && env $envs YRT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_h1_$v -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 --capture 0 > $R/gpurun_out/bench_prof_h1_$v.json 2>&1 || exit $?
  cd $R && python3 tools/kstats_csv.py gpurun_out/prof_h1_$v 12 > gpurun_out/kstats_h1_$v.txt 2>&1; head -9 gpurun_out/kstats_h1_$v.txt
done
for v in order queue; do
  envs=""; [ $v = queue ] && envs="YRT_SHADE_ORDER=0"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_h_$v.json > gpurun_out/c5_h_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_h_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-300
done
