# round-4 GPU batch B: the round's evidence on HEAD — the GPU suite, PMC passes of the C3 bench
# workload (-> profiles/pmc_c3.json), the default bench line reading them and its rocprof split,
# a same-box A/B against the round-3 build (lib_variants/r3), the C4 cube-job shares, the N=2
# gloo rehearsal line, C5 render-only, and the 8-wide any-hit PMC pass
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 480 python -u -m pytest tests -m gpu -q --maxfail=12 --timeout 200 --timeout-method thread > gpurun_out/pytest_r4b.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_r4b.log | tail -n 14
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_pmc.sh r4b || exit $?
cp gpurun_out/pmc_r4b/pmc.json profiles/pmc_c3.json
timeout -k 10 400 python bench.py > gpurun_out/bench_r4b.json 2> gpurun_out/bench_r4b.err || exit $?
cut -c1-220 gpurun_out/bench_r4b.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r4b -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof_r4b.json 2> $R/gpurun_out/bench_prof_r4b.err || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_r4b 5
bash tools/gpu_kstats.sh r3ab || exit $?
for v in base r3; do
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 200 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,8 > gpurun_out/c4_r4b_$v.log 2>&1 || exit $?
  echo "C4 $v"; grep '^{' gpurun_out/c4_r4b_$v.log | cut -c1-160
done
YRT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_n2_r4b.json 2> gpurun_out/bench_n2_r4b.err || exit $?
grep "^{" gpurun_out/bench_n2_r4b.json | cut -c1-200
timeout -k 10 400 python -u tools/c5_bench.py --no-face --no-startrt --no-cpu --out gpurun_out/c5_r4b.json > gpurun_out/c5_r4b.log 2>&1 || exit $?
tail -n 2 gpurun_out/c5_r4b.log | cut -c1-300
YRT_ANY_BVH8=1 bash tools/gpu_pmc.sh w8
