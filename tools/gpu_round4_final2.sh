# round-4 end-state evidence, part 2: the C4 cube-job rank shares for N = 1, 2, 4, 8 and the C4
# kernel split, the N=2 gloo rehearsal line, every BASELINE config, and C5 render-only
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r4f}
timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,2,4,8 > gpurun_out/c4_$T.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,8 --capacity 134217728 > gpurun_out/c4cap_$T.log 2>&1 || exit $?
grep "^{" gpurun_out/c4cap_$T.log | cut -c1-200
grep '^{' gpurun_out/c4_$T.log | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4_$T -o run -- \
  python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 1 > $R/gpurun_out/prof_c4_$T.log 2>&1 || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_c4_$T 6
YRT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29543 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_n2_$T.json 2> gpurun_out/bench_n2_$T.err || exit $?
grep "^{" gpurun_out/bench_n2_$T.json | cut -c1-200
timeout -k 10 400 python -u tools/configs_bench.py > gpurun_out/configs_$T.txt 2>&1 || exit $?
tail -n 8 gpurun_out/configs_$T.txt
timeout -k 10 400 python -u tools/c5_bench.py --no-face --no-startrt --no-cpu --out gpurun_out/c5_$T.json > gpurun_out/c5_$T.log 2>&1 || exit $?
tail -n 2 gpurun_out/c5_$T.log | cut -c1-300
