# round-6 batch P: sharded jobs cover image tiles through a fixed pseudo-random bijection
# (common/yrt_tile_scatter.h) instead of the round-robin columns, where C3's shard 2 of 8 cost
# 16 % above the mean (batch M). GPU suite (the sharded-composite and gather tests check the
# frames bit for bit), then the C3 / C4 rank shares on one GPU (tools/cube_shard_time.py, three
# repetitions) and the unsharded C3/C4 A/B against the previous build (lib_variants/rr, must be
# unchanged: N = 1 keeps the identity map).
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06p.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r06p.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r06p.log
timeout -k 10 300 python -u tools/cube_shard_time.py C3 --reps 3 > gpurun_out/scaling_prediction_c3_r06p.txt 2>&1 || exit $?
grep '^{' gpurun_out/scaling_prediction_c3_r06p.txt | cut -c1-400
timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --reps 3 > gpurun_out/scaling_prediction_c4_r06p.txt 2>&1 || exit $?
grep '^{' gpurun_out/scaling_prediction_c4_r06p.txt | cut -c1-400
bash tools/gpu_ab_cfg.sh r06p "head|-|" "rr|rr|" || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_r06p.json 2> gpurun_out/bench_r06p.err || { tail -20 gpurun_out/bench_r06p.err; exit 1; }
cut -c1-300 gpurun_out/bench_r06p.json
