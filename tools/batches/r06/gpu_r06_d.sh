# round-6 batch D: where the reference reciprocals cost on C4 — one-lane kernel stats of the C4
# cube job (tools/cube_shard_time.py C4 --mode cube --gpus 1) for the default build and the
# round-5 reciprocals (ieee), and of C3 for both; then the bench A/B head / ieee / rsqint (the
# batch-B rsqrtps: v_rsq estimate + 64-bit integer check) twice.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06d.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r06d.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r06d.log
for v in head ieee; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v"
  cd /tmp && env $envs YRT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4l1_${v}_r06d -o run -- \
    python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 1 > $R/gpurun_out/c4l1_${v}_r06d.log 2>&1 || exit $?
  cd $R && python3 tools/kstats_csv.py gpurun_out/prof_c4l1_${v}_r06d 8 > gpurun_out/kstats_c4l1_${v}_r06d.txt 2>&1; echo "== C4 $v"; head -8 gpurun_out/kstats_c4l1_${v}_r06d.txt
  cd /tmp && env $envs YRT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3l1_${v}_r06d -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 2 --capture 0 > $R/gpurun_out/c3l1_${v}_r06d.json 2>&1 || exit $?
  cd $R && python3 tools/kstats_csv.py gpurun_out/prof_c3l1_${v}_r06d 8 > gpurun_out/kstats_c3l1_${v}_r06d.txt 2>&1; echo "== C3 $v"; head -6 gpurun_out/kstats_c3l1_${v}_r06d.txt
done
for v in head ieee; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v"
  cd $R && env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_d_$v.json > gpurun_out/c5_d_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_d_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-300
done
bash tools/gpu_ab_cfg.sh r06d "head|-|" "ieee|ieee|" "rsqint|rsqint|" "head2|-|" "ieee2|ieee|" "rsqint2|rsqint|" || exit $?
