# round-5 batch J: the fused depth-0 kernel at 96 VGPRs / 5 waves (register target 5, miss
# radiance read from the render parameters, traced count after the loop, v_mbcnt lane ranks).
# head: rays stored with their hit at completion (hits only); rA: rays stored at refill (every
# camera ray) and read by path id in k_shade; w6B: head at the old 6-wave target (100-104 VGPRs,
# 4 waves). GPU suite, same-box A/B (C4 cube job N=1 / N=8 shares, C3) with and without the
# identity layout (YRT_PRIMARY_IDENTITY=1), one-lane rocprof of the C4 cube job.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r05j.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r05j.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r05j.log
YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/rA timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_cubes.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "fused_primary or c4_stereo_face or cube_job_equals" > gpurun_out/pytest_rA_r05j.log 2>&1 \
  || { tail -30 gpurun_out/pytest_rA_r05j.log; exit 1; }
tail -1 gpurun_out/pytest_rA_r05j.log
bash tools/gpu_ab_cfg.sh r05j "base|base|" "head|-|" "rA|rA|" "w6B|w6B|" "headI|-|YRT_PRIMARY_IDENTITY=1" \
  "rAI|rA|YRT_PRIMARY_IDENTITY=1" "baseb|base|" "headb|-|" "rAb|rA|" || exit $?
for v in head base rA; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v"
  cd /tmp && env $envs YRT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4l1_$v -o run -- \
    python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 1 > $R/gpurun_out/c4l1_prof_$v.log 2>&1 || exit $?
  cd $R && python3 tools/kstats_csv.py gpurun_out/prof_c4l1_$v 10 > gpurun_out/kstats_c4l1_$v.txt 2>&1; head -8 gpurun_out/kstats_c4l1_$v.txt
done
for v in head headI; do
  envs=""; [ $v = headI ] && envs="YRT_PRIMARY_IDENTITY=1"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_j_$v.json > gpurun_out/c5_j_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_j_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-300
done
