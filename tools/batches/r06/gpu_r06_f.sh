# round-6 batch F: (1) the two-rays-per-lane any-hit kernel on the quantized nodes (any2 =
# -DYRT_ANY2=1, 118 VGPRs, 4 waves/SIMD) — parity first (GPU parity tests on that build), then
# same-box A/B; (2) a 16-entry any-hit LDS ring (a16: 72 VGPRs -> 7 waves/SIMD instead of the
# LDS-bound 4.75); (3) the float nodes for the any-hit traversal (fany) on C5, where round 6 is
# 4 % slower than round 5 (batch E); (4) ray-stream statistics of head vs the round-5 reciprocals
# (ieee: non-finite rays, visits per query) and the YRT_PROFILE wave-step counters of both.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
V=$R/yulio-raytracer_amd/lib_variants
YRT_LIB_DIR=$V/any2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_any2_r06f.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_any2_r06f.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_any2_r06f.log
for v in head ieee; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$V/$v"
  env $envs timeout -k 10 300 python -u tools/ray_stream_stats.py 512 16 1048576 > gpurun_out/raystats_${v}_r06f.txt 2>&1 || exit $?
  grep -v '^{' gpurun_out/raystats_${v}_r06f.txt | cut -c1-400
done
for v in prof prof_ieee; do
  YRT_LIB_DIR=$V/$v timeout -k 10 120 python tools/trace_profile.py 1024 > gpurun_out/trace_profile_${v}_r06f.txt 2>&1 || exit $?
  echo "== $v"; cat gpurun_out/trace_profile_${v}_r06f.txt
done
bash tools/gpu_ab_cfg.sh r06f "head|-|" "any2|any2|" "any2r96|any2r96|" "a16|a16|" "fany|fany|" \
  "head2|-|" "any2b|any2|" "a16b|a16|" "fanyb|fany|" || exit $?
for v in head any2 a16 fany r5; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$V/$v"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_f_$v.json > gpurun_out/c5_f_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_f_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-300
done
