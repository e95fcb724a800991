# round-6 batch G: the 16-entry any-hit LDS ring is the default now (batch F). GPU suite on it;
# one-lane kernel stats of C3 with the round-5 reciprocals FIRST and the default second (batch D
# ran them the other way round: is the closest-hit kernel's 4 % an ordering effect?); then the
# any-hit occupancy and tuning around the new ring: a8 (8 entries), a16w8 (8 waves/SIMD target,
# 64 VGPRs), a16r24 (refill 24), a16b28 (node bias 28) — C3/C4 A/B twice and C5 128 spp.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
V=$R/yulio-raytracer_amd/lib_variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06g.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r06g.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r06g.log
for v in ieee head; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$V/$v"
  cd /tmp && env $envs YRT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3l1_${v}_r06g -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 2 --capture 0 > $R/gpurun_out/c3l1_${v}_r06g.json 2>&1 || exit $?
  cd $R && python3 tools/kstats_csv.py gpurun_out/prof_c3l1_${v}_r06g 8 > gpurun_out/kstats_c3l1_${v}_r06g.txt 2>&1; echo "== C3 $v"; head -5 gpurun_out/kstats_c3l1_${v}_r06g.txt
done
bash tools/gpu_ab_cfg.sh r06g "head|-|" "a8|a8|" "a16w8|a16w8|" "a16r24|a16r24|" "a16b28|a16b28|" \
  "head2|-|" "a8b|a8|" "a16w8b|a16w8|" "a16r24b|a16r24|" "a16b28b|a16b28|" || exit $?
for v in head a8 a16w8 a16r24 a16b28 r5; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$V/$v"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_g_$v.json > gpurun_out/c5_g_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_g_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-300
done
