# round-6 batch E: round 6 against the round-5 end build on the same box — r5 = commit 0cd7790's
# sources built into lib_variants/r5 (IEEE reciprocals, float nodes everywhere, its own tuning).
# C4 cube job (N=1, N=8 shares) and C3 bench twice each, then the C5 1024-spp FPR cubemap once
# each (the north-star config).
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/gpu_ab_cfg.sh r06e "head|-|" "r5|r5|" "head2|-|" "r5b|r5|" || exit $?
for v in head r5; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v"
  env $envs timeout -k 10 400 python tools/c5_bench.py --no-face --no-startrt --no-cpu --out gpurun_out/c5_e_$v.json > gpurun_out/c5_e_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_e_$v.json')); print('$v C5 1024spp', d['render_cube_job'])" | cut -c1-300
done
