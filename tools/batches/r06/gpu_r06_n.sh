# round-6 batch N: the queued closest-hit kernels at a 7-wave register target (cw7: 72 VGPRs, one
# 4-byte spill outside the node/leaf steps) against 6 (74 VGPRs): C3/C4 twice, C5 128 spp.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
V=$R/yulio-raytracer_amd/lib_variants
bash tools/gpu_ab_cfg.sh r06n "head|-|" "cw7|cw7|" "head2|-|" "cw7b|cw7|" || exit $?
for v in head cw7; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$V/$v"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_n_$v.json > gpurun_out/c5_n_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_n_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-300
done
