# round-6 batch O: trace grid (blocks per traversal launch) at the new occupancies (6 waves/SIMD
# closest hit, 8 any hit, three lanes): 32768 (g32k) and 8192 (g8k) against 16384. C3/C4 twice, C5 128 spp.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
V=$R/yulio-raytracer_amd/lib_variants
bash tools/gpu_ab_cfg.sh r06o "head|-|" "g32k|g32k|" "g8k|g8k|" "head2|-|" "g32kb|g32k|" "g8kb|g8k|" || exit $?
for v in head g32k g8k; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$V/$v"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_o_$v.json > gpurun_out/c5_o_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_o_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-300
done
