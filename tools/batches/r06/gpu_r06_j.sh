# round-6 batch J: default = any-hit ring 16 at 8 waves, fused depth-0 ring 16 (batches F-I).
# GPU suite; then the quantized nodes for the closest-hit traversal at this state: qc32 (32-entry
# ring, LDS-bound 4.75 waves/SIMD) and qc16 (16-entry ring, 74 VGPRs -> 6 waves/SIMD; the smaller
# node footprint may pay for the extra waves' cache interference that batch I's q16 lost to).
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
V=$R/yulio-raytracer_amd/lib_variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06j.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r06j.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r06j.log
bash tools/gpu_ab_cfg.sh r06j "head|-|" "qc32|qc32|" "qc16|qc16|" "head2|-|" "qc32b|qc32|" "qc16b|qc16|" || exit $?
for v in head qc32 qc16; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$V/$v"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_j_$v.json > gpurun_out/c5_j_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_j_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-300
done
