# round-6 batch K: default = quantized nodes for both traversal kinds, 16-entry LDS rings
# everywhere (batch J). GPU suite on it; then the closest-hit kernel's tuning at this state: c8
# (8-entry ring), refill threshold 32 / 48 (cr32, cr48; 40 default), node bias 6 / 12 (cb6, cb12;
# 8 default): C3/C4 twice, C5 128 spp.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
V=$R/yulio-raytracer_amd/lib_variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06k.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r06k.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r06k.log
bash tools/gpu_ab_cfg.sh r06k "head|-|" "c8|c8|" "cr32|cr32|" "cr48|cr48|" "cb6|cb6|" "cb12|cb12|" \
  "head2|-|" "c8b|c8|" "cr32b|cr32|" "cr48b|cr48|" "cb6b|cb6|" "cb12b|cb12|" || exit $?
for v in head c8 cr32 cr48 cb6 cb12; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$V/$v"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_k_$v.json > gpurun_out/c5_k_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_k_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-300
done
