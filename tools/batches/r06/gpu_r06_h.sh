# round-6 batch H: default = 16-entry any-hit ring at 8 waves/SIMD (batch G). GPU parity tests on
# it; the GPU's reciprocal estimates against the Intel tables (all 2^32 inputs) on the br3 build
# (out-of-range inputs handled behind a ballot + uniform branch); then same-box A/B: br2 (the
# branch for rsqrtps only), br3 (both; 72 B scratch in the C4 shade kernel), c16 (16-entry
# closest-hit LDS ring, 79 VGPRs -> 6 waves/SIMD instead of LDS-bound 4.75), C3/C4 twice, C5 128 spp.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
V=$R/yulio-raytracer_amd/lib_variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_parity_r06h.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_parity_r06h.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_parity_r06h.log
YRT_LIB_DIR=$V/br3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread \
  -k "sse_estimates or c1 or c2 or c3 or c4 or hdri" > gpurun_out/pytest_gpu_br3_r06h.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_br3_r06h.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_br3_r06h.log
bash tools/gpu_ab_cfg.sh r06h "head|-|" "br2|br2|" "br3|br3|" "c16|c16|" "head2|-|" "br2b|br2|" "br3b|br3|" "c16b|c16|" || exit $?
for v in head br2 br3 c16 r5; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$V/$v"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_h_$v.json > gpurun_out/c5_h_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_h_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-300
done
