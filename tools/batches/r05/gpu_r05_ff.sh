# round-5 batch FF: refill threshold 48 per instantiation (batch EE: 48 everywhere C5 +1.6 %) —
# fused depth 0 only (p48), any hit only (a48), both (p48a48), everywhere (all48) against 40;
# C3 / C4 (gpu_ab_cfg) and C5 at 256 spp, same box, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/gpu_ab_cfg.sh r05ff "head|-|" "p48|p48|" "a48|a48|" "p48a48|p48a48|" "all48|all48|" "headb|-|" "p48b|p48|" "a48b|a48|" "p48a48b|p48a48|" "all48b|all48|" || exit $?
for rep in a b; do
  for v in head p48 a48 p48a48 all48; do
    libenv=""; [ $v != head ] && libenv="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v"
    env $libenv timeout -k 10 300 python tools/c5_bench.py --spp 256 --no-face --no-startrt --no-cpu \
      --out gpurun_out/c5_r05ff_${v}_${rep}.json > gpurun_out/c5_r05ff_${v}_${rep}.log 2>&1 || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/c5_r05ff_${v}_${rep}.json')); print('C5 256spp $v $rep', d['render_cube_job']['seconds'])"
  done
done
