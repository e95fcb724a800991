# round-5 batch JJ: on the any-hit retune (bias 20, refill 32) — any-hit triangles per leaf step
# 1 / 3 (default 2), any-hit node unroll 2, closest-hit node bias 12 / 16 (default 8); C3 / C4
# (gpu_ab_cfg) and C5 at 256 spp, same box, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/gpu_ab_cfg.sh r05jj "head|-|" "ts1|ts1|" "ts3|ts3|" "nu2|nu2|" "nb12|nb12|" "nb16|nb16|" "headb|-|" "ts1b|ts1|" "ts3b|ts3|" "nu2b|nu2|" "nb12b|nb12|" "nb16b|nb16|" || exit $?
for rep in a b; do
  for v in head ts1 ts3 nu2 nb12 nb16; do
    libenv=""; [ $v != head ] && libenv="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v"
    env $libenv timeout -k 10 300 python tools/c5_bench.py --spp 256 --no-face --no-startrt --no-cpu \
      --out gpurun_out/c5_r05jj_${v}_${rep}.json > gpurun_out/c5_r05jj_${v}_${rep}.log 2>&1 || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/c5_r05jj_${v}_${rep}.json')); print('C5 256spp $v $rep', d['render_cube_job']['seconds'])"
  done
done
