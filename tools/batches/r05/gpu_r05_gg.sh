# round-5 batch GG: any-hit refill threshold 32 / 36 / 44 and any-hit node bias 10 / 16 against 40 / 12 (batch FF: 48 costs C5 1.4 %)
# C3 / C4 (gpu_ab_cfg) and C5 at 256 spp, same box, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/gpu_ab_cfg.sh r05gg "head|-|" "a32|a32|" "a36|a36|" "a44|a44|" "nba10|nba10|" "nba16|nba16|" "headb|-|" "a32b|a32|" "a36b|a36|" "a44b|a44|" "nba10b|nba10|" "nba16b|nba16|" || exit $?
for rep in a b; do
  for v in head a32 a36 a44 nba10 nba16; do
    libenv=""; [ $v != head ] && libenv="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v"
    env $libenv timeout -k 10 300 python tools/c5_bench.py --spp 256 --no-face --no-startrt --no-cpu \
      --out gpurun_out/c5_r05gg_${v}_${rep}.json > gpurun_out/c5_r05gg_${v}_${rep}.log 2>&1 || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/c5_r05gg_${v}_${rep}.json')); print('C5 256spp $v $rep', d['render_cube_job']['seconds'])"
  done
done
