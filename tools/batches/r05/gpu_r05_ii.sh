# round-5 batch II: any-hit node bias 20 / 24 / 32 with any-hit refill 32 or 24 (batch HH: bias 24
# C3 +2.0 % but C5 +1.6 %; refill 32 takes C5 back) against 12 / 40 (head); C3 / C4 (gpu_ab_cfg)
# and C5 at 256 spp, same box, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/gpu_ab_cfg.sh r05ii "head|-|" "nba20a32|nba20a32|" "nba24a32|nba24a32|" "nba32a32|nba32a32|" "nba24a24|nba24a24|" "nba32|nba32|" "headb|-|" "nba20a32b|nba20a32|" "nba24a32b|nba24a32|" "nba32a32b|nba32a32|" "nba24a24b|nba24a24|" "nba32b|nba32|" || exit $?
for rep in a b; do
  for v in head nba20a32 nba24a32 nba32a32 nba24a24 nba32; do
    libenv=""; [ $v != head ] && libenv="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v"
    env $libenv timeout -k 10 300 python tools/c5_bench.py --spp 256 --no-face --no-startrt --no-cpu \
      --out gpurun_out/c5_r05ii_${v}_${rep}.json > gpurun_out/c5_r05ii_${v}_${rep}.log 2>&1 || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/c5_r05ii_${v}_${rep}.json')); print('C5 256spp $v $rep', d['render_cube_job']['seconds'])"
  done
done
