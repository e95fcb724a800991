# round-5 batch HH: any-hit node bias 16 (batch GG: C3 +1.1 %, C5 +0.4 %) and any-hit refill 32
# (GG: C5 -0.5 %) combined, and node bias 20 / 24, against 12 / 40 (head); C3 / C4 (gpu_ab_cfg)
# and C5 at 256 spp, same box, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/gpu_ab_cfg.sh r05hh "head|-|" "nba16|nba16|" "a32|a32|" "nba16a32|nba16a32|" "nba20|nba20|" "nba24|nba24|" "nba20a32|nba20a32|" "headb|-|" "nba16b|nba16|" "a32b|a32|" "nba16a32b|nba16a32|" "nba20b|nba20|" "nba24b|nba24|" "nba20a32b|nba20a32|" || exit $?
for rep in a b; do
  for v in head nba16 a32 nba16a32 nba20 nba24 nba20a32; do
    libenv=""; [ $v != head ] && libenv="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v"
    env $libenv timeout -k 10 300 python tools/c5_bench.py --spp 256 --no-face --no-startrt --no-cpu \
      --out gpurun_out/c5_r05hh_${v}_${rep}.json > gpurun_out/c5_r05hh_${v}_${rep}.log 2>&1 || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/c5_r05hh_${v}_${rep}.json')); print('C5 256spp $v $rep', d['render_cube_job']['seconds'])"
  done
done
