# round-5 batch Q: wavefront lanes 2 (default) / 3 / 4, same box, twice: C4 cube job N=1 / N=8
# shares and the C3 bench (tools/gpu_ab_cfg.sh), C5 at 128 spp
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh r05q "l2|-|" "l4|-|YRT_LANES=4" "l3|-|YRT_LANES=3" "l2b|-|" "l4b|-|YRT_LANES=4" "l3b|-|YRT_LANES=3" || exit $?
for v in l2 l4 l2b l4b; do
  envs=""; case $v in l4*) envs="YRT_LANES=4";; esac
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_q_$v.json > gpurun_out/c5_q_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_q_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-200
done
