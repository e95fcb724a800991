# round-6 batch R: three wavefront lanes instead of four (batch Q: N = 8 shares C3 mean 44.1
# against 50.4 ms, C4 45.9 against 48.8). Unsharded C3 / C4 / C5 at 3 lanes (YRT_LANES=3)
# against 4, twice, and every rank's N = 8 share for both.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/gpu_ab_cfg.sh r06r "head|-|" "l3|-|YRT_LANES=3" "head2|-|" "l3b|-|YRT_LANES=3" || exit $?
for L in 4 3; do
  YRT_LANES=$L timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_r_l$L.json > gpurun_out/c5_r_l$L.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_r_l$L.json')); print('lanes $L C5 128spp', d['render_cube_job'])" | cut -c1-300
  YRT_LANES=$L timeout -k 10 300 python -u tools/cube_shard_time.py C3 --gpus 8 > gpurun_out/shares8_c3_l${L}_r06r.txt 2>&1 || exit $?
  echo "C3 N=8 lanes $L: $(grep '^{' gpurun_out/shares8_c3_l${L}_r06r.txt | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d["ms_max"], d["ms_mean"], d["ms_per_rank"])')"
done
