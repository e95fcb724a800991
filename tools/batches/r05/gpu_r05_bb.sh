# round-5 batch BB: band bounds balanced by the previous render's rays (head) against uniform
# bounds (lib_variants/nobal): GPU suite, C3 shares, same-box A/B (C4 cube job N=1 / N=8 shares,
# C3 bench) twice, C5 at 128 spp
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r05bb.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r05bb.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r05bb.log
for v in bal nobal balb nobalb; do
  envs=""; case $v in nobal*) envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/nobal";; esac
  env $envs timeout -k 10 300 python -u tools/cube_shard_time.py C3 > gpurun_out/c3_shares_bb_$v.txt 2>&1 || exit 1
  echo "$v"; grep '^{' gpurun_out/c3_shares_bb_$v.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('  N=%d max %.1f mean %.1f eff %.3f' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
done
bash tools/gpu_ab_cfg.sh r05bb "bal|-|" "nobal|nobal|" "balb|-|" "nobalb|nobal|" || exit $?
for v in bal nobal; do
  envs=""; [ $v = nobal ] && envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/nobal"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_bb_$v.json > gpurun_out/c5_bb_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_bb_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-200
done
