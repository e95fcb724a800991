# round-5 batch O: shards deal the row-rotated raster order (a stride dividing the tiles per row
# dealt whole tile columns): GPU suite, C3 rank shares at N = 1/2/4/8 for both orders, same-box
# A/B (C4 cube job N=1 / N=8 shares, C3 bench) against the column deal (lib_variants/norot)
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r05o.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r05o.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r05o.log
for v in rot norot rotb norotb; do
  envs=""; case $v in norot*) envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/norot";; esac
  env $envs timeout -k 10 300 python -u tools/cube_shard_time.py C3 > gpurun_out/c3_shares_$v.txt 2>&1 || { tail -5 gpurun_out/c3_shares_$v.txt; exit 1; }
  echo "$v"; grep '^{' gpurun_out/c3_shares_$v.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('  N=%d max %.1f mean %.1f eff %.3f' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']), d['ms_per_rank'])"
done
bash tools/gpu_ab_cfg.sh r05o "rot|-|" "norot|norot|" "rotb|-|" "norotb|norot|" || exit $?
