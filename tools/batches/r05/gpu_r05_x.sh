# round-5 batch X: batches enqueued step by step round-robin over the lanes (head) against whole
# batches per lane (lib_variants/whole): GPU suite, timeline of a C3 N = 8 share, C3 shares,
# same-box A/B (C4 cube job N=1 / N=8 shares, C3 bench), twice
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r05x.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r05x.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r05x.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl_c3_n8x -o run -- \
  python3 $R/tools/cube_shard_time.py C3 --gpus 8 --ranks 0 > $R/gpurun_out/tl_c3_n8x.log 2>&1 || exit $?
cd $R && python3 tools/c4_timeline.py gpurun_out/tl_c3_n8x > gpurun_out/tl_c3_n8x.txt 2>&1; head -16 gpurun_out/tl_c3_n8x.txt
for v in step whole; do
  envs=""; [ $v = whole ] && envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/whole"
  env $envs timeout -k 10 300 python -u tools/cube_shard_time.py C3 > gpurun_out/c3_shares_x_$v.txt 2>&1 || exit 1
  echo "$v"; grep '^{' gpurun_out/c3_shares_x_$v.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('  N=%d max %.1f mean %.1f eff %.3f' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
done
bash tools/gpu_ab_cfg.sh r05x "step|-|" "whole|whole|" "stepb|-|" "wholeb|whole|" || exit $?
