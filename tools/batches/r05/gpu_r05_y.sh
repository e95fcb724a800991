# round-5 batch Y: a shard's batches interleaved over its tiles (head: batch b = tiles b, b + nb, ...)
# against contiguous tile ranges (lib_variants/contig): GPU suite, timeline of a C3 N = 8 share,
# C3 shares, same-box A/B (C4 cube job N=1 / N=8 shares, C3 bench), twice, C5 at 128 spp
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r05y.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r05y.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r05y.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl_c3_n8y -o run -- \
  python3 $R/tools/cube_shard_time.py C3 --gpus 8 --ranks 0 > $R/gpurun_out/tl_c3_n8y.log 2>&1 || exit $?
cd $R && python3 tools/c4_timeline.py gpurun_out/tl_c3_n8y > gpurun_out/tl_c3_n8y.txt 2>&1; head -16 gpurun_out/tl_c3_n8y.txt
for v in inter contig; do
  envs=""; [ $v = contig ] && envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/contig"
  env $envs timeout -k 10 300 python -u tools/cube_shard_time.py C3 > gpurun_out/c3_shares_y_$v.txt 2>&1 || exit 1
  echo "$v"; grep '^{' gpurun_out/c3_shares_y_$v.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('  N=%d max %.1f mean %.1f eff %.3f' % (d['n'], d['ms_max'], d['ms_mean'], d['predicted_efficiency']))"
done
bash tools/gpu_ab_cfg.sh r05y "inter|-|" "contig|contig|" "interb|-|" "contigb|contig|" || exit $?
for v in inter contig; do
  envs=""; [ $v = contig ] && envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/contig"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_y_$v.json > gpurun_out/c5_y_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_y_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-200
done
