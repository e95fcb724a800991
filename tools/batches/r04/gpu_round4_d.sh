# round-4 batch D: the fused depth-0 kernel against k_raygen + the queued trace (YRT_PRIMARY)
# on C3 (rocprof split), C4 and C5 at 64 spp (cube job, N = 1 and the N = 8 rank shares)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for p in 0 1; do
  cd /tmp && YRT_PRIMARY=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ks_prim$p -o run -- \
      python3 $R/bench.py --no-cpu-baseline --steps 3 --capture 0 > $R/gpurun_out/ks_prim$p.json 2> $R/gpurun_out/ks_prim$p.err || exit $?
  cd $R && echo "== C3 YRT_PRIMARY=$p $(python3 -c "import json; d=json.load(open('gpurun_out/ks_prim$p.json')); print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step')")"
  python3 tools/kstats_csv.py gpurun_out/ks_prim$p 7
done
for p in 0 1 0 1; do
  YRT_PRIMARY=$p timeout -k 10 300 python -u tools/cube_shard_time.py C5 --mode cube --spp 64 --gpus 1,8 > gpurun_out/c5p_$p.log 2>&1 || exit $?
  echo "C5 64spp YRT_PRIMARY=$p"; grep '^{' gpurun_out/c5p_$p.log | cut -c1-130
done
for p in 0 1; do
  YRT_PRIMARY=$p timeout -k 10 200 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,8 > gpurun_out/c4p_$p.log 2>&1 || exit $?
  echo "C4 YRT_PRIMARY=$p"; grep '^{' gpurun_out/c4p_$p.log | cut -c1-130
done
