# round-4 batch G: the identity-layout fused depth 0 (YRT_PRIMARY=3) — its invariance test, then
# same-box C3 and C5 (64 spp) against k_raygen + the queued trace (YRT_PRIMARY=0)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "fused_primary or batch_capacity" --timeout 200 --timeout-method thread > gpurun_out/pytest_r4g.log 2>&1 || { tail -20 gpurun_out/pytest_r4g.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_r4g.log
for p in 0 3 0 3; do
  cd /tmp && YRT_PRIMARY=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ksg_prim$p -o run -- \
      python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 --capture 0 > $R/gpurun_out/ksg_prim$p.json 2> $R/gpurun_out/ksg_prim$p.err || exit $?
  cd $R && echo "== C3 YRT_PRIMARY=$p $(python3 -c "import json; d=json.load(open('gpurun_out/ksg_prim$p.json')); print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step')")"
  python3 tools/kstats_csv.py gpurun_out/ksg_prim$p 5
done
for p in 0 3; do
  YRT_PRIMARY=$p timeout -k 10 300 python -u tools/cube_shard_time.py C5 --mode cube --spp 64 --gpus 1,1 > gpurun_out/c5g_$p.log 2>&1 || exit $?
  echo "C5 64spp YRT_PRIMARY=$p"; grep '^{' gpurun_out/c5g_$p.log | cut -c1-130
done
