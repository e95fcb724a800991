# round-4 GPU batch A: the GPU suite and smoke on HEAD, the default bench line + its rocprof
# split, then same-box A/Bs (shadow origin index, C4 read-back / grid-hint pad, trace and shade
# variants)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 480 python -u -m pytest tests -m gpu -q --maxfail=12 --timeout 200 --timeout-method thread > gpurun_out/pytest_r4a.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_r4a.log | tail -n 14
# parity failures (rc 1) still leave the measurements below meaningful; anything else ends the batch
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4a.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke_r4a.log
timeout -k 10 400 python bench.py > gpurun_out/bench_r4a.json 2> gpurun_out/bench_r4a.err || exit $?
cut -c1-220 gpurun_out/bench_r4a.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r4a -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof_r4a.json 2> $R/gpurun_out/bench_prof_r4a.err || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_r4a 5
bash tools/gpu_env_ab.sh oi YRT_SHADOW_ORG_IDX=0 YRT_SHADOW_ORG_IDX=1 2 || exit $?
bash tools/batches/r04/gpu_round4_c4.sh || exit $?
bash tools/gpu_kstats.sh nu || exit $?
