# round-4 batch C: GPU suite after the unfused triangle test / pipelined lanes / pair append
# off, a same-box A/B against the round-3 build (lane pipeline depth, tapered batches, the
# round-3 libm), and the C4 N=8 rank-share kernel timeline of the current build
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 480 python -u -m pytest tests -m gpu -q --maxfail=12 --timeout 200 --timeout-method thread > gpurun_out/pytest_r4c.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_r4c.log | tail -n 14
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_ab_cfg.sh r4c "r3|r3|" "cur|-|" "cur_pd1|-|YRT_PEND_DEPTH=1" "cur_taper|-|YRT_TAPER=1" "cur_noprim|-|YRT_PRIMARY=0" "oldlm|oldlm|" "r3_again|r3|" "cur_again|-|" || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c4trace_r4c -o run -- \
  python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 8 --ranks 0 > $R/gpurun_out/c4trace_r4c.log 2>&1 || exit $?
cd $R && python3 tools/c4_timeline.py gpurun_out/c4trace_r4c
