# round-5 batch W: host-side cost of enqueueing a batch — HIP API trace (rocprofv3 --hip-trace
# --kernel-trace, no counters) of a C3 rank-0 share at N = 8, four lanes
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $R/gpurun_out/ht_c3_n8 -o run -- \
  python3 $R/tools/cube_shard_time.py C3 --gpus 8 --ranks 0 > $R/gpurun_out/ht_c3_n8.log 2>&1 || exit $?
cd $R && ls gpurun_out/ht_c3_n8
