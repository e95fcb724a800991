# round-5 batch V: kernel timeline of a C3 rank-0 share at N = 8 (four lanes) under rocprofv3
# --kernel-trace: idle time of the job, kernels per lane (tools/c4_timeline.py)
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl_c3_n8 -o run -- \
  python3 $R/tools/cube_shard_time.py C3 --gpus 8 --ranks 0 > $R/gpurun_out/tl_c3_n8.log 2>&1 || exit $?
cd $R && python3 tools/c4_timeline.py gpurun_out/tl_c3_n8 > gpurun_out/tl_c3_n8.txt 2>&1; cat gpurun_out/tl_c3_n8.txt | head -30
