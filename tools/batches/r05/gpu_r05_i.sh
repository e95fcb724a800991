# round-5 batch I: the fused depth-0 kernel at 94-95 VGPRs (rays stored at refill, miss radiance
# filled before the launch, traced count after the loop, v_mbcnt lane ranks): GPU suite, same-box
# A/B against the committed round-5 tree (base) and the ablations (mb0: popcount lane ranks;
# pw5: a 5-wave register target for the fused kernels), rocprof of the C4 cube job (head, base);
# PMC of the shading-order variant (ord, batch H's negative result).
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r05i.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r05i.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r05i.log
bash tools/gpu_ab_cfg.sh r05i "base|base|" "head|-|" "mb0|mb0|" "pw5|pw5|" "baseb|base|" "headb|-|" || exit $?
for v in head base; do
  envs=""; [ $v = base ] && envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/base"
  cd /tmp && env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4_$v -o run -- \
    python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 1 > $R/gpurun_out/c4_prof_$v.log 2>&1 || exit $?
  cd $R && python3 tools/kstats_csv.py gpurun_out/prof_c4_$v 10 > gpurun_out/kstats_c4_$v.txt 2>&1; head -8 gpurun_out/kstats_c4_$v.txt
done
YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/ord bash tools/gpu_pmc.sh ord_r05i || exit $?
