# round-4 batch O: the fused depth-0 instantiations scheduled for 5 waves/SIMD (lib_variants/pw5:
# 96 VGPRs with 9-23 spilled) against the default build: C3 identity layout, C4 (compact)
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh r4o "cur_p0|-|YRT_PRIMARY=0" "cur_p3|-|YRT_PRIMARY=3" "pw5_p3|pw5|YRT_PRIMARY=3" "pw5|pw5|" "cur|-|" "cur_p0_again|-|YRT_PRIMARY=0"
