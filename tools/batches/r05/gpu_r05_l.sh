# round-5 batch L: k_shade phase breakdown on C3 and C4 (shader-clock cycles per phase, builds
# -DYRT_SHADE_PROF=1 / 2 in lib_variants/sprof1, sprof2; tools/shade_profile.py)
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for c in C3 C4; do
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/sprof1 timeout -k 10 200 python tools/shade_profile.py $c 1024 16 > gpurun_out/sprof1_$c.txt 2>&1 || { cat gpurun_out/sprof1_$c.txt; exit 1; }
  cat gpurun_out/sprof1_$c.txt
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/sprof2 timeout -k 10 200 python tools/shade_profile.py $c 1024 16 fine > gpurun_out/sprof2_$c.txt 2>&1 || { cat gpurun_out/sprof2_$c.txt; exit 1; }
  cat gpurun_out/sprof2_$c.txt
done
