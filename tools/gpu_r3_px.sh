#!/bin/bash
# GPU-box: k_shade computes the pixel only for hits / backplate lookups (variant px) vs HEAD
# (base): C3 bench, C4 cube job, C5 64 spp, two rounds; then rocprof kernel splits of the C4
# cube job and of C5 at 64 spp on the HEAD build (end-of-round profiles).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/gpu_r3_ab3.sh px || exit $?
for w in C4 C5; do
  if [ $w = C4 ]; then CMD="$R/tools/cube_shard_time.py C4 --mode cube --gpus 1"; else CMD="$R/tools/c5_profile.py --spp 64"; fi
  cd /tmp && YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/base timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/gpurun_out/ks_end_$w -o run -- python3 $CMD > $R/gpurun_out/ks_end_$w.log 2>&1
  rc=$?; echo "rocprof $w rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 $R/tools/kstats_csv.py $R/gpurun_out/ks_end_$w 6
done
exit 0
