#!/bin/bash
# GPU-box: C3 bench and C5 (64 spp, one view pair) for every built variant under
# yulio-raytracer_amd/lib_variants, two rounds back to back on one box.
# usage: tools/gpu_r3_ab2.sh <tag>
export TMPDIR=/tmp
TAG=${1:-ab2}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for round in 1 2; do
  for d in $R/yulio-raytracer_amd/lib_variants/*/; do
    v=$(basename $d)
    [ -f $d/libdevice_singleray_mi355x.so ] || continue
    YRT_LIB_DIR=$d timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c3_$v.json 2> gpurun_out/${TAG}_c3_$v.err
    rc=$?; echo "C3 $v rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_c3_$v.json')); print(d['ms_per_step'], 'ms', {k: round(x, 1) for k, x in d['roofline']['kernel_ms_per_step'].items()})" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
    YRT_LIB_DIR=$d timeout -k 10 300 python -u tools/c5_profile.py --spp 64 --views 2 > gpurun_out/${TAG}_c5_$v.log 2>&1
    rc=$?; echo "C5 $v rc=$rc $(grep '^{' gpurun_out/${TAG}_c5_$v.log | cut -c40-90)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
