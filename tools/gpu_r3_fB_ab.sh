#!/bin/bash
# GPU-box: round-3 evidence part B (tools/gpu_r3_finalB.sh) on the in-tree build, then a short
# C3 / C5 A/B of lib_variants/base against lib_variants/curS.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_r3_finalB.sh r3f || exit $?
for v in base curS base curS; do
  YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abS_c3_$v.json 2> gpurun_out/abS_c3_$v.err
  rc=$?; echo "C3 $v rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/abS_c3_$v.json')); print(d['ms_per_step'], 'ms', {k: round(x, 1) for k, x in d['roofline']['kernel_ms_per_step'].items()})" 2>/dev/null)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
