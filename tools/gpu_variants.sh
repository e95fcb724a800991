#!/bin/bash
# GPU-box: default bench for every built variant under yulio-raytracer_amd/lib_variants.
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-var}
ARGS=${2:-"--no-cpu-baseline --steps 2"}
for d in yulio-raytracer_amd/lib_variants/*/; do
  v=$(basename $d)
  [ -f $d/libdevice_singleray_mi355x.so ] || continue
  YRT_LIB_DIR=$GRAFT_REPO_ROOT/$d timeout -k 10 300 python bench.py $ARGS > gpurun_out/var_${TAG}_$v.json 2> gpurun_out/var_${TAG}_$v.err
  rc=$?
  echo "$v rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/var_${TAG}_$v.json')); print(d['value'], d['roofline']['kernel_ms_per_step'])" 2>/dev/null)"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
