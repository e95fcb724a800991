#!/bin/bash
# GPU-box: per-kernel average durations (rocprofv3 --kernel-trace --stats) of the default bench
# for every built variant under yulio-raytracer_amd/lib_variants (same box, back to back).
# usage: tools/gpu_kstats.sh <tag> ["<bench args>"]
export TMPDIR=/tmp
TAG=${1:-ks}
ARGS=${2:-"--no-cpu-baseline --steps 2 --capture 0"}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for d in $R/yulio-raytracer_amd/lib_variants/*/; do
  v=$(basename $d)
  [ -f $d/libdevice_singleray_mi355x.so ] || continue
  case $v in pathdbg|prof*) continue;; esac
  cd /tmp && YRT_LIB_DIR=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/gpurun_out/ks_${TAG}_$v -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/ks_${TAG}_$v.json 2> $R/gpurun_out/ks_${TAG}_$v.err
  rc=$?
  echo "== $v rc=$rc $(python3 -c "import json; d=json.load(open('$R/gpurun_out/ks_${TAG}_$v.json')); print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step')" 2>/dev/null)"
  [ $rc -ne 0 ] && exit $rc
  python3 $R/tools/kstats_csv.py $R/gpurun_out/ks_${TAG}_$v
done
exit 0
