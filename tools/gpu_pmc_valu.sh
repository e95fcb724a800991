#!/bin/bash
# GPU-box: dynamic VALU/SALU/VMEM instruction counts per k_shade / k_trace item for every built
# variant under yulio-raytracer_amd/lib_variants (one rocprofv3 --pmc pass each, C3 one frame).
export TMPDIR=/tmp
TAG=${1:-pv}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for d in $R/yulio-raytracer_amd/lib_variants/*/; do
  v=$(basename $d)
  [ -f $d/libdevice_singleray_mi355x.so ] || continue
  cd /tmp && YRT_LIB_DIR=$d timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES \
      --output-format csv -d $R/gpurun_out/pv_${TAG}_$v -o run -- \
      python3 $R/bench.py --steps 1 --warmup 0 --capture 0 --no-cpu-baseline > $R/gpurun_out/pv_${TAG}_$v.json 2> $R/gpurun_out/pv_${TAG}_$v.err
  rc=$?
  echo "== $v rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 $R/tools/pmc_valu.py $R/gpurun_out/pv_${TAG}_$v $R/gpurun_out/pv_${TAG}_$v.json
done
exit 0
