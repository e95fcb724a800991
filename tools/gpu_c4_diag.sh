#!/bin/bash
# GPU-box: C4 diagnostics — k_shade phase profile of one stereo face (YRT_SHADE_PROF build in
# yulio-raytracer_amd/lib_prof_sprof) and PMC passes of the C4 cube job's kernels.
# usage: tools/gpu_c4_diag.sh <tag>
export TMPDIR=/tmp
TAG=${1:-c4d}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/c4d_$TAG
mkdir -p $OUT
cd $R && YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_prof_sprof timeout -k 10 200 python -u tools/shade_profile.py C4 1536 256 > $OUT/shade_prof.txt 2>&1
rc=$?; echo "shade profile rc=$rc"; cat $OUT/shade_prof.txt | tail -10
[ $rc -ne 0 ] && exit $rc
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
     python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 1 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
  python3 - $OUT/p$i <<'PY'
import csv, sys
from collections import defaultdict
from pathlib import Path
f = next(Path(sys.argv[1]).rglob("*counter_collection.csv"))
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    k = "trace_any" if "k_trace<true" in k else "trace_closest" if "k_trace<false" in k else "shade" if "k_shade" in k else "raygen" if "k_raygen" in k else "resolve" if "k_resolve" in k else None
    if k is None: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r.get("Dispatch_Id", ""))
for k, c in sorted(acc.items()):
    d = max(len(n[k]), 1)
    extra = ""
    if "SQ_ACTIVE_INST_VALU" in c and "GRBM_GUI_ACTIVE" in c:
        extra = f" valu_busy={4 * c['SQ_ACTIVE_INST_VALU'] / (1024 * c['GRBM_GUI_ACTIVE'] / 8):.3f} wait_any/wave_cycles={c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f} valu_per_wave={c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.0f}"
    print(f"  {k:14s} dispatches={d} " + " ".join(f"{x}={v / d:.4g}" for x, v in sorted(c.items())) + extra)
PY
done
exit 0
