#!/bin/bash
# GPU-box: one rocprofv3 --pmc pass per argument group over the C3 bench workload (kernels are
# serialized under counter collection), printed per kernel as the mean per dispatch.
# usage: tools/gpu_pmc_pass.sh <tag> "<counters group 1>" ["<group 2>" ...]
export TMPDIR=/tmp
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcp_$TAG
mkdir -p $OUT
i=0
for grp in "$@"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
     python3 $R/bench.py --steps 1 --warmup 0 --capture 0 --no-cpu-baseline > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
  python3 - $OUT/p$i <<'PY'
import csv, sys
from collections import defaultdict
from pathlib import Path
f = next(Path(sys.argv[1]).rglob("*counter_collection.csv"))
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    k = "trace_any" if "k_trace<true" in k else "trace_closest" if "k_trace<false" in k else "shade" if "k_shade" in k else None
    if k is None: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r.get("Dispatch_Id", ""))
for k, c in sorted(acc.items()):
    print(f"  {k:14s} " + " ".join(f"{x}={v / max(len(n[k]), 1):.4g}" for x, v in sorted(c.items())))
PY
done
exit 0
