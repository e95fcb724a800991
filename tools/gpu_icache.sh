#!/bin/bash
# GPU-box: instruction-cache counters of the C3 bench kernels, two lanes (default) and one lane
# (YRT_LANES=1: no kernel overlap), one rocprofv3 --pmc pass each, to see whether the trace
# kernels' instruction-issue waits come from sharing a CU with k_shade's code.
# usage: tools/gpu_icache.sh <tag>
export TMPDIR=/tmp
TAG=${1:-ic}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ic_$TAG
mkdir -p $OUT
cd /tmp && timeout -k 10 -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1
grep -io "SQC_[A-Z_]*ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*" $OUT/avail.txt | sort -u > $OUT/names.txt
cat $OUT/names.txt | tr '\n' ' '; echo
C=""
for n in SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH; do
  grep -qx "$n" $OUT/names.txt && C="$C $n"
done
C="$C SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES"
echo "counters:$C"
for lanes in 2 1; do
  cd /tmp && YRT_LANES=$lanes timeout -k 10 -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/l$lanes -o run -- \
     python3 $R/bench.py --steps 1 --warmup 0 --capture 0 --no-cpu-baseline > $OUT/l$lanes.log 2>&1
  rc=$?; echo "lanes $lanes rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/l$lanes.log; exit $rc; }
  python3 - $OUT/l$lanes <<'PY'
import csv, sys
from collections import defaultdict
from pathlib import Path
f = next(Path(sys.argv[1]).rglob("*counter_collection.csv"))
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    k = "trace_any" if "k_trace<true" in k else "trace_closest" if "k_trace<false" in k else "shade" if "k_shade" in k else k.split("(")[0][-24:]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, c in acc.items():
    wc = c.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"  {k:24s} " + " ".join(f"{x}={v / max(len(n[k]), 1):.4g}" for x, v in sorted(c.items())) + f"  wait_inst/wave_cycles={c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}")
PY
done
exit 0
