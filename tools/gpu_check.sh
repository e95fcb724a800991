#!/bin/bash
# GPU-box check: smoke, parity tests, short bench. Stops at the first crash/timeout
# (exit >= 124 or signal); ordinary test failures (exit 1) still let the bench run.
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 900 python -m pytest tests -m gpu -q -rA --timeout 600
run bench_small 300 python bench.py --size 512 --spp 16 --steps 2 --warmup 1 --cpu-rows 16
