#!/bin/bash
# GPU-box: parity tests then the default bench (no CPU baseline), stop on crash.
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-dev}
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout 600 > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 gpurun_out/pytest_$TAG.log
[ $rc -ge 2 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
exit $rc
