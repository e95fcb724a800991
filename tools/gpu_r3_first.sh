#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/r3a_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --stereo-frames 1 > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r3a_bench.json; tail -3 gpurun_out/r3a_bench.err
exit $rc
