#!/bin/bash
# GPU-box: GPU suite + smoke on the working tree (any-hit node bias 12), the default bench line,
# then C3 for any-hit node bias 12 / 16 / 24 (lib_variants), two rounds.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_nb.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 1 gpurun_out/pytest_gpu_nb.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_nb.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke_nb.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_nb.json 2> gpurun_out/bench_nb.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/bench_nb.json
[ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for v in nb12 nb16 nb24; do
    YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/nb_c3_$v.json 2> gpurun_out/nb_c3_$v.err
    rc=$?; echo "C3 $v rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/nb_c3_$v.json')); print(d['ms_per_step'], 'ms', {k: round(x, 1) for k, x in d['roofline']['kernel_ms_per_step'].items()})" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
