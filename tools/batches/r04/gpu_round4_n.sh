# round-4 batch N: the final tree — GPU suite, smoke(), and the default bench line
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -q --maxfail=12 --timeout 200 --timeout-method thread > gpurun_out/pytest_r4n.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_r4n.log | tail -n 14
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4n.log 2>&1 || { tail -5 gpurun_out/smoke_r4n.log; exit 1; }
tail -n 1 gpurun_out/smoke_r4n.log
timeout -k 10 400 python bench.py > gpurun_out/bench_r4n.json 2> gpurun_out/bench_r4n.err || exit $?
cut -c1-300 gpurun_out/bench_r4n.json
