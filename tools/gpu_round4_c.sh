# round-4 batch C: GPU suite after the unfused triangle test / pipelined lanes / pair append
# off, then a same-box A/B against the round-3 build and of the lane pipeline depth
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -q --maxfail=12 --timeout 200 --timeout-method thread > gpurun_out/pytest_r4c.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_r4c.log | tail -n 14
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_ab_cfg.sh r4c "r3|r3|" "cur|-|" "cur_pd1|-|YRT_PEND_DEPTH=1" "r3_again|r3|" "cur_again|-|"
