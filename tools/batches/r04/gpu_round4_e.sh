# round-4 batch E: GPU suite with the per-scene depth-0 choice, and a same-box A/B of the
# choice (auto) against never (YRT_PRIMARY=0) and always (YRT_PRIMARY=2) fused
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -q --maxfail=12 --timeout 200 --timeout-method thread > gpurun_out/pytest_r4e.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_r4e.log | tail -n 14
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_ab_cfg.sh r4e "auto|-|" "never|-|YRT_PRIMARY=0" "always|-|YRT_PRIMARY=2" "mp3|mp3|" "auto_again|-|"
