# round-5 batch A: GPU suite + smoke on the working tree (namespace Yulio harness, bench --gpus
# spawn, multi-device shard clear, reference-order dot/cross/lmul), then a same-box A/B of the
# round-4 end build (lib_variants/r4) against HEAD on C3 (bench, 5 steps) and the C4 cube job.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r05a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu_r05a.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu_r05a.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05a.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke_r05a.log
bash tools/gpu_ab_cfg.sh r05a "r4|r4|" "head|-|" "r4b|r4|" "headb|-|"
