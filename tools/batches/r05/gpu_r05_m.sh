# round-5 batch M: one fused depth-0 instantiation (the identity layout and the pinhole-only
# kernel removed): GPU suite, same-box A/B against the round-5 base build on C4 / C3.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r05m.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r05m.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r05m.log
bash tools/gpu_ab_cfg.sh r05m "base|base|" "head|-|" "baseb|base|" "headb|-|" || exit $?
