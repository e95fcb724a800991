# round-6 batch A: the reference's rcp/rsqrt (Intel rcpps/rsqrtps emulated exactly + math.h's
# Newton steps) in the product and the oracle. GPU suite on the default build (rsqrtps via the
# 4 KB table), then same-box A/B of C4 cube job / C3 bench against the round-5 arithmetic
# (ieee: -DYRT_IEEE_RCP) and the table-free rsqrtps (rsqarith: -DYRT_RSQ_ARITH), twice each.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06a.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r06a.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r06a.log
bash tools/gpu_ab_cfg.sh r06a "lut|-|" "ieee|ieee|" "arith|rsqarith|" "lut2|-|" "ieee2|ieee|" "arith2|rsqarith|" || exit $?
