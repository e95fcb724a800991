# round-6 batch A: the reference's rcp/rsqrt (Intel rcpps/rsqrtps emulated exactly + math.h's
# Newton steps) in the product and the oracle, and the closest-hit kernels' hit geometry id
# (k_shade loads the geometry record beside the shading record). GPU suite on the default build,
# then same-box A/B of the C4 cube job / C3 bench: ieee (-DYRT_IEEE_RCP, round-5 arithmetic),
# rsqarith (-DYRT_RSQ_ARITH, table-free rsqrtps), nohg (-DYRT_NO_HIT_GEOM), twice each.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06a.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r06a.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r06a.log
bash tools/gpu_ab_cfg.sh r06a "head|-|" "ieee|ieee|" "arith|rsqarith|" "nohg|nohg|" "head2|-|" "ieee2|ieee|" "arith2|rsqarith|" "nohg2|nohg|" || exit $?
