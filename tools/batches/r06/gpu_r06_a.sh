# round-6 batch A: (1) the reference's rcp/rsqrt (Intel rcpps/rsqrtps emulated exactly + math.h's
# Newton steps) in the product and the oracle; (2) the closest-hit kernels' hit geometry id
# (k_shade loads the geometry record beside the shading record); (3) 64-B quantized nodes for
# the any-hit traversal. GPU suite on the default build, then same-box A/B of the C4 cube job /
# C3 bench against one-macro variants: ieee (-DYRT_IEEE_RCP, round-5 arithmetic), rsqarith
# (-DYRT_RSQ_ARITH), nohg (-DYRT_NO_HIT_GEOM), fp32any (-DYRT_QNODES_ANY=0), qclose
# (-DYRT_QNODES_CLOSEST=1), twice each; one-lane kernel stats of head / fp32any / qclose / nohg.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r06a.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r06a.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r06a.log
bash tools/gpu_ab_cfg.sh r06a "head|-|" "ieee|ieee|" "arith|rsqarith|" "nohg|nohg|" "fp32any|fp32any|" "qclose|qclose|" \
  "head2|-|" "ieee2|ieee|" "arith2|rsqarith|" "nohg2|nohg|" "fp32any2|fp32any|" "qclose2|qclose|" || exit $?
for v in head fp32any qclose nohg; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$v"
  cd /tmp && env $envs YRT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3l1_$v -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 2 --capture 0 > $R/gpurun_out/c3l1_$v.json 2> $R/gpurun_out/c3l1_$v.err || exit $?
  cd $R && python3 tools/kstats_csv.py gpurun_out/prof_c3l1_$v 8 > gpurun_out/kstats_c3l1_$v.txt 2>&1; echo "== $v"; head -6 gpurun_out/kstats_c3l1_$v.txt
done
