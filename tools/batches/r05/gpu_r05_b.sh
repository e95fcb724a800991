# round-5 batch B: GPU suite + smoke after removing the rejected experiment paths (BVH8, shared
# shadow origins, paired appends, grid hints, taper, lane order, pending depth, eager readback)
# with the product's FMA vector helpers kept and the reference-arithmetic oracle compared under
# the §8(d) gate; then the same-box A/B against the round-4 end build.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r05b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu_r05b.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu_r05b.log | head -20; exit $rc; }
grep -E "reference arithmetic" gpurun_out/pytest_gpu_r05b.log | cut -c1-400
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05b.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke_r05b.log
bash tools/gpu_ab_cfg.sh r05b "r4|r4|" "head|-|" "r4b|r4|" "headb|-|"
# the C3 shadow-query streams (depths 0-2, 128^2 16 spp) for the CPU stack-depth experiment
timeout -k 10 200 python tools/dump_shadow_stream.py 128 16 > gpurun_out/dump_shadow_r05b.log 2>&1 || exit $?
tail -1 gpurun_out/dump_shadow_r05b.log
