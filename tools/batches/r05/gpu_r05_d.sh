# round-5 batch D: as C, after putting dot / cross / L*v on the reference order (product and oracle)
# scenes' shadow query (and the cleanup of batch B); same-box A/B on C3 and C4: the round-4 end
# build, HEAD (k_occluded, 3 waves), HEAD with YRT_ANY2=0 (one-ray k_trace<true>), k_occluded at
# 4 waves (64 B scratch); the C3 shadow streams for the CPU stack-depth experiment.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r05d.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu_r05d.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu_r05d.log | head -20; exit $rc; }
grep -E "reference arithmetic" gpurun_out/pytest_gpu_r05d.log | cut -c1-300
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05d.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke_r05d.log
bash tools/gpu_ab_cfg.sh r05d "r4|r4|" "any2|-|" "any1|-|YRT_ANY2=0" "a2w4|a2w4|" "any2b|-|" "any1b|-|YRT_ANY2=0" || exit $?
for t in r4 any2 any1 a2w4 any2b any1b; do python3 -c "
import json; d=json.load(open('gpurun_out/ab_c3_r05d_$t.json')); k=d['roofline']['kernel_ms_per_step']
print('$t', 'closest %.1f shadow %.1f shade %.1f ms/step (HIP events, lanes overlap)' % (k['trace_closest'], k['trace_shadow'], k['shade']))"; done
timeout -k 10 200 python tools/dump_shadow_stream.py 128 16 > gpurun_out/dump_shadow_r05d.log 2>&1 || exit $?
tail -1 gpurun_out/dump_shadow_r05d.log
