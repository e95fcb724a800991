# round-5 batch E: PMC passes of the C3 frame with the two-ray any-hit kernel (YRT_ANY2=1) and
# the one-ray one (the record of the k_occluded negative result); same-box A/B of smaller LDS
# stack rings (the any-hit stack stays <= 8 entries for 99.9 % of C3 shadow queries,
# tools/anyhit_stack_exp.py): any-hit 16 / 8 entries (6 waves/SIMD), both kernels 16; and the
# closest-hit streams for the same CPU experiment.
export TMPDIR=/tmp
mkdir -p gpurun_out
YRT_ANY2=1 bash tools/gpu_pmc.sh any2_r05e || exit $?
bash tools/gpu_pmc.sh any1_r05e || exit $?
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_cfg.sh r05e "head|-|" "aL16|aL16|" "aL8|aL8|" "cL16|cL16|" "headb|-|" "aL16b|aL16|" "aL8b|aL8|" || exit $?
for t in head aL16 aL8 cL16 headb aL16b aL8b; do python3 -c "
import json; d=json.load(open('gpurun_out/ab_c3_r05e_$t.json')); k=d['roofline']['kernel_ms_per_step']
print('$t', 'closest %.1f shadow %.1f shade %.1f ms/step (HIP events, lanes overlap)' % (k['trace_closest'], k['trace_shadow'], k['shade']))"; done
timeout -k 10 200 python tools/dump_shadow_stream.py 128 16 > gpurun_out/dump_shadow_r05e.log 2>&1 || exit $?
tail -1 gpurun_out/dump_shadow_r05e.log
