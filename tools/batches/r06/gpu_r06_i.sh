# round-6 batch I: (1) is the closest-hit kernel's 2.5-4 % per launch in head against the round-5
# reciprocals (identical ISA, identical wave steps, batches D and G) a clock effect? One PMC pass
# of GRBM_GUI_ACTIVE with the kernel trace, one lane, for each build, in both orders
# (tools/clock_check.py: busy cycles and implied MHz per launch). (2) any-hit triangles per leaf
# step 1 / 3 (tri1, tri3) against 2 and node bias 14 (b14) against 20 at 8 waves/SIMD; (3) batch H's
# 16-entry closest-hit ring (C4 -2.5 %, C3 -2 %) split: p16 = the fused depth-0 kernel's ring only,
# q16 = the queued closest-hit kernels' only. C3/C4 twice, C5 128 spp.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
V=$R/yulio-raytracer_amd/lib_variants
for v in head ieee ieee2 head2; do
  envs=""; case $v in ieee*) envs="YRT_LIB_DIR=$V/ieee";; esac
  cd /tmp && env $envs YRT_LANES=1 YRT_PRIMARY=0 timeout -k 10 -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d $R/gpurun_out/clk_${v}_r06i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --capture 0 --no-cpu-baseline > $R/gpurun_out/clk_${v}_r06i.log 2>&1 || exit $?
  cd $R && echo "== $v" && python3 tools/clock_check.py gpurun_out/clk_${v}_r06i 5 | tee gpurun_out/clk_${v}_r06i.txt
done
bash tools/gpu_ab_cfg.sh r06i "head|-|" "p16|p16|" "q16|q16|" "tri1|tri1|" "tri3|tri3|" "b14|b14|" "head2|-|" "p16b|p16|" "q16b|q16|" "tri1b|tri1|" "tri3b|tri3|" "b14b|b14|" || exit $?
for v in head p16 q16 tri1 tri3 b14; do
  envs=""; [ $v != head ] && envs="YRT_LIB_DIR=$V/$v"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_i_$v.json > gpurun_out/c5_i_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_i_$v.json')); print('$v C5 128spp', d['render_cube_job'])" | cut -c1-300
done
