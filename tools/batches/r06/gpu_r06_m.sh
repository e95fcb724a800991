# round-6 batch M (end state, part 2): the default bench line (roofline as the VALU issue
# fraction, from the batch-L PMC passes now in profiles/pmc_c3.json), every BASELINE config, C3 / C4 strong-scaling predictions
# on one GPU (rank shares), C5 1024 spp with the CPU port, and the end state against the round-5
# build and against the round-5 reciprocals on the same box (C3/C4 twice).
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py > gpurun_out/bench_r06m.json 2> gpurun_out/bench_r06m.err || { tail -20 gpurun_out/bench_r06m.err; exit 1; }
cut -c1-300 gpurun_out/bench_r06m.json
timeout -k 10 600 python -u tools/configs_bench.py > gpurun_out/configs_r06m.txt 2>&1 || { tail -20 gpurun_out/configs_r06m.txt; exit 1; }
tail -4 gpurun_out/configs_r06m.txt | cut -c1-200
timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube > gpurun_out/scaling_prediction_c4_r06m.txt 2>&1 || exit $?
grep '^{' gpurun_out/scaling_prediction_c4_r06m.txt | cut -c1-110
timeout -k 10 300 python -u tools/cube_shard_time.py C3 > gpurun_out/scaling_prediction_c3_r06m.txt 2>&1 || exit $?
grep '^{' gpurun_out/scaling_prediction_c3_r06m.txt | cut -c1-110
timeout -k 10 600 python tools/c5_bench.py --no-face --no-startrt --out gpurun_out/c5_render_r06m.json > gpurun_out/c5_render_r06m.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/c5_render_r06m.json')); print('C5', d['render_cube_job'], d['cpu_baseline'])" | cut -c1-400
YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/r5 timeout -k 10 600 python tools/c5_bench.py --no-face --no-startrt --no-cpu --out gpurun_out/c5_render_r5_r06m.json > gpurun_out/c5_render_r5_r06m.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/c5_render_r5_r06m.json')); print('C5 r5', d['render_cube_job'])" | cut -c1-300
bash tools/gpu_ab_cfg.sh r06m "head|-|" "r5|r5|" "ieee|ieee|" "head2|-|" "r5b|r5|" "ieee2|ieee|" || exit $?
