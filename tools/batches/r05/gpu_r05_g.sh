# round-5 batch G: k_shade over a hit queue sorted by triangle id (variant
# lib_variants/ssort, -DYRT_SHADE_SORT_EXP=1: per depth >= 1 a key pass + hipcub radix sort of
# (triangle id, queue slot), k_shade reads its queue through the sorted slots). Parity of the
# variant, rocprof kernel stats and PMC of C3 for both builds, frame A/B on C3, C4 and C5 (128 spp).
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
V=$R/yulio-raytracer_amd/lib_variants/ssort
YRT_LIB_DIR=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "c3_standin or c2_pathtracer or c3_full_size_band or c4_stereo_face" > gpurun_out/pytest_ssort_r05g.log 2>&1 || { tail -20 gpurun_out/pytest_ssort_r05g.log; exit 1; }
tail -1 gpurun_out/pytest_ssort_r05g.log
for v in head ssort; do
  envs=""; [ $v = ssort ] && envs="YRT_LIB_DIR=$V"
  cd /tmp && env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$v -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 --capture 0 > $R/gpurun_out/bench_prof_$v.json 2>&1 || exit $?
  cd $R && python3 tools/kstats_csv.py gpurun_out/prof_$v 12 > gpurun_out/kstats_$v.txt 2>&1; head -12 gpurun_out/kstats_$v.txt
done
cd $R
YRT_LIB_DIR=$V bash tools/gpu_pmc.sh ssort_r05g || exit $?
bash tools/gpu_ab_cfg.sh r05g "head|-|" "ssort|ssort|" "headb|-|" "ssortb|ssort|" || exit $?
for v in head ssort; do
  envs=""; [ $v = ssort ] && envs="YRT_LIB_DIR=$V"
  env $envs timeout -k 10 300 python tools/c5_bench.py --spp 128 --no-face --no-startrt --no-cpu --out gpurun_out/c5_$v.json > gpurun_out/c5_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c5_$v.json')); print('$v C5 128spp', {k: v for k, v in d.items() if 'cube' in k or 'ms' in k or 'Mrays' in k})" | cut -c1-400
done
# the roofline's launch time against rocprof: the default command on one wavefront lane
cd /tmp && YRT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_lanes1 -o run -- \
  python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 --capture 0 > $R/gpurun_out/bench_prof_lanes1.json 2>&1 || exit $?
cd $R && python3 tools/kstats_csv.py gpurun_out/prof_lanes1 6
# C5 at its own size: the 1024-spp cube job and the CPU port (round-5 tree)
timeout -k 10 600 python tools/c5_bench.py --no-face --no-startrt --out gpurun_out/c5_full_r05g.json > gpurun_out/c5_full_r05g.log 2>&1 || exit $?
tail -3 gpurun_out/c5_full_r05g.log | cut -c1-600
