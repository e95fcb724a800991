# round-5 batch EE: refill threshold 48 adopted — GPU suite, smoke, default bench line, C5 at 256 spp
# against the 40 build (lib_variants/r40), same box, alternating, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r05ee.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r05ee.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r05ee.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05ee.log 2>&1 || { tail -20 gpurun_out/smoke_r05ee.log; exit 1; }
tail -1 gpurun_out/smoke_r05ee.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r05ee.json 2> gpurun_out/bench_r05ee.err || { tail -20 gpurun_out/bench_r05ee.err; exit 1; }
cut -c1-200 gpurun_out/bench_r05ee.json
for rep in a b; do
  for v in head r40; do
    libenv=""; [ $v = r40 ] && libenv="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/r40"
    env $libenv timeout -k 10 300 python tools/c5_bench.py --spp 256 --no-face --no-startrt --no-cpu \
      --out gpurun_out/c5_r05ee_${v}_${rep}.json > gpurun_out/c5_r05ee_${v}_${rep}.log 2>&1 || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/c5_r05ee_${v}_${rep}.json')); print('C5 256spp $v $rep', d['render_cube_job'])" | cut -c1-200
  done
done
