# round-6 batch U: PMC passes of the final tree (one lane, as the roofline frame) into profiles/pmc_c3.json, then the
# default bench line reading them.
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_pmc.sh r06u || exit $?
cp gpurun_out/pmc_r06u/pmc.json profiles/pmc_c3.json
timeout -k 10 600 python bench.py > gpurun_out/bench_r06u.json 2> gpurun_out/bench_r06u.err || { tail -20 gpurun_out/bench_r06u.err; exit 1; }
cut -c1-300 gpurun_out/bench_r06u.json
