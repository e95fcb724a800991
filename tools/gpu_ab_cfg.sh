# Same-box A/B of library variants and env settings on the C4 cube job (one GPU: N=1 and the
# N=8 rank shares) and the C3 bench (5 steps).
# usage: tools/gpu_ab_cfg.sh <tag> "<name>|<lib variant or ->|<env assignments>" ...
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
TAG=$1; shift
for spec in "$@"; do
  IFS='|' read -r name lib envs <<< "$spec"
  libenv=""
  [ "$lib" != "-" ] && libenv="YRT_LIB_DIR=$R/yulio-raytracer_amd/lib_variants/$lib"
  t=${TAG}_$name
  env $libenv $envs timeout -k 10 200 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,8 > gpurun_out/ab_c4_$t.log 2>&1 || exit $?
  env $libenv $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --capture 0 > gpurun_out/ab_c3_$t.json 2> gpurun_out/ab_c3_$t.err || exit $?
  python3 - gpurun_out/ab_c4_$t.log gpurun_out/ab_c3_$t.json "$name [$lib $envs]" <<'PY'
import json, sys
c4 = {json.loads(l)["n"]: json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")}
c3 = json.load(open(sys.argv[2]))
print("%-34s C4 N=1 %.1f ms  N=8 max %.1f ms (eff %.3f)   C3 %.1f Mrays/s %.2f ms/step" % (
    sys.argv[3], c4[1]["ms_max"], c4[8]["ms_max"], c4[8]["predicted_efficiency"], c3["value"], c3["ms_per_step"]))
PY
done
