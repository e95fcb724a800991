# round-4 same-box bisect of the C3 / C4 regression against the round-3 build: every variant
# under lib_variants (round-3 end, round-4 commits, shade-register variants) times the C4 cube
# job on one GPU (two samples) and the C3 bench (5 steps); r3 runs first and last
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
V=$R/yulio-raytracer_amd/lib_variants
one() {  # variant tag
  local v=$1 t=$2
  YRT_LIB_DIR=$V/$v timeout -k 10 200 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,1 > gpurun_out/bis_c4_$t.log 2>&1 || return $?
  YRT_LIB_DIR=$V/$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --capture 0 > gpurun_out/bis_c3_$t.json 2> gpurun_out/bis_c3_$t.err || return $?
  python3 - gpurun_out/bis_c4_$t.log gpurun_out/bis_c3_$t.json $t <<'PY'
import json, sys
c4 = [json.loads(l)["ms_max"] for l in open(sys.argv[1]) if l.startswith("{")]
c3 = json.load(open(sys.argv[2]))
print("%-10s C4 cube %s ms   C3 %.1f Mrays/s %.2f ms/step" % (sys.argv[3], " / ".join("%.1f" % x for x in c4), c3["value"], c3["ms_per_step"]))
PY
}
for v in r3 c_9fc4714 c_90c76bc c_03d0598 base cur nopair w3; do one $v $v || exit $?; done
one r3 r3_again || exit $?
