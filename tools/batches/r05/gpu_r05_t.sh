# round-5 batch T: wavefront batch capacity with four lanes — 32 / 48 / 64 (default) / 96 M paths
# per batch, same box, twice: C3 bench (5 steps) and the C4 cube job (N=1, N=8 shares)
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in a b; do
  for cap in 33554432 50331648 67108864 100663296; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --capture 0 --capacity $cap > gpurun_out/cap_c3_${cap}_$rep.json 2>/dev/null || exit 1
    timeout -k 10 200 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,8 --capacity $cap > gpurun_out/cap_c4_${cap}_$rep.log 2>&1 || exit 1
    python3 - gpurun_out/cap_c3_${cap}_$rep.json gpurun_out/cap_c4_${cap}_$rep.log "$cap $rep" <<'PY'
import json, sys
c3 = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c4 = {json.loads(l)["n"]: json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")}
print("cap %-14s C3 %.1f Mrays/s %.2f ms  C4 N=1 %.1f ms N=8 max %.1f mean %.1f" % (sys.argv[3], c3["value"], c3["ms_per_step"], c4[1]["ms_max"], c4[8]["ms_max"], c4[8]["ms_mean"]))
PY
  done
done
