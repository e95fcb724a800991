# round-4 batch P: PMC passes of the C4 cube job (one GPU; the fused depth-0 kernel reported
# apart) -> profiles/r04/pmc_c4_r04.json
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_c4
mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
     python3 $R/tools/cube_shard_time.py C4 --mode cube --gpus 1 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
done
cd $R && python3 tools/pmc_json.py $OUT $OUT/pmc.json > /dev/null && python3 - $OUT/pmc.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k, v in d.items():
    print("%-32s dispatches %5d valu_busy %.3f hbm/dispatch %.3f GB l2_hit %.3f wait_any %.2f" % (k, v.get("dispatches", 0), v.get("valu_busy", 0), v.get("hbm_bytes_per_dispatch", 0) / 1e9, v.get("l2_hit", 0), v.get("sq_wait_any_frac_of_wave_cycles", 0)))
PY
