#!/bin/bash
# GPU-box: default batch capacity 64 / 96 / 128 M paths (variants c064 / c096 / c128): C3 bench,
# C4 cube job at N = 1 and rank shares at N = 8, C5 at 64 spp, two rounds on one box.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for round in 1 2; do
  for v in c064 c096 c128; do
    d=$R/yulio-raytracer_amd/lib_variants/$v
    YRT_LIB_DIR=$d timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/capab_c3_$v.json 2> gpurun_out/capab_c3_$v.err
    rc=$?; echo "C3 $v rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/capab_c3_$v.json')); print(d['ms_per_step'], 'ms')" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
    YRT_LIB_DIR=$d timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --gpus 1,8 > gpurun_out/capab_c4_$v.log 2>&1
    rc=$?; echo "C4 $v rc=$rc $(grep '^{' gpurun_out/capab_c4_$v.log | python3 -c "import json,sys; print([(json.loads(l)['n'], json.loads(l)['ms_max']) for l in sys.stdin])")"
    [ $rc -ne 0 ] && exit $rc
    YRT_LIB_DIR=$d timeout -k 10 300 python -u tools/c5_profile.py --spp 64 --views 2 > gpurun_out/capab_c5_$v.log 2>&1
    rc=$?; echo "C5 $v rc=$rc $(grep '^{' gpurun_out/capab_c5_$v.log | cut -c40-90)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
