#!/bin/bash
# GPU-box: same-box A/B of runtime switches (environment variables) on the default C3 bench:
# per setting one rocprofv3 kernel-stats run of bench.py, alternating A B A B.
# usage: tools/gpu_env_ab.sh <tag> "<ENV=a ...>" "<ENV=b ...>" [rounds] ["<bench args>"]
export TMPDIR=/tmp
TAG=${1:-envab}
A=${2:-""}
B=${3:-""}
ROUNDS=${4:-2}
ARGS=${5:-"--no-cpu-baseline --steps 3 --capture 0"}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for i in $(seq 1 $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then E="$A"; else E="$B"; fi
    out=$R/gpurun_out/ab_${TAG}_${v}$i
    cd /tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
      python3 $R/bench.py $ARGS > $out.json 2> $out.err
    rc=$?
    echo "== $v$i [$E] rc=$rc $(python3 -c "import json; d=json.load(open('$out.json')); print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step')" 2>/dev/null)"
    [ $rc -ne 0 ] && { tail -5 $out.err; exit $rc; }
    python3 $R/tools/kstats_csv.py $out 4
  done
done
exit 0
