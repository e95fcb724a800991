# round-5 batch Z: C3 N = 8 shares (four lanes) with 4 batches (default: one per lane), 8 and 12
# batches (two / three per lane: a lane that ends its band early takes the next), twice
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in a b; do
  for cap in 0 5000000 3000000; do
    a=""; [ $cap != 0 ] && a="--capacity $cap"
    timeout -k 10 300 python -u tools/cube_shard_time.py C3 --gpus 8 $a > gpurun_out/c3z_${cap}_$rep.txt 2>&1 || { tail -5 gpurun_out/c3z_${cap}_$rep.txt; exit 1; }
    grep '^{' gpurun_out/c3z_${cap}_$rep.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('cap $cap $rep N=%d max %.1f mean %.1f' % (d['n'], d['ms_max'], d['ms_mean']), d['ms_per_rank'])"
  done
done
