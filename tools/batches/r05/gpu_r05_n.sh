# round-5 batch N: C3 rank shares at N = 1/2/4/8 on one GPU (the bench line's weak-scaling step
# renders one share per frame per rank), with 2 (default), 3 and 4 wavefront lanes
export TMPDIR=/tmp
mkdir -p gpurun_out
for l in 2 3 4; do
  YRT_LANES=$l timeout -k 10 300 python -u tools/cube_shard_time.py C3 > gpurun_out/c3_shares_l$l.txt 2>&1 || { tail -5 gpurun_out/c3_shares_l$l.txt; exit 1; }
  echo "lanes $l"; grep '^{' gpurun_out/c3_shares_l$l.txt | cut -c1-200
done
