# round-6 batch Q: a rank's share at N = 8 runs 4 concurrent lane batches of 1/32 of a frame;
# its mean (49.4 ms on C3) is 15 % above 1/8 of the whole frame (43 ms). Does the lane count
# (concurrent batches) change that? C3 and C4 N = 8 shares (tools/cube_shard_time.py, three
# repetitions, ranks 0-3) with YRT_LANES = 4 / 2 / 3 (4 is the most the device opens).
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in 4 2 3; do
  YRT_LANES=$L timeout -k 10 300 python -u tools/cube_shard_time.py C3 --gpus 8 --ranks 0,1,2,3 > gpurun_out/shares_c3_l${L}_r06q.txt 2>&1 || exit $?
  echo "C3 lanes $L: $(grep '^{' gpurun_out/shares_c3_l${L}_r06q.txt | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d["ms_max"], d["ms_mean"], d["ms_per_rank"])')"
  YRT_LANES=$L timeout -k 10 300 python -u tools/cube_shard_time.py C4 --mode cube --gpus 8 --ranks 0,1,2,3 > gpurun_out/shares_c4_l${L}_r06q.txt 2>&1 || exit $?
  echo "C4 lanes $L: $(grep '^{' gpurun_out/shares_c4_l${L}_r06q.txt | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d["ms_max"], d["ms_mean"], d["ms_per_rank"])')"
done
