# round-5 batch AA: is rank 0's slower C3 N = 8 share its tiles or its place in the timing loop?
# ranks timed in the order 3, 0, 5, 0
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/cube_shard_time.py C3 --gpus 8 --ranks 3,0,5 > gpurun_out/c3aa_a.txt 2>&1 || exit 1
grep 'rank' gpurun_out/c3aa_a.txt | grep -v '^{'
timeout -k 10 300 python -u tools/cube_shard_time.py C3 --gpus 8 --ranks 0,3,0 > gpurun_out/c3aa_b.txt 2>&1 || exit 1
grep 'rank' gpurun_out/c3aa_b.txt | grep -v '^{'
