#!/bin/bash
# GPU-box: parity suite, then bench with the fused shadow resolve on and off, then the N=2
# multi-rank path rehearsed over gloo with both ranks on the one GPU.
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-fuse}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 > gpurun_out/${TAG}_on.json 2> gpurun_out/${TAG}_on.err
rc=$?; echo "bench fused rc=$rc"; [ $rc -ne 0 ] && exit $rc
YRT_NO_SHADOW_FUSE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 > gpurun_out/${TAG}_off.json 2> gpurun_out/${TAG}_off.err
rc=$?; echo "bench unfused rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 -c "
import json
for k in ('on','off'):
    d=json.load(open('gpurun_out/${TAG}_'+k+'.json')); print(k, d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
YRT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline --size 1024 > gpurun_out/${TAG}_n2.json 2> gpurun_out/${TAG}_n2.err
rc=$?; echo "n2 rc=$rc"; cat gpurun_out/${TAG}_n2.json; tail -3 gpurun_out/${TAG}_n2.err
exit $rc
