# round-5 batch U: grid sizes re-swept with four lanes — trace grid 8192 / 32768 blocks (default
# 16384), shade grid 8192 (default 16384), same box, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh r05u "head|-|" "g8k|g8k|" "g32k|g32k|" "s8k|s8k|" "headb|-|" "g8kb|g8k|" "g32kb|g32k|" "s8kb|s8k|" || exit $?
