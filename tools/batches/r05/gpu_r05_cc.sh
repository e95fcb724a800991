# round-5 batch CC: refill threshold (40 default: 32 / 48) and closest-hit node bias (8 default:
# 6 / 10) re-swept with four lanes, same box, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh r05cc "head|-|" "r32|r32|" "r48|r48|" "nb6|nb6|" "nb10|nb10|" "headb|-|" "r32b|r32|" "r48b|r48|" "nb6b|nb6|" "nb10b|nb10|" || exit $?
