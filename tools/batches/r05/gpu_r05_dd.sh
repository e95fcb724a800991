# round-5 batch DD: refill threshold 48 (batch CC: C4 N = 8 share 47.8 / 47.5 against 48.2 / 48.4 ms,
# C3 level) split by kernel — closest 48 / any-hit 40, closest 40 / any-hit 48 — and 56, same box, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh r05dd "head|-|" "r48|r48|" "r56|r56|" "r48a40|r48a40|" "r40a48|r40a48|" "headb|-|" "r48b|r48|" "r56b|r56|" "r48a40b|r48a40|" "r40a48b|r40a48|" || exit $?
