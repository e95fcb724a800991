# round-5 batch S: more wavefront lanes than HIP's default 4 hardware queues — 6 and 8 lanes
# (lib_variants/l8, -DYRT_MAX_LANES=8) with GPU_MAX_HW_QUEUES=8, against the 4-lane default
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab_cfg.sh r05s "l4|-|" "l4q8|-|GPU_MAX_HW_QUEUES=8" "l6q8|l8|GPU_MAX_HW_QUEUES=8 YRT_LANES=6" \
  "l8q8|l8|GPU_MAX_HW_QUEUES=8 YRT_LANES=8" "l4b|-|" "l8q8b|l8|GPU_MAX_HW_QUEUES=8 YRT_LANES=8" || exit $?
