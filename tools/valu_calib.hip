// valu_calib.hip — calibration of the VALU-busy formula used for the bench roofline.
//
// A pure-VALU kernel: every lane runs 8 independent FMA chains (no memory traffic inside the
// loop), 8 waves per SIMD on all 256 CUs, so the SIMDs' vector issue is saturated. Its PMC
// pass (tools/gpu_pmc.sh) fixes the normalisation of SQ_ACTIVE_INST_VALU against
// GRBM_GUI_ACTIVE that DESIGN.md §3 uses: busy = 4 * SQ_ACTIVE_INST_VALU /
// (SIMDs * GRBM_GUI_ACTIVE / XCDs) should read ~1 here (see tools/pmc_json.py).
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_calib.hip -o tools/valu_calib
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void k_valu_calib(float* out, int iters, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < iters; ++i) {
    a0 = __builtin_fmaf(a0, s, 1.0f); a1 = __builtin_fmaf(a1, s, 1.0f);
    a2 = __builtin_fmaf(a2, s, 1.0f); a3 = __builtin_fmaf(a3, s, 1.0f);
    a4 = __builtin_fmaf(a4, s, 1.0f); a5 = __builtin_fmaf(a5, s, 1.0f);
    a6 = __builtin_fmaf(a6, s, 1.0f); a7 = __builtin_fmaf(a7, s, 1.0f);
  }
  const float r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (r == 12345.0f) out[blockIdx.x * 256 + threadIdx.x] = r;  // keeps the chains live
}

int main() {
  float* out = nullptr;
  const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU -> 8 waves per SIMD
  if (hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 1 << 16;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(a);
    k_valu_calib<<<blocks, 256>>>(out, iters, 0.999f);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double instr = (double)blocks * 4 * iters * 8;  // wave-level FMA instructions
    printf("valu_calib: %.3f ms, %.4g wave-FMA/s\n", ms, instr / (ms * 1e-3));
  }
  hipFree(out);
  return 0;
}
