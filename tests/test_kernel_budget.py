"""Register / scratch budgets of the built gfx950 kernels (CPU only: the code object's metadata,
tools/code_object_resources.py). The traversal kernels' occupancy is part of their design
(DESIGN §3, §5): since round 6 every 64-lane block holds a 16-entry (4 KB) LDS stack ring, so
registers set the occupancy — 8 waves/SIMD for any-hit rays (<= 64 VGPRs), 6 for closest-hit
rays (<= 80), 5 for the fused depth 0 (<= 96) — and a kernel above its budget (or one that
spills) silently loses waves."""
from pathlib import Path
import shutil
import sys

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))

from code_object_resources import DEFAULT_LIB, LLVM, kernel_resources  # noqa: E402

pytestmark = pytest.mark.skipif(not DEFAULT_LIB.exists() or not (LLVM / "clang-offload-bundler").exists()
                                or shutil.which("c++filt") is None,
                                reason="device library not built or ROCm LLVM tools absent")


@pytest.fixture(scope="module")
def res():
    return kernel_resources(DEFAULT_LIB)


def test_trace_kernels_fit_their_waves(res):
    trace = {k: v for k, v in res.items() if "k_trace<" in k}
    # closest hit (static, moving), the fused depth 0, any hit (static, moving)
    assert len(trace) == 5, sorted(trace)
    for name, r in trace.items():
        # 512 VGPRs per SIMD lane slot / waves, 8-register granularity
        budget = 64 if "k_trace<true" in name else 96 if "k_trace<false, false, 1>" in name else 80
        assert r["vgpr"] <= budget, (name, r)
        assert r["lds"] <= 4228, (name, r)  # 16 entries x 64 lanes x 4 B + the queue map
        assert r["scratch"] == 0, (name, r)
    assert any("k_trace<false, false, 1>" in k for k in trace)


def test_shade_kernels_hold_four_waves(res):
    shade = {k: v for k, v in res.items() if "k_shade<" in k}
    assert shade
    for name, r in shade.items():
        if "8339454" in name:  # the generic every-material instantiation (2 waves, rare scenes)
            continue
        assert r["vgpr"] <= 128, (name, r)
        # round 6: no scratch at all (round 5's 12 / 16 B in C4's and the Collada set's
        # instantiations sat in rcp_rn's IEEE-division fallback, which the reference's rcp
        # sequence, yrt_sse_rcp.h, does not have)
        assert r["scratch"] == 0, (name, r)
