"""Writes tests/golden/sse_rcp_tables.json: the rcpps / rsqrtps tables of the CPU this runs on.

    make -C oracle ref && python tests/golden/make_sse_tables.py

The reference's rcp()/rsqrt() (common/math/math.h:38-59) start from the SSE estimate
instructions, whose tables are vendor-specific. The fixture records what an Intel CPU returns
(this container: "Intel(R) Xeon(R) Processor"): the 12-bit mantissa of rcpps(1 + i/2048) for the
2048 values of the top 11 input mantissa bits, and of rsqrtps(2^p (1 + j/1024)) for the 1024
values of the top 10 bits and both exponent parities — the instructions ignore the lower bits
(checked exhaustively by tests/test_ref_pin.py). The values come from oracle/_ref/libref_math.so
(ref_sse_tables, which executes the instructions). The product's exact emulation
(yulio-raytracer_amd/csrc/common/yrt_sse_rcp.h) is checked against this fixture on the CPU
(tests/test_ref_pin.py) and on the GPU (tests/test_gpu_parity.py), on any vendor's host.
"""
import ctypes as C
import json
import platform
import subprocess
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

import oracle  # noqa: E402


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_vendor():
    for line in Path("/proc/cpuinfo").read_text().splitlines():
        if line.startswith("vendor_id"):
            return line.split(":", 1)[1].strip()
    return "?"


def main():
    lib = C.CDLL(str(oracle.REF_MATH_LIB))
    rcp = np.zeros(2048, np.uint16)
    rsq = np.zeros(2048, np.uint16)
    special = np.zeros(12, np.float32)
    lib.ref_sse_tables(rcp.ctypes.data_as(C.c_void_p), rsq.ctypes.data_as(C.c_void_p),
                       special.ctypes.data_as(C.c_void_p))
    names = ["+0", "-0", "subnormal 0x5", "+inf", "-inf", "2^-126"]
    doc = {
        "cpu": cpu_model(), "vendor": cpu_vendor(),
        "rcpps_mantissa12": rcp.tolist(),
        "rsqrtps_mantissa12": rsq.tolist(),
        "special": {n: {"rcpps": float(special[2 * k]).hex(), "rsqrtps": float(special[2 * k + 1]).hex()}
                    for k, n in enumerate(names)},
    }
    (HERE / "sse_rcp_tables.json").write_text(json.dumps(doc))


if __name__ == "__main__":
    main()
