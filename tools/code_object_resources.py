#!/usr/bin/env python3
"""Registers, scratch and LDS of every kernel in a built library, read from its gfx950 code
object (the .hip_fatbin section unbundled with clang-offload-bundler, metadata notes by
llvm-readelf) — what the GPU actually runs, no recompilation.

    python tools/code_object_resources.py [lib.so]      (default: the in-tree device library)
"""
from __future__ import annotations

import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
LLVM = Path("/opt/rocm/llvm/bin")
DEFAULT_LIB = ROOT / "yulio-raytracer_amd" / "lib" / "libdevice_singleray_mi355x.so"


def _demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    return [re.sub(r"\(.*", "", d) for d in out]


def kernel_resources(lib: Path = DEFAULT_LIB, arch: str = "gfx950") -> dict:
    """{demangled kernel name: {"vgpr", "sgpr", "scratch", "lds"}} of the library's code object."""
    with tempfile.TemporaryDirectory() as td:
        fat, co = Path(td) / "fat.bin", Path(td) / "co.o"
        subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(lib), str(Path(td) / "x")],
                       check=True, capture_output=True)
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o",
                        f"--targets=hipv4-amdgcn-amd-amdhsa--{arch}", f"--input={fat}", f"--output={co}"],
                       check=True, capture_output=True)
        notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], check=True, capture_output=True,
                               text=True).stdout
    # one kernel's metadata keys come in alphabetical order, its block opening with
    # `- .agpr_count` (.group_segment_fixed_size comes before .name)
    rows, cur = [], None
    keys = {".vgpr_count": "vgpr", ".sgpr_count": "sgpr", ".private_segment_fixed_size": "scratch",
            ".group_segment_fixed_size": "lds", ".name": "mangled"}
    for line in notes.splitlines():
        m = re.match(r"\s*(-?)\s*(\.[a-z_]+):\s+(\S+)", line)
        if not m:
            continue
        dash, k, v = m.groups()
        if dash and k == ".agpr_count":
            cur = {}
            rows.append(cur)
        elif cur is not None and k in keys and keys[k] not in cur:
            cur[keys[k]] = v if k == ".name" else int(v)
    rows = [r for r in rows if "mangled" in r]
    names = _demangle([r["mangled"] for r in rows])
    return {n: {k: r.get(k) for k in ("vgpr", "sgpr", "scratch", "lds")} for n, r in zip(names, rows)}


def main():
    lib = Path(sys.argv[1]) if len(sys.argv) > 1 else DEFAULT_LIB
    for name, r in kernel_resources(lib).items():
        print(f"{name[:60]:60s} vgpr {r['vgpr']:>4} sgpr {r['sgpr']:>4} scratch {r['scratch']:>4} lds {r['lds']}")


if __name__ == "__main__":
    main()
