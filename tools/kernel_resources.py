#!/usr/bin/env python3
"""VGPRs, scratch and occupancy of every kernel in pathtrace.hip, from the compiler's
-Rpass-analysis=kernel-resource-usage remarks with the Makefile's flags (no GPU needed).

    python tools/kernel_resources.py [extra hipcc flags...]
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "yulio-raytracer_amd"


def main():
    flags = subprocess.run(["make", "-s", "-C", str(PKG), "-pn"], capture_output=True, text=True).stdout
    hip = re.search(r"^HIPFLAGS := (.*)$", flags, re.M)
    cxx = re.search(r"^CXXFLAGS := (.*)$", flags, re.M)
    env = {"OPT": "-O3", "EXTRA": "", "STACK": "64", "LDSSTACK": "16", "ARCH": "gfx950", "HIPEXTRA": ""}
    def expand(t):
        t = t.replace("$(CXXFLAGS)", cxx.group(1))
        for k, v in env.items():
            t = t.replace(f"$({k})", v)
        return t
    cmd = ["/opt/rocm/bin/hipcc"] + expand(hip.group(1)).split() + [a for a in sys.argv[1:] if a != "--raw"] + [
        "-Rpass-analysis=kernel-resource-usage", "-c", "csrc/kernels/pathtrace.hip", "-o", "/tmp/kr.o"]
    out = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True).stderr
    if "--raw" in sys.argv:
        print(out)
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    demangle = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                              text=True).stdout.splitlines()
    for r, d in zip(rows, demangle):
        d = re.sub(r"\(.*", "", d)
        print(f"{d[:60]:60s} vgpr {r.get('vgpr', '?'):>4} agpr {r.get('agpr', 0):>3} scratch {r.get('scratch', '?'):>4} "
              f"waves {r.get('occ', '?'):>2} lds {r.get('lds', '?')}")


if __name__ == "__main__":
    main()
