#!/usr/bin/env python3
"""GPU-box: StartRT on the cornell box at the DLL defaults, polling GetCurrentStatusRT (state,
progress, last error) every 0.25 s until it is done or 20 s have passed, then StopRT."""
import shutil
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "yulio-raytracer_amd")]
import yrt  # noqa: E402

d = Path(tempfile.mkdtemp())
for f in ("cornell_box.ecs", "cornell_box.obj", "cornell_box.mtl"):
    shutil.copy(ROOT / "scenes" / f, d / f)
p = yrt.InitParamsRT()
t0 = time.time()
print("StartRT", yrt.StartRT(d / "cornell_box.ecs", p), flush=True)
while time.time() - t0 < 20:
    st = yrt.GetCurrentStatusRT()
    print(f"{time.time() - t0:6.2f} s state {st.state} progress {st.progress:.3f} err {yrt.GetLastErrorRT()}", flush=True)
    if st.state in (3, 4):
        break
    time.sleep(0.25)
print("StopRT", yrt.StopRT(False), "WaitRT", yrt.WaitRT(), flush=True)
print(sorted(x.name for x in d.iterdir()))
