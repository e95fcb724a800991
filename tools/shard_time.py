"""GPU-box: time of one rank's share of a weak-scaling step (tile shard rank 0 of N, N frames),
on one GPU, for the device library in YRT_LIB_DIR (tools/build_variants.sh)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "yulio-raytracer_amd"), str(ROOT)]
import yrt  # noqa: E402
from yrt import standin  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = yrt.Device(0)
ses = yrt.Session(["-i", str(standin.write_xml())] + standin.C3_ARGS + ["-size", "2048", "2048", "-spp", "64"],
                  device=dev)
i = ses.info()
cam = ses.camera()
dev.set_tile_shard(0, N)
for k in range(N):  # warmup: allocations, sample tables of every iteration
    dev.rtRenderFrame(i["renderer"], cam, i["scene"], i["tonemapper"], i["framebuffer"], 1 if k else 0)
t = time.perf_counter()
rays = 0.0
for k in range(N):
    dev.rtRenderFrame(i["renderer"], cam, i["scene"], i["tonemapper"], i["framebuffer"], 1 if k else 0)
    st = dev.render_stats()
    rays += st["raysClosest"] + st["raysShadow"]
dt = time.perf_counter() - t
print(f"shard 0/{N}: {dt * 1e3:.1f} ms per step, {rays / dt / 1e6:.1f} Mrays/s per GPU")
