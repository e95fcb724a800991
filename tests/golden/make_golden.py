"""Regenerates the golden fixtures of tests/golden from the oracle (CPU restatement).

    python tests/golden/make_golden.py

Fixtures: embree::Random sequences (KAT 1; also pinned independently by the pure-Python
restatement in tests/test_cpu_host.py), sample tables (KAT 2), per-tile pixel sample-set
indices, DebugRenderer id-hash image (KAT 3), hit records of 4096 incoherent closest and
occlusion queries on C2/C3 (KAT 4) and 64x64 RGB_FLOAT32 thumbnails of C1/C2/C4 (KAT 6). The reference itself cannot run here (Embree is binary-only for Windows, SURVEY
§8(c)), so these pin the restatement against regressions; parity at the Embree boundary
is unpinned.
"""
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "yulio-raytracer_amd"), str(ROOT / "tests")]

import oracle  # noqa: E402
import yrt  # noqa: E402
from helpers import c1_args, c2_args, c3_args, c4_args  # noqa: E402


def main():
    seeds = [1, 27, 3433, 81551, 91711, 16 * 91711 + 32 * 81551]
    (HERE / "random_ints.json").write_text(json.dumps({str(s): oracle.random_ints(s, 64).tolist() for s in seeds}))
    for spp, depth in [(1, 2), (16, 2), (64, 10)]:
        np.save(HERE / f"sample_table_spp{spp}_d{depth}.npy", oracle.sample_table(spp, 64, 0, depth, depth + 1))
    np.save(HERE / "pixel_sets_100x70.npy", oracle.pixel_sets(100, 70, 64))
    dev = yrt.Device(host=True)
    for name, args, face in [("c1_64", c1_args(64, 1), -1), ("c2_64", c2_args(64, 4), -1),
                             ("c4_face3_64", c4_args(64, 4), 3)]:
        s = yrt.Session(args + ["-fb", "RGB_FLOAT32"], device=dev)
        img, _ = oracle.render(s.export_frame(face), 64, 64, s.info()["gamma"])
        np.save(HERE / f"thumb_{name}.npy", img)
        s.close()
    s = yrt.Session(c2_args(64, 1) + ["-renderer", "debug", "-fb", "RGB_FLOAT32"], device=dev)
    img, _ = oracle.render(s.export_frame(), 64, 64, 1.0)
    np.save(HERE / "debug_c2_64.npy", img)
    s.close()
    # KAT 4: hit records of incoherent rays; every other occlusion query
    # with a finite tfar
    for name, args in [("c2", c2_args(32, 1)), ("c3", c3_args(32, 1))]:
        s = yrt.Session(args, device=dev)
        blob = s.export_frame()
        org4, dir4 = incoherent_rays(blob, 4096, seed=42)
        occ_dir = dir4.copy()
        occ_dir[::2, 3] = 50.0
        np.savez_compressed(HERE / f"hits_{name}_4096.npz", org=org4, dir=dir4, occ_dir=occ_dir,
                            hit=oracle.trace(blob, org4, dir4),
                            occ=oracle.trace(blob, org4, occ_dir, any_hit=True)[:, 3].view(np.int32))
        s.close()
    dev.close()


def incoherent_rays(blob, n, seed):
    """Origins uniform in the scene AABB, directions uniform on S^2, tnear 0, tfar inf."""
    tris = oracle.scene_triangles(blob).reshape(-1, 3, 3)
    lo, hi = tris.min(axis=(0, 1)), tris.max(axis=(0, 1))
    rng = np.random.default_rng(seed)
    org = rng.uniform(lo, hi, size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    org4 = np.concatenate([org, np.zeros((n, 1), np.float32)], 1).astype(np.float32)
    dir4 = np.concatenate([d.astype(np.float32), np.full((n, 1), np.inf, np.float32)], 1)
    return org4, dir4


if __name__ == "__main__":
    main()
