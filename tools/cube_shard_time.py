#!/usr/bin/env python3
"""GPU-box: strong-scaling prediction of the stereo cubemaps on ONE GPU.

For N = 1, 2, 4, 8 the cubemap's 16x16 tiles are dealt round-robin over N ranks (SURVEY
§8(e)); this times rank r's share (yrtSetTileShard(r, N)) of one full cubemap, the way that
rank renders it in an N-GPU run, minus the RCCL gather. The predicted N-GPU time of a cubemap
is the slowest share; efficiency = T(1) / (N * T(N)).

  C4: test_stereo.ecs stereo cubemap, 12 x 1536^2 at 256 spp (non-FPR stereo branch,
      renderer.cpp:742-878)
  C5: the Frederick stand-in (yrt.frederick) FPR view, 12 x 1536^2 at 1024 spp (renderer.cpp:
      543-737: faceCamera update, scene commit, render)
  C3: the bench frame (Sponza stand-in 2048^2 at 64 spp): one rank's share of one frame, as
      bench.py's weak-scaling step renders it N times per step (--mode is ignored)

--mode face: one rtRenderFrame per face (the reference's loop);
--mode cube: the 12 faces in one yrtRenderFrames call (tiles of all faces in one sequence).
Times are render-only: the frames stay in HBM until mapped (as the product does) and are not
converted to numpy arrays. Each rank's share is rendered twice untimed first: the steady state of
an N-GPU run, where a rank renders the same share every frame.

usage: python tools/cube_shard_time.py C4|C5 [--mode face|cube] [--gpus 1,2,4,8] [--ranks all|0]
       [--spp N] [--size S]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "yulio-raytracer_amd"), str(ROOT), str(ROOT / "tests")]

import yrt  # noqa: E402


def session(cfg, dev, size, spp):
    if cfg == "C3":
        from helpers import c3_args
        return yrt.Session(c3_args(size, spp), device=dev)
    if cfg == "C4":
        from helpers import c4_args
        return yrt.Session(c4_args(size, spp), device=dev)
    from yrt import frederick
    dae = frederick.write_dae(ROOT / "scenes" / "_generated" / "frederick_c5" / "frederick.dae")
    return yrt.Session(["-fprCollada", "-faceCullingMode", "default", "-i", str(dae), "-stereo", "-size", str(size),
                        str(size), "-spp", str(spp), "-depth", "10", "-tMaxShadowRay", "120", "-ambientlight",
                        "0.83", "0.95", "0.98", "-toeIn"], device=dev)


def render_cube(ses, cfg, mode):
    """One full cubemap; returns rays traced (closest + shadow)."""
    dev = ses.device
    if cfg == "C3":  # one frame (bench.py's step at N = 1; at N GPUs each rank renders its share)
        ses.render(read=False)
        st = dev.render_stats()
        return st["raysClosest"] + st["raysShadow"]
    # render only: the frames are written back into the session's (host) framebuffers as the
    # product does, but not converted to numpy here
    if mode == "cube":
        if cfg == "C4":
            ses.render_cube(read=False)
        else:
            ses.render_scene_cube(0, read=False)
        st = dev.render_stats()
        return st["raysClosest"] + st["raysShadow"]
    rays = 0.0
    for f in range(12):
        if cfg == "C4":
            ses.render(f, read=False)
        else:
            ses.render_scene_camera(f, read=False)
        st = dev.render_stats()
        rays += st["raysClosest"] + st["raysShadow"]
    return rays


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg", choices=["C3", "C4", "C5"])
    ap.add_argument("--mode", choices=["face", "cube"], default="face")
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--ranks", default="all", help="'all' or a comma list of ranks to time")
    ap.add_argument("--size", type=int, default=1536)
    ap.add_argument("--spp", type=int, default=0, help="0: the config's own (C4 256, C5 1024)")
    ap.add_argument("--out", default="")
    ap.add_argument("--capacity", type=int, default=0, help="paths per wavefront batch (0: device default)")
    ap.add_argument("--reps", type=int, default=3,
                    help="timed renders per share; its time is their median (one render of a ~50 ms share "
                         "varies by a few ms from run to run, and the max over ranks picks that noise up)")
    a = ap.parse_args()
    spp = a.spp or {"C3": 64, "C4": 256, "C5": 1024}[a.cfg]
    if a.cfg == "C3" and a.size == 1536:
        a.size = 2048
    dev = yrt.Device(0)
    if a.capacity:
        dev.set_batch_capacity(a.capacity)
    ses = session(a.cfg, dev, a.size, spp)
    render_cube(ses, a.cfg, a.mode)  # untimed: allocations, sample table, BVH
    rows = []
    t1 = None
    for n in [int(x) for x in a.gpus.split(",")]:
        ranks = range(n) if a.ranks == "all" else [int(r) for r in a.ranks.split(",") if int(r) < n]
        times = {}
        spread = {}
        rays = 0.0
        if n > 1:  # untimed: the share's batch size reallocates the path queues once
            dev.set_tile_shard(0, n)
            render_cube(ses, a.cfg, a.mode)
        for r in ranks:
            dev.set_tile_shard(r, n)
            if n > 1:
                # untimed: a rank of an N-GPU run renders the same share every frame, so its
                # two frame blocks (render k+1 writes the block render k's unread frames do
                # not hold) already hold zeros outside the share (device.cpp FrameBlock::zeroKey)
                for _ in range(2):
                    render_cube(ses, a.cfg, a.mode)
            reps = []
            for _ in range(max(1, a.reps)):
                t = time.perf_counter()
                rays_r = render_cube(ses, a.cfg, a.mode)
                reps.append(time.perf_counter() - t)
            rays += rays_r
            times[r] = sorted(reps)[len(reps) // 2]
            spread[r] = (min(reps), max(reps))
            print(f"{a.cfg} {a.mode} N={n} rank {r}: {times[r] * 1e3:.1f} ms (median of {len(reps)}: "
                  f"{', '.join(f'{x * 1e3:.1f}' for x in reps)})", flush=True)
        tmax = max(times.values())
        if n == 1:
            t1 = tmax
        row = {"config": a.cfg, "mode": a.mode, "capacity": a.capacity or "default", "n": n, "ranks_timed": list(times), "ms_max": round(tmax * 1e3, 1),
               "ms_mean": round(sum(times.values()) / len(times) * 1e3, 1),
               "ms_per_rank": {str(k): round(v * 1e3, 1) for k, v in times.items()},
               "ms_per_rank_min_max": {str(k): [round(v[0] * 1e3, 1), round(v[1] * 1e3, 1)] for k, v in spread.items()},
               "reps": a.reps, "max_over_mean": round(tmax / (sum(times.values()) / len(times)), 4),
               "predicted_efficiency": round(t1 / (n * tmax), 3) if t1 else None,
               "Mrays_per_s_per_gpu": round(rays / sum(times.values()) / 1e6, 1)}
        # (the per-rank time is the median of --reps renders; rays are those of the last one)
        rows.append(row)
        print(json.dumps(row), flush=True)
    dev.set_tile_shard(0, 1)
    ses.close()
    dev.close()
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text("\n".join(json.dumps(r) for r in rows) + "\n")


if __name__ == "__main__":
    main()
