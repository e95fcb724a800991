#!/usr/bin/env python3
"""Headline benchmark: Mrays/s (+ samples/s) of the MI355X wavefront path tracer on the
BASELINE.json C3 workload — Sponza-class atrium stand-in (yrt.standin, seed 1234, 67 k tris,
Uber + Sponza JPEG textures, dome light 8 8 8), 2048x2048, 64 spp, depth 10,
tMaxShadowRay 120, camera of models/test_stereo_view.ecs:2-10.

One step = one full frame (all W*H*spp paths to termination) rendered through the C ABI
(yrtRenderFrame), scene resident in HBM. With N GPUs (torch.distributed launches one process
per GPU) the frame's 16x16 tiles are dealt round-robin over the ranks, each
rank renders its shard, and the device plugin gathers the tiles on rank 0 inside
rtRenderFrame with its own RCCL communicator (yrtSetShardComm: grouped send/recv of tile
slabs over xGMI); see setup_gather for the fallback.

Weak scaling: at N GPUs one step is N progressive iterations of that frame (AccuBuffer
accumulation, integratorrenderer.cpp:166), all tiles of all N iterations dealt round-robin;
per-GPU work stays one C3 frame. N=1 is exactly C3.

Counting: rays = closest-hit + shadow queries (numRays of
pathtraceintegrator.cpp:74,161); Mrays/s = rays of all ranks / max-over-ranks wall time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "yulio-raytracer_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md §HBM
L2_PEAK_GBS = 34500.0          # MI355X_MICROARCH.md §L2 (per XCD, 32 MiB aggregate): ≈34.5 TB/s
# node and triangle record bytes come from the scene (YRTSceneInfo nodeBytesClosest / nodeBytesAny:
# 128-B float nodes or 64-B quantized ones; triRecordBytes: GpuTri, 48)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--size", type=int, default=2048)
    p.add_argument("--spp", type=int, default=64)
    p.add_argument("--cpu-tile-stride", type=int, default=18,
                   help="CPU-baseline sample: the 16x16 tiles t %% N == 0 of the frame (0: a centred band of --cpu-rows)")
    p.add_argument("--cpu-rows", type=int, default=112, help="rows of the centred CPU-baseline band (--cpu-tile-stride 0)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--capture", type=int, default=4096,
                   help="rays per depth sampled for visit counts (0: no capture frame, e.g. PMC passes)")
    p.add_argument("--capacity", type=int, default=0, help="paths per wavefront batch (0: device default)")
    p.add_argument("--stereo-size", type=int, default=1536, help="cube face size (C4: 1536; smaller for tests)")
    p.add_argument("--stereo-spp", type=int, default=256, help="cube spp (C4: 256; smaller for tests)")
    p.add_argument("--stereo-frames", type=int, default=None,
                   help="C4 stereo cubemaps (12 x 1536^2 x 256spp, one job, tiles dealt over the ranks) timed "
                        "after the main loop and reported under 'stereo_cubemap' (median and min per cubemap). "
                        "Default: 6 at N>1 (the BASELINE 1/2/4/8-GPU cubemap, gather checked against a one-GPU "
                        "render), 0 at N=1 so a rocprof summary of the default command averages only the C3 "
                        "launches of the roofline kernel")
    return p.parse_args()


def launch_ranks(a):
    """`bench.py --gpus N` (N > 1) started without a launcher: this process has not touched the
    GPU (no torch import yet), so it starts the N ranks itself as the driver would —
    `python -m torch.distributed.run --nproc-per-node N bench.py <same arguments>` on 127.0.0.1 —
    lets rank 0's JSON line through on the shared stdout and exits with the launcher's status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ, YRT_BENCH_LAUNCHER="bench.py --gpus (torch.distributed.run child ranks)")
    return subprocess.run(cmd, env=env).returncode


def main():
    a = parse()
    if a.gpus < 1:
        sys.exit(f"--gpus {a.gpus}: at least one GPU")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        sys.exit(f"WORLD_SIZE={world} but --gpus {a.gpus}: the launcher's rank count and --gpus must agree")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    # YRT_DIST_BACKEND=gloo rehearses the N>1 path with several ranks on one GPU (ranks share
    # device local % device_count); the driver's multi-GPU runs use RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("YRT_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if a.stereo_frames is None:
        a.stereo_frames = 6 if world > 1 else 0
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    gpus_used = physical_gpus(world, local)

    import yrt
    from yrt import standin
    from yrt.dist import gather_frame
    xml = ROOT / "scenes" / "_generated" / f"sponza_standin_r{rank}.xml"
    standin.write_xml(xml)
    dev = yrt.Device(local)
    args = ["-i", str(xml)] + standin.C3_ARGS + ["-size", str(a.size), str(a.size), "-spp", str(a.spp)]
    ses = yrt.Session(args, device=dev)
    info = ses.info()
    cam = ses.camera()
    R, S, T, F = info["renderer"], info["scene"], info["tonemapper"], info["framebuffer"]
    sinfo = dev.scene_info(S)
    dev.set_tile_shard(rank, world)
    gather = setup_gather(dev, rank, world, backend) if world > 1 else "single GPU"
    if a.capacity:
        dev.set_batch_capacity(a.capacity)

    # ---- untimed capture frame: visit counts of the real query streams (roofline bytes)
    per_kind = {}
    if a.capture > 0:
        per_kind = visit_counts(a, dev, R, cam, S, T, F, sinfo)

    # ---- warmup + timed frames
    dev.set_kernel_timing(True)
    fb_t = None
    if world > 1:
        stride = (3 * a.size + 3) // 4 * 4
        fb_t = torch.empty(stride * a.size, dtype=torch.uint8, device="cuda" if backend == "nccl" else "cpu")

    def step():
        # weak scaling: the job is `world` progressive iterations of the C3 frame (sampler
        # iteration k = frame k); every frame's tiles are dealt round-robin over the ranks,
        # so each rank renders one frame's worth of tiles per step.
        st = None
        for k in range(world):
            dev.rtRenderFrame(R, cam, S, T, F, 1 if k else 0)
            s_k = dev.render_stats()
            st = s_k if st is None else {n: st[n] + s_k[n] for n in st}
        if world > 1 and not gather.startswith("C++"):
            import ctypes
            p = dev.rtMapFrameBuffer(F)
            host = np.ctypeslib.as_array((ctypes.c_uint8 * fb_t.numel()).from_address(p))
            fb_t.copy_(torch.from_numpy(host), non_blocking=False)
            dev.rtUnmapFrameBuffer(F)
            gather_frame(fb_t, dst=0)
        return st

    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    acc = {"rays": 0.0, "closest": 0.0, "shadow": 0.0, "samples": 0.0, "msClosest": 0.0, "msShadow": 0.0,
           "msShade": 0.0, "nClosest": 0.0, "nShadow": 0.0, "msRender": 0.0, "msGather": 0.0}
    for _ in range(a.steps):
        st = step()
        acc["closest"] += st["raysClosest"]
        acc["shadow"] += st["raysShadow"]
        acc["rays"] += st["raysClosest"] + st["raysShadow"]
        acc["msClosest"] += st["msTraceClosest"]
        acc["msShadow"] += st["msTraceShadow"]
        acc["msShade"] += st["msShade"]
        acc["nClosest"] += st["launchesClosest"]
        acc["nShadow"] += st["launchesShadow"]
        acc["msRender"] += st["msRender"]
        acc["msGather"] += st["msGather"]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    samples_total = float(a.size) * a.size * 2 ** int(np.ceil(np.log2(a.spp))) * a.steps * world

    red_dev = "cuda" if backend == "nccl" else "cpu"
    tot = torch.tensor([acc["rays"], acc["closest"], acc["shadow"]], dtype=torch.float64, device=red_dev)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    rays, closest, shadow = tot.tolist()
    elapsed = tmax.item()
    per_rank = rank_times(acc["msRender"] / a.steps, acc["msGather"] / a.steps, world, red_dev, gather)

    # one more frame, untimed, on one wavefront lane: no two kernels overlap, so its HIP-event
    # durations are each kernel's own (what a rocprof --kernel-trace summary averages); the
    # timed frames' per-kernel durations include the time a kernel shares the GPU with the other
    # lane's kernels. Single-rank runs only (every rank of N > 1 would have to join the gather).
    serial = None
    if world == 1:
        dev.set_lanes(1)
        dev.rtRenderFrame(R, cam, S, T, F, 0)
        serial = dev.render_stats()
        dev.set_lanes(0)  # back to the default (4, or YRT_LANES)

    stereo = stereo_cubemap(a, dev, rank, world, backend, gather, local, gpus_used) if a.stereo_frames > 0 else None

    if rank == 0:
        # dominant trace kernel: what binds it. The BVH and the
        # triangles are L2/MALL-resident, so the traversal is not HBM-bound: the roofline is
        # the VALU-issue one (PMC pass of this same config, profiles/pmc_c3.json), with the
        # counter-measured HBM bytes beside it; the SURVEY §8(d) algorithmic bytes are
        # reported as what they are (mostly L2/MALL hits), never as an HBM rate.
        kern = {
            "closest": (acc["msClosest"], acc["closest"], acc["nClosest"]),
            "shadow": (acc["msShadow"], acc["shadow"], acc["nShadow"]),
        }
        dom = max(kern, key=lambda k: kern[k][0])
        ms, nr, nl = kern[dom]
        avg_ms_overlapped = ms / max(nl, 1)
        avg_ms = avg_ms_overlapped
        if serial:
            # the one-lane frame's own launches, queries and time (its batches may be split
            # differently from the timed frames': ADVICE r5)
            sk = {"closest": ("msTraceClosest", "launchesClosest", "raysClosest"),
                  "shadow": ("msTraceShadow", "launchesShadow", "raysShadow")}[dom]
            avg_ms = serial[sk[0]] / max(serial[sk[1]], 1)
            nr, nl = serial[sk[2]], serial[sk[1]]
        kname = "k_trace<false>" if dom == "closest" else "k_trace<true>"
        alg = nr * per_kind[dom]["bytes_per_ray"] / max(nl, 1) if per_kind else None
        alg_gbs = alg / (avg_ms * 1e-3) / 1e9 if alg and avg_ms > 0 else None
        pmc, pmc_note = load_pmc(a, sinfo, world)
        kp = (pmc or {}).get("kernels", {}).get(kname, {})
        traffic = kp.get("hbm_bytes_per_dispatch")
        valu = kp.get("valu_issue_frac")
        hbm_gbs = traffic / (avg_ms * 1e-3) / 1e9 if traffic and avg_ms > 0 else None
        roof = {"bound": "valu-issue", "achieved": round(valu, 4) if valu is not None else None, "peak": 1.0,
                "unit": "fraction of the SIMDs' VALU issue cycles (2 per wave64 VALU instruction on a 32-wide "
                        "SIMD; SQ_INSTS_VALU, tools/pmc_json.py)",
                "frac": round(valu, 4) if valu is not None else None,
                "traffic": round(traffic) if traffic else None,
                "kernel": "k_trace_closest" if dom == "closest" else "k_trace_any",
                "launches": int(nl), "avg_launch_ms": round(avg_ms, 4),
                "avg_launch_ms_note": ("the kernel alone: a one-lane frame after the timed ones (rocprof-consistent); "
                                       "avg_launch_ms_overlapped is the timed frames' HIP-event average, which includes "
                                       "the other lane's concurrent kernels") if serial else "timed frames (lanes overlap)",
                "avg_launch_ms_overlapped": round(avg_ms_overlapped, 4),
                "valu_issue_note": ("a lower bound of the issue-cycle share: packed (v_pk_*) instructions take 4 "
                                    "cycles and transcendentals 8; the packed-FMA calibration kernel "
                                    "(tools/valu_calib.hip, 8 waves/SIMD) fills valu_calibration_packed of its "
                                    "4-cycle issue slots"),
                # rounds 2-6's headline formula (quad-cycles of SQ_ACTIVE_INST_VALU): 2x the issue
                # cycles of unpacked code, so it can exceed 1; kept for comparison with their records
                "valu_busy_quad": _r4(kp.get("valu_busy")),
                "valu_calibration_packed": _r4((pmc or {}).get("calibration", {}).get("valu_busy")) if pmc else None,
                # busy counts issue cycles, not active lanes
                "valu_lane_util": _r4(kp.get("valu_lane_util")),
                "useful_valu_frac": _r4(kp.get("useful_valu_frac")),
                "lane_util_by_kernel": {k: {"valu_issue_frac": _r4(v.get("valu_issue_frac")),
                                            "valu_busy_quad": _r4(v.get("valu_busy")),
                                            "valu_lane_util": _r4(v.get("valu_lane_util")),
                                            "useful_valu_frac": _r4(v.get("useful_valu_frac"))}
                                        for k, v in (pmc or {}).get("kernels", {}).items()
                                        if k in ("k_trace<false>", "k_trace<true>", "k_shade")} or None,
                "hbm": {"achieved": round(hbm_gbs, 1) if hbm_gbs else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(hbm_gbs / HBM_PEAK_GBS, 4) if hbm_gbs else None,
                        "bytes_per_launch": round(traffic) if traffic else None},
                "algorithmic_bytes_per_launch": round(alg) if alg else None,
                # north_star's "fraction of HBM roofline", read directly: the SURVEY 8(d) bytes per
                # launch over the launch time, against HBM and against the L2 (where they are served)
                "algorithmic_gbs": round(alg_gbs, 1) if alg_gbs else None,
                "algorithmic_hbm_frac": round(alg_gbs / HBM_PEAK_GBS, 4) if alg_gbs else None,
                "l2_frac": round(alg_gbs / L2_PEAK_GBS, 4) if alg_gbs else None,
                "l2_peak_gbs": L2_PEAK_GBS,
                "algorithmic_note": "SURVEY 8(d) bytes (ray+hit+N_node*node_bytes+N_tri*48, node_bytes 128 float "
                                    "or 64 quantized); node/triangle reads are "
                                    "L2/MALL hits (counter HBM traffic is 'hbm'), so algorithmic_hbm_frac can exceed "
                                    "1; l2_frac is the same bytes against the L2 peak",
                "pmc_source": pmc_note,
                "visits": per_kind,
                "kernel_ms_per_step": {"trace_closest": acc["msClosest"] / a.steps,
                                       "trace_shadow": acc["msShadow"] / a.steps,
                                       "shade": acc["msShade"] / a.steps,
                                       "note": "HIP-event time per kernel kind, summed per step; the two "
                                               "wavefront lanes' kernels overlap, so these are not additive "
                                               "(their sum exceeds ms_per_step)"}}
        cpu = None
        if not a.no_cpu_baseline:
            cpu = cpu_baseline(ses, a)
        out = {
            "metric": f"Mrays/s (Sponza stand-in {a.size}^2 {a.spp}spp, closest+shadow queries)",
            "value": round(rays / elapsed / 1e6, 2),
            "unit": "Mrays/s",
            "n_gpus": gpus_used,
            "ranks": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (procedural Sponza-class atrium, seed 1234; Sponza.DAE absent)",
            "config": workload_config(a, sinfo, world),
            "samples_per_s": round(samples_total / elapsed, 1),
            "rays_closest": closest, "rays_shadow": shadow,
            "roofline": roof,
            "cpu_baseline": cpu,
            "gather": gather,
            "per_rank": per_rank,
            "launcher": os.environ.get("YRT_BENCH_LAUNCHER", "torch.distributed.run" if world > 1 else "none"),
            "stereo_cubemap": stereo,
        }
        print(json.dumps(out), flush=True)
    ses.close()
    dev.close()
    if world > 1:
        dist.destroy_process_group()
    if stereo and stereo.get("gather_check") not in (None, "bit_exact"):
        sys.exit(f"stereo cubemap gather check failed: {stereo['gather_check']}")


def _r4(x):
    return round(x, 4) if isinstance(x, (int, float)) else None


def rank_times(render_ms, gather_ms, world, red_dev, gather):
    """Per-rank diagnosis of an N-rank step: each rank's wall time until its tiles were
    rendered and its gather time after that (YRTRenderStats msRender / msGather: the gather
    includes waiting for the slowest rank), as max / mean / min over the ranks, so a weak scaling
    curve says whether imbalance or the gather costs it."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([render_ms, gather_ms], dtype=torch.float64, device=red_dev)
    if world > 1:
        allt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        rows = [x.tolist() for x in allt]
    else:
        rows = [t.tolist()]
    r = np.array([x[0] for x in rows])
    g = np.array([x[1] for x in rows])
    return {"render_ms": {"max": round(float(r.max()), 2), "mean": round(float(r.mean()), 2),
                          "min": round(float(r.min()), 2), "imbalance": round(float(r.max() / max(r.mean(), 1e-9)), 4)},
            "gather_ms": {"max": round(float(g.max()), 2), "mean": round(float(g.mean()), 2),
                          "min": round(float(g.min()), 2)},
            "gather_path": gather,
            "note": "per timed step; render = this rank's tiles rendered, gather = after that (waits for peers)"}


def physical_gpus(world, local):
    """Distinct GPUs the ranks run on (host, HIP device): the gloo rehearsal puts several
    ranks on one GPU, the driver's N-GPU runs one rank per GPU."""
    if world == 1:
        return 1
    import socket
    import torch.distributed as dist
    keys = [None] * world
    dist.all_gather_object(keys, (socket.gethostname(), local))
    return len(set(keys))


def setup_gather(dev, rank, world, backend):
    """The frame gather of an N-rank run: the device plugin's own RCCL communicator (rank 0's
    ncclGetUniqueId broadcast over torch.distributed, then yrtSetShardComm): every rtRenderFrame
    ends with each rank's tile slab sent to rank 0 over xGMI (grouped send/recv) — the C++
    product path. If that communicator cannot be formed on every rank (e.g. the gloo rehearsal
    with several ranks on one GPU, which RCCL refuses), the run falls back to one
    torch.distributed reduce of the RGB8 frames (disjoint tiles) and says so."""
    import torch
    import torch.distributed as dist
    dd = "cuda" if backend == "nccl" else "cpu"
    err = "" if backend == "nccl" else f"backend {backend}"
    uid = None
    if not err:
        # every rank first checks that librccl loads (a rank failing inside the collective
        # ncclCommInitRank would hang the others); only rank 0 makes the unique id
        try:
            if rank == 0:
                uid = dev.shard_comm_unique_id()
            elif not dev.rccl_available():
                err = "librccl cannot be loaded"
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            err = str(e)[:200]
    ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=dd)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if ok.item() == 1:
        box = [uid if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        dev.set_shard_comm(rank, world, box[0])
        return "C++ RCCL gather to rank 0 inside rtRenderFrame (yrtSetShardComm)"
    dev.set_tile_shard(rank, world)
    return f"torch.distributed reduce of RGB8 frames (C++ RCCL comm unavailable: {err or 'on another rank'})"


def workload_config(a, sinfo, world):
    """config.workload built from the run's own arguments (C3 only at its BASELINE size)."""
    c3 = a.size == 2048 and a.spp == 64
    name = "C3" if c3 else "C3-reduced"
    return {"workload": f"{name} sponza_standin {a.size}x{a.size} {a.spp}spp depth10 dome(8,8,8) tMaxShadowRay120",
            "width": a.size, "height": a.size, "spp": a.spp, "triangles": sinfo["numTriangles"],
            "bvh_nodes": sinfo["numNodes"], "batch_capacity": a.capacity or "default",
            "parallelism": f"tiles-roundrobin{world}"}


def visit_counts(a, dev, R, cam, S, T, F, sinfo):
    """Untimed capture frame: node/triangle visits per query of the real query streams (a
    strided sample per depth, counted by the oracle's restatement of this traversal) for the
    SURVEY §8(d) algorithmic bytes."""
    import oracle
    dev.set_ray_capture(a.capture)
    dev.rtRenderFrame(R, cam, S, T, F, 0)
    dev.set_ray_capture(0)
    nodes, tris = dev.export_bvh(S)
    qnodes = dev.export_qbvh(S)
    per_kind = {}
    for shadow in (0, 1):
        # the node format the kernel traverses: 64-B quantized nodes (any-hit by default) or the
        # 128-B float ones; the oracle counts visits on the same records
        nb = sinfo["nodeBytesAny" if shadow else "nodeBytesClosest"]
        tot_rays = tot_nodes = tot_tris = 0.0
        for depth in range(64):
            org, dr, total = dev.captured_rays(shadow, depth)
            if len(org):
                nv, tv, _ = oracle.count_visits(nodes, tris, org, dr, any_hit=bool(shadow),
                                                tri_bytes=sinfo["triRecordBytes"],
                                                qnodes=qnodes if nb == 64 else None)
                tot_rays += total
                tot_nodes += nv / len(org) * total
                tot_tris += tv / len(org) * total
        n_node = tot_nodes / max(tot_rays, 1)
        n_tri = tot_tris / max(tot_rays, 1)
        io = 32 + (4 if shadow else 16)
        per_kind["shadow" if shadow else "closest"] = {
            "nodes_per_ray": n_node, "tris_per_ray": n_tri, "node_bytes": nb,
            "bytes_per_ray": io + n_node * nb + n_tri * sinfo["triRecordBytes"]}
    return per_kind


def load_pmc(a, sinfo, world):
    """PMC counters of this same workload (tools/gpu_pmc.sh -> tools/pmc_json.py ->
    profiles/pmc_c3.json). Used only when the recorded config equals this run's; else null."""
    f = ROOT / "profiles" / "pmc_c3.json"
    if not f.exists():
        return None, "no profiles/pmc_c3.json"
    try:
        pmc = json.loads(f.read_text())
    except ValueError:
        return None, "unreadable profiles/pmc_c3.json"
    want = workload_config(a, sinfo, world)
    got = pmc.get("config", {})
    keys = ("width", "height", "spp", "triangles", "bvh_nodes", "batch_capacity")
    if any(got.get(k) != want[k] for k in keys) or world != 1:
        return None, "profiles/pmc_c3.json was collected on another config: " + json.dumps({k: got.get(k) for k in keys})
    return pmc, f"profiles/pmc_c3.json ({pmc.get('source', 'rocprofv3 --pmc')}, same config)"


def cpu_info():
    """nproc, the lscpu model name and the cgroup CPU quota of this host."""
    import subprocess
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        pass
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "model": model,
            "cgroup_cpu_quota": quota}


def stereo_cubemap(a, dev, rank, world, backend, gather, local, gpus_used):
    """BASELINE.json configs[3]: the test_stereo stereo cubemap (12 faces x 1536^2, 256 spp,
    depth 10, test_stereo_view.ecs) as one job per cubemap (yrtRenderFrames): the 110,592
    16x16 tiles of the 12 faces dealt round-robin over the ranks and gathered on
    rank 0 by the device's RCCL send/recv inside the call. Strong scaling: the same cubemap at
    every N; Mrays/s = closest + shadow queries of all ranks / max-over-ranks time.

    Untimed check at N>1: rank 0 renders the same cubemap alone (a second device on its GPU, no
    sharding) and compares it with the gathered one byte for byte (gather_check); that render's
    time is the same-box one-GPU reference of the strong-scaling line."""
    import torch
    import torch.distributed as dist
    import yrt
    args = ["-i", str(ROOT / "scenes" / "test_stereo.xml"), "-c", str(ROOT / "scenes" / "test_stereo_view.ecs"),
            "-size", str(a.stereo_size), str(a.stereo_size), "-spp", str(a.stereo_spp), "-stereo"]
    ses = yrt.Session(args, device=dev)
    info = ses.info()
    W, H = info["width"], info["height"]
    stride = (3 * W + 3) // 4 * 4
    cxx = gather.startswith("C++") or world == 1
    faces_t = None
    if not cxx:
        faces_t = torch.zeros((12, stride * H), dtype=torch.uint8, device="cuda" if backend == "nccl" else "cpu")

    def one_cube():
        if cxx:
            ses.render_cube(read=False)
        else:  # fallback: every rank's faces (zero outside its tiles) summed on rank 0
            for f, img in enumerate(ses.render_cube()):
                faces_t[f].copy_(torch.from_numpy(rgb8_rows(img, stride)))
            dist.reduce(faces_t, dst=0, op=dist.ReduceOp.SUM)
        st = dev.render_stats()
        cube_ms[0] += st["msRender"]
        cube_ms[1] += st["msGather"]
        return st["raysClosest"] + st["raysShadow"]

    cube_ms = [0.0, 0.0]
    one_cube()  # untimed: allocations, sample table
    cube_ms = [0.0, 0.0]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    rays = 0.0
    per = []  # this rank's time per cubemap (the C++ gather ends each one on rank 0)
    t0 = time.perf_counter()
    for _ in range(a.stereo_frames):
        t1 = time.perf_counter()
        rays += one_cube()
        per.append(time.perf_counter() - t1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    red = "cuda" if backend == "nccl" else "cpu"
    tot = torch.tensor([rays], dtype=torch.float64, device=red)
    tm = torch.tensor([dt] + per, dtype=torch.float64, device=red)
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
    dt = tm[0].item()
    per = sorted(tm[1:].tolist())  # per cubemap, max over ranks
    samples = 12.0 * W * H * a.stereo_spp * a.stereo_frames
    c4 = (W, a.stereo_spp) == (1536, 256)
    out = {"metric": f"Mrays/s (test_stereo stereo cubemap 12x{W}^2 {a.stereo_spp}spp, closest+shadow queries)",
           "workload": "C4" if c4 else "C4-reduced",
           "value": round(tot.item() / dt / 1e6, 2), "unit": "Mrays/s", "n_gpus": gpus_used, "ranks": world,
           "scaling": "strong", "ms_per_cubemap": round(dt / a.stereo_frames * 1e3, 1),
           "ms_per_cubemap_median": round(float(np.median(per)) * 1e3, 1),
           "ms_per_cubemap_min": round(per[0] * 1e3, 1),
           "samples_per_s": round(samples / dt, 1), "frames": a.stereo_frames,
           "parallelism": f"cube-tiles-roundrobin{world}", "gather": "C++ RCCL" if cxx else "torch reduce",
           "gather_check": None,
           "per_rank": rank_times(cube_ms[0] / a.stereo_frames, cube_ms[1] / a.stereo_frames, world,
                                  "cuda" if backend == "nccl" else "cpu", gather)}
    if world > 1:
        # the gathered cubemap (rank 0) against a one-GPU render of the same cubemap
        got = None
        if rank == 0:
            got = [rgb8_rows(img, stride) for img in ses._cube_faces()] if cxx else \
                [faces_t[f].cpu().numpy() for f in range(12)]
        check = single_gpu_cube(args, local, stride) if rank == 0 else None
        if rank == 0:
            ref, t_single = check
            bad = sum(int(np.count_nonzero(g != r)) for g, r in zip(got, ref))
            out["gather_check"] = "bit_exact" if bad == 0 else f"{bad} bytes differ"
            out["single_gpu_ms_per_cubemap"] = round(t_single * 1e3, 1)
            out["strong_scaling_efficiency"] = round(t_single / (world * dt / a.stereo_frames), 3)
        dist.barrier()
    ses.close()
    return out


def rgb8_rows(img, stride):
    """An (H, W, 3) RGB8 face as the framebuffer's padded rows (api/framebuffer.h:194-226)."""
    h, w, _ = img.shape
    rows = np.zeros((h, stride), np.uint8)
    rows[:, :3 * w] = img.reshape(h, 3 * w)
    return rows.reshape(-1)


def single_gpu_cube(args, local, stride):
    """Rank 0's reference: the cubemap rendered by an unsharded device on its own GPU (timed,
    after one warm-up render)."""
    import yrt
    d1 = yrt.Device(local)
    s1 = yrt.Session(args, device=d1)
    s1.render_cube(read=False)
    t = time.perf_counter()
    s1.render_cube(read=False)
    dt = time.perf_counter() - t
    ref = [rgb8_rows(img, stride) for img in s1._cube_faces()]
    s1.close()
    d1.close()
    return ref, dt


def cpu_baseline(ses, a):
    """The oracle (CPU restatement of the reference path) on a bounded sample of the same frame
    (same spp/depth/scene/camera): by default the multi-GPU tile split's shard 0 of
    a.cpu_tile_stride (logical tiles t % N == 0, which cover a pseudo-random 1/N of the image's
    16x16 tiles, common/yrt_tile_scatter.h), spread over the whole frame so its rays per sample
    are the frame's; or a centred band of a.cpu_rows rows (--cpu-tile-stride 0). On every logical
    core this process can use (the reference default numThreads=0 -> all cores,
    common/sys/taskscheduler.cpp:105): one worker thread per CPU of the affinity
    mask, capped at the cgroup CPU quota when one is set (the GPU box grants 16 CPUs of a
    256-thread host: 256 threads time-sliced on 16 CPUs measured 40 % slower than 16), over a
    dynamic 16x16 tile queue."""
    import oracle
    blob = ses.export_frame()
    info = cpu_info()
    threads = info["affinity"]
    if info["cgroup_cpu_quota"]:
        threads = max(1, min(threads, int(info["cgroup_cpu_quota"])))
    t = time.perf_counter()
    if a.cpu_tile_stride > 0:
        _, st = oracle.render_shard(blob, a.size, a.size, ses.info()["gamma"], 0, a.cpu_tile_stride, threads=threads)
        what = (f"the 16x16 tiles of shard 0 of {a.cpu_tile_stride} (logical t % {a.cpu_tile_stride} == 0, "
                f"scattered over the image) of the {a.size}^2 frame")
    else:
        y0 = (a.size - a.cpu_rows) // 2
        _, st = oracle.render(blob, a.size, a.size, ses.info()["gamma"], rect=(0, y0, a.size, y0 + a.cpu_rows),
                              threads=threads)
        what = f"rows [{y0},{y0 + a.cpu_rows}) x {a.size} px of the frame"
    dt = time.perf_counter() - t
    rays = st["raysClosest"] + st["raysShadow"]
    # the oracle's sample count is the whole frame's; the sample's own is its pixels x spp
    tx, ty = (a.size + 15) // 16, (a.size + 15) // 16
    if a.cpu_tile_stride > 0:
        from yrt import _native as N
        img = [N.dev.yrtDebugTileScatter(t, tx * ty) for t in range(0, tx * ty, a.cpu_tile_stride)]
        px = sum(min(16, a.size - 16 * (t % tx)) * min(16, a.size - 16 * (t // tx)) for t in img)
    else:
        px = a.cpu_rows * a.size
    samples = float(px) * a.spp
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{what} at {a.spp} spp ({px} px, {samples:.0f} samples, {rays:.0f} rays, "
                      f"{rays / max(samples, 1):.2f} rays per sample, in {dt:.1f} s)",
            "samples_per_s": round(samples / dt, 1), "nproc": info["nproc"], "cpu_model": info["model"],
            "cgroup_cpu_quota": info["cgroup_cpu_quota"], "affinity_cpus": info["affinity"]}

if __name__ == "__main__":
    main()
