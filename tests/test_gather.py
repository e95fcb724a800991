"""The multi-GPU frame gather's transport (csrc/device/gather.h) and its bounded waits.

After each sharded render the ranks exchange their render status (min of every rank's flag)
and rank r > 0 sends its tile slab to rank 0 (the reference's analogue is
device_network's row bands, devices/device_network/network_device.cpp:255-300). Two transports
implement it: RCCL (one process per GPU, yrtSetShardComm) and an in-process hub
(yrtSetShardHub: several Device objects of one process, which may share one GPU). The hub runs
Device::gather_process's whole bookkeeping — status exchange, per-rank tile counts, pack,
unpack, the failing-rank path — on a one-GPU box, so the GPU tests here compare its gathered
frames with a one-device render bit for bit; RCCL only swaps the transport underneath.

CPU tests drive the hub's two phases on host memory: a peer that never arrives, never sends or
sends the wrong size ends the call within the deadline with an error naming the rank, and the
hub stays aborted afterwards.
"""
import threading
import time

import numpy as np
import pytest

import yrt
from helpers import c4_args


def _threads(fns):
    """Runs fns concurrently; returns their results or exceptions, in order."""
    out = [None] * len(fns)

    def run(i, f):
        try:
            out[i] = f()
        except Exception as e:  # noqa: BLE001 - returned to the test
            out[i] = e

    th = [threading.Thread(target=run, args=(i, f)) for i, f in enumerate(fns)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a hub thread hung past its deadline"
    return out


# ----------------------------------------------------------------------------- host-memory hub (CPU)
def test_hub_status_and_slabs():
    """World 3: the status exchange returns the min flag on every rank, and rank 0 receives
    ranks 1 and 2's slabs in rank order, for several consecutive gathers."""
    hub = yrt.ShardHub(3)
    for g in range(3):
        flags = [1, 1, 1] if g != 1 else [1, 0, 1]
        res = _threads([lambda r=r: hub.status(r, flags[r], 10.0) for r in range(3)])
        assert res == [min(flags)] * 3, res
        if min(flags) == 0:
            continue  # a failed gather moves no slab
        data = {r: bytes([(17 * r + g + i) % 256 for i in range(64)]) for r in (1, 2)}
        res = _threads([lambda: hub.slab(0, recv_bytes_per_rank=64, timeout=10.0),
                        lambda: hub.slab(1, data[1], timeout=10.0),
                        lambda: hub.slab(2, data[2], timeout=10.0)])
        assert res[0].tobytes() == data[1] + data[2]
        assert res[1] is None and res[2] is None
    hub.close()


def test_hub_peer_never_arrives():
    """A rank that never joins the status exchange: the waiting rank fails within the deadline
    with an error naming it, and the hub stays aborted for every later gather."""
    hub = yrt.ShardHub(2)
    t = time.perf_counter()
    with pytest.raises(RuntimeError, match=r"rank\(s\) 1 never arrived"):
        hub.status(0, 1, 0.5)
    dt = time.perf_counter() - t
    assert 0.4 < dt < 5.0, dt
    with pytest.raises(RuntimeError, match="aborted by an earlier gather"):
        hub.status(1, 1, 5.0)
    hub.close()


def test_hub_peer_never_sends():
    """Both ranks pass the status exchange, then rank 1 never sends its slab: rank 0's receive
    fails within the deadline, naming rank 1."""
    hub = yrt.ShardHub(2)
    assert _threads([lambda: hub.status(0, 1, 5.0), lambda: hub.status(1, 1, 5.0)]) == [1, 1]
    t = time.perf_counter()
    with pytest.raises(RuntimeError, match=r"rank\(s\) 1 never sent"):
        hub.slab(0, recv_bytes_per_rank=16, timeout=0.5)
    assert time.perf_counter() - t < 5.0
    hub.close()


def test_hub_root_never_receives():
    """Rank 0 never collects: the sender's wait ends at its deadline instead of holding its slab
    buffer forever."""
    hub = yrt.ShardHub(2)
    assert _threads([lambda: hub.status(0, 1, 5.0), lambda: hub.status(1, 1, 5.0)]) == [1, 1]
    with pytest.raises(RuntimeError, match="not received by rank 0"):
        hub.slab(1, b"x" * 32, timeout=0.5)
    hub.close()


def test_hub_slab_size_mismatch():
    """A slab of the wrong size (a rank with another tile count) fails both sides, never a
    partial copy."""
    hub = yrt.ShardHub(2)
    assert _threads([lambda: hub.status(0, 1, 5.0), lambda: hub.status(1, 1, 5.0)]) == [1, 1]
    res = _threads([lambda: hub.slab(0, recv_bytes_per_rank=64, timeout=5.0),
                    lambda: hub.slab(1, b"y" * 100, timeout=5.0)])
    assert all(isinstance(r, RuntimeError) for r in res), res
    assert "sent 100 bytes, rank 0 expects 64" in str(res[0])
    hub.close()


def test_shard_hub_arming_rules(host_device):
    """yrtSetShardHub: a world-1 hub is a plain single shard; a multi-rank hub needs a GPU
    device; an out-of-range rank is refused; None disarms."""
    h1, h2 = yrt.ShardHub(1), yrt.ShardHub(2)
    host_device.set_shard_hub(h1, 0)
    with pytest.raises(RuntimeError, match="host-only"):
        host_device.set_shard_hub(h2, 1)
    with pytest.raises(RuntimeError, match="invalid rank"):
        host_device.set_shard_hub(h2, 2)
    host_device.set_shard_hub(None, 0)
    with pytest.raises(RuntimeError):
        host_device.set_gather_timeout(0)
    host_device.set_gather_timeout(30)
    h1.close()
    h2.close()


# ----------------------------------------------------------------------------- devices on one GPU
def _ranks(world, fb, timeout=60.0):
    hub = yrt.ShardHub(world)
    devs = [yrt.Device(0) for _ in range(world)]
    sess = []
    for r, d in enumerate(devs):
        d.set_batch_capacity(1 << 20)
        d.set_gather_timeout(timeout)
        d.set_shard_hub(hub, r)
        sess.append(yrt.Session(c4_args(96, 2) + ["-fb", fb], device=d))
    return hub, devs, sess


def _close(hub, devs, sess):
    for s in sess:
        s.close()
    for d in devs:
        d.set_shard_hub(None, 0)
        d.close()
    hub.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,fb", [(2, "RGB8"), (3, "RGB_FLOAT32")])
def test_hub_gather_equals_single(gpu_device, world, fb):
    """`world` devices on this GPU, one thread each, gathered through the hub inside
    rtRenderFrame(s): rank 0's cube (12 faces as one job, tiles dealt over the ranks) and mono
    frame equal one unsharded device's bit for bit, and the render stats name the hub gather."""
    s = yrt.Session(c4_args(96, 2) + ["-fb", fb], device=gpu_device)
    ref_cube, ref_face = s.render_cube(), s.render(5)
    s.close()
    hub, devs, sess = _ranks(world, fb)
    try:
        for _ in range(2):  # consecutive gathers on the same hub
            res = _threads([lambda s=s: s.render_cube() for s in sess])
            assert not any(isinstance(r, Exception) for r in res), res
            for f in range(12):
                assert np.array_equal(res[0][f], ref_cube[f]), f
            assert yrt.GATHER_PATHS[int(devs[0].render_stats()["gather"])] == "hub"
        res = _threads([lambda s=s: s.render(5) for s in sess])
        assert not any(isinstance(r, Exception) for r in res), res
        assert np.array_equal(res[0], ref_face)
    finally:
        _close(hub, devs, sess)


@pytest.mark.gpu
def test_hub_failing_rank_fails_every_rank():
    """A rank whose render throws (uncommitted scene) or whose call fails on its arguments (null
    camera) makes every rank's call fail through the status exchange, without a hang; the next
    frame gathers normally."""
    hub, devs, sess = _ranks(2, "RGB8")
    try:
        i1 = sess[1].info()
        bad_scene = devs[1].rtNewScene()

        def bad_render():
            devs[1].rtRenderFrame(i1["renderer"], sess[1].camera(0), bad_scene, i1["tonemapper"],
                                  i1["framebuffer"], 0)

        def bad_args():
            devs[1].rtRenderFrame(i1["renderer"], None, i1["scene"], i1["tonemapper"], i1["framebuffer"], 0)

        for bad, msg in ((bad_render, "not committed"), (bad_args, "null handle")):
            res = _threads([lambda: sess[0].render(0), bad])
            assert isinstance(res[0], RuntimeError) and "peer rank" in str(res[0]), res
            assert isinstance(res[1], RuntimeError) and msg in str(res[1]), res
        res = _threads([lambda s=s: s.render(0) for s in sess])
        assert not any(isinstance(r, Exception) for r in res), res
    finally:
        _close(hub, devs, sess)


@pytest.mark.gpu
def test_hub_missing_rank_times_out():
    """Rank 1 never renders: rank 0's frame fails at the gather deadline with the phase and the
    missing rank named, and its next frame fails at once (aborted transport) instead of hanging."""
    hub, devs, sess = _ranks(2, "RGB8", timeout=2.0)
    try:
        t = time.perf_counter()
        with pytest.raises(RuntimeError, match=r"status exchange.*rank\(s\) 1 never arrived"):
            sess[0].render(0)
        assert time.perf_counter() - t < 60
        t = time.perf_counter()
        with pytest.raises(RuntimeError, match="aborted"):
            sess[0].render(0)
        assert time.perf_counter() - t < 30
    finally:
        _close(hub, devs, sess)
