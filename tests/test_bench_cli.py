"""bench.py's launch contract (task: `bench.py --gpus N` measures N GPUs or fails).

CPU: a rank count from a launcher that disagrees with --gpus exits non-zero before any GPU or
torch work. GPU: `bench.py --gpus 2` without a launcher starts its own two ranks
(torch.distributed.run children; gloo rehearsal on the one GPU) and rank 0's line says so."""
import json
import os
import subprocess
import sys

import pytest

from helpers import ROOT


def _bench(args, env_extra, timeout):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "YRT_BENCH_LAUNCHER"):
        env.pop(k, None)
    env.update(env_extra)
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env)


@pytest.mark.parametrize("world,gpus", [("3", "2"), ("1", "2"), ("2", "1")])
def test_world_size_must_match_gpus(world, gpus):
    r = _bench(["--gpus", gpus], {"WORLD_SIZE": world, "RANK": "0", "LOCAL_RANK": "0"}, 60)
    assert r.returncode != 0
    assert f"WORLD_SIZE={world} but --gpus {gpus}" in r.stderr


def test_gpus_must_be_positive():
    r = _bench(["--gpus", "0"], {}, 60)
    assert r.returncode != 0 and "--gpus 0" in r.stderr


@pytest.mark.gpu
def test_gpus_two_without_launcher(tmp_path):
    """The driver's plain `python bench.py --gpus 2` (no torchrun): two ranks render, the
    cubemap gather is bit-exact against rank 0's one-GPU render."""
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--size", "128", "--spp", "4", "--capture", "0",
                "--no-cpu-baseline", "--stereo-size", "64", "--stereo-spp", "2"], {"YRT_DIST_BACKEND": "gloo"}, 240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["ranks"] == 2 and line["launcher"].startswith("bench.py --gpus")
    assert line["stereo_cubemap"]["gather_check"] == "bit_exact"
    # the N > 1 diagnosis: each rank's render and gather time, max / mean / min
    for pr in (line["per_rank"], line["stereo_cubemap"]["per_rank"]):
        r_ms, g_ms = pr["render_ms"], pr["gather_ms"]
        assert 0 < r_ms["min"] <= r_ms["mean"] <= r_ms["max"] and r_ms["imbalance"] >= 1.0
        assert 0 <= g_ms["min"] <= g_ms["mean"] <= g_ms["max"] and pr["gather_path"]
