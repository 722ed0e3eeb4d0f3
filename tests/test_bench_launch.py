"""bench.py's multi-rank path on the CPU: `bench.py --gpus 2` (no torch.distributed.run
environment) launches the two ranks itself; with the stub workload (CPU oracle, gloo,
codewords keyed by global index exactly like the GPU workloads' Philox streams, offsets
from mc.rank_offset) the summed counters of the two ranks must equal one process over
[0, 2B) -- the sharding contract of SURVEY.md section 8(e)."""
import json
import os
import subprocess
import sys

import pytest

from polarcub_amd import mc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args), capture_output=True, text=True,
                       timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [2])
def test_launcher_counters_equal_single_process(world):
    B = 48
    multi = _bench("--gpus", str(world), "--workload", "stub", "--batch", str(B), "--steps", "2", "--warmup", "1")
    single = _bench("--gpus", "1", "--workload", "stub", "--batch", str(world * B), "--steps", "1", "--warmup", "0")
    assert multi["n_gpus"] == world and single["n_gpus"] == 1
    assert multi["codewords_per_step"] == single["codewords_per_step"] == world * B
    assert multi["frame_errors"] == single["frame_errors"]
    assert multi["bit_errors"] == single["bit_errors"]
    assert multi["frame_errors"] > 0  # the comparison is not vacuous
    assert [p["codewords"] for p in multi["per_rank"]] == [B] * world
    assert multi["value"] > 0 and all(p["value"] > 0 for p in multi["per_rank"])


def test_rank_offsets_tile_the_global_batch():
    B = 1 << 20
    offs = [mc.rank_offset(r, B) for r in range(8)]
    assert offs == [r * B for r in range(8)]
    assert mc.gather_floats([1.0, 2.0]) == [[1.0, 2.0]]
