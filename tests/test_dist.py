"""The multi-rank path of bench.py / polarcub_amd.mc on CPU: world_size 2 over gloo.
Rank r's counters are summed and the elapsed time maxed by the same reduce_counters
call bench.py makes over RCCL; shard ranges tile the global batch."""
import os
import socket

import pytest
import torch.multiprocessing as tmp

from polarcub_amd import mc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, r, lr = mc.dist_env()
    lo, hi = mc.shard_range(1000, r, w)
    counters, el = mc.reduce_counters([hi - lo, 3 + r, 10 * (r + 1), 0], 1.5 + r)
    q.put((r, counters, el, (lo, hi), mc.shard_seed(7, r)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_reduce_counters_gloo(world):
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    for r, counters, el, rng, seed in res:
        assert counters == [1000, sum(3 + k for k in range(world)), sum(10 * (k + 1) for k in range(world)), 0]
        assert el == 1.5 + (world - 1)
    ranges = [x[3] for x in res]
    assert ranges[0][0] == 0 and ranges[-1][1] == 1000
    assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
    assert len({x[4] for x in res}) == world


def test_single_process_is_identity():
    counters, el = mc.reduce_counters([5, 1, 2, 0], 0.25)
    assert counters == [5, 1, 2, 0] and el == 0.25
