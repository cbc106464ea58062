"""World-size-2 gloo test of the multi-GPU sharding protocol (CPU only): the
global first hit equals the single-process sweep's, and the shards partition
the index space."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from mythril_amd.distributed import chunk_start, sharded_first_hit


def _pred(i: int) -> bool:
    # deterministic sparse "satisfying" set
    return (i * 2654435761) % 1000003 < 3


def _search(start: int, count: int):
    for i in range(start, start + count):
        if _pred(i):
            return i
    return None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, chunk, out):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hit, epochs = sharded_first_hit(_search, rank, world, chunk, max_epochs=1000)
    out[rank] = (hit, epochs)
    dist.destroy_process_group()


def test_chunks_partition_index_space():
    world, chunk = 4, 8
    seen = set()
    for e in range(3):
        for r in range(world):
            s = chunk_start(e, r, world, chunk)
            seen.update(range(s, s + chunk))
    assert seen == set(range(3 * world * chunk))


@pytest.mark.parametrize("world", [2])
def test_sharded_first_hit_matches_single_process(world):
    chunk = 512
    single = _search(0, 1 << 22)
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_worker, args=(world, port, chunk, out), nprocs=world, join=True)
    hits = {out[r][0] for r in range(world)}
    assert hits == {single}
