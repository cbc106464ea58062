"""World-size-2 gloo test of the multi-GPU sharding protocol (CPU only): the
global first hit equals the single-process sweep's, and the shards partition
the index space.  The engine-level case runs each rank's chunk through the C port's search
(``oracle/bveval.c``: the same GEN3 candidates and verdicts the GPU kernels compute) over real
workload queries with a ~2^-12 needle, so the protocol is exercised on the product's
candidate stream, not on a toy predicate."""
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


def _engine_query(workload: str):
    import bench
    from mythril_amd import search, workloads

    roots = bench.hard_query(workloads.WORKLOADS[workload](), 12)
    P, blob = search.prepare(roots)
    return P.to_bytes(), blob


def _engine_worker(rank, world, port, chunk, workload, out):
    import torch.distributed as dist

    from oracle import cport

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pb, blob = _engine_query(workload)
    hit, epochs = sharded_first_hit(lambda s, n: cport.search(pb, blob, SEED, s, n, threads=2)[0], rank, world, chunk,
                                    max_epochs=4096)
    out[rank] = (hit, epochs)
    dist.destroy_process_group()


SEED = 0x6D797468


@pytest.mark.parametrize("workload", ["token_transfer_underflow", "walletlibrary_kill"])
def test_sharded_engine_search_matches_one_process(workload):
    """gloo world size 2: each rank sweeps its chunks with the C port's search of the workload's
    hard query, one all_reduce(MIN) per epoch; both ranks agree on the global first hit, which is
    the first hit of one process sweeping [0, N) in order, and it is not in rank 0's first chunk."""
    from oracle import cport

    world, chunk = 2, 1024
    pb, blob = _engine_query(workload)
    single, _, _ = cport.search(pb, blob, SEED, 0, 1 << 20, threads=4)
    assert single is not None and single >= chunk, single
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_engine_worker, args=(world, _free_port(), chunk, workload, out), nprocs=world, join=True)
    assert {out[r][0] for r in range(world)} == {single}
    # every rank ran the same number of epochs: the epoch of the chunk that holds the hit
    assert {out[r][1] for r in range(world)} == {single // (world * chunk) + 1}


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
