"""Multi-GPU sharding of slice pairs, exercised on CPU with gloo."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from optflow_amd import stack


def test_stack_pairs_counts():
    # C3 255 pairs; C4 4095; C5 strides 1/4/16 -> 4095 + 4092 + 4080
    assert len(stack.stack_pairs(256)) == 255
    assert len(stack.stack_pairs(4096)) == 4095
    assert len(stack.stack_pairs(4096, (1, 4, 16))) == 4095 + 4092 + 4080
    assert stack.stack_pairs(5, (2,)) == [(0, 2), (1, 3), (2, 4)]


@pytest.mark.parametrize("n,world,chunk", [(255, 2, 16), (4095, 8, 16), (7, 3, 2), (0, 2, 4)])
def test_shard_is_a_partition(n, world, chunk):
    got = [stack.shard(n, r, world, chunk) for r in range(world)]
    flat = sorted(i for g in got for i in g)
    assert flat == list(range(n))
    # contiguous chunks => adjacent pairs mostly reuse a resident slice
    pairs = stack.stack_pairs(n + 1)
    for g in got:
        if g:
            assert stack.uploads_needed(pairs, g) <= 2 * ((len(g) + chunk - 1) // chunk) + len(g)


def test_contiguous_chunks_reuse_slices():
    pairs = stack.stack_pairs(257)
    order = stack.shard(len(pairs), 0, 1, 16)
    assert stack.uploads_needed(pairs, order) == len(pairs) + 1   # one new slice per pair


def _worker(rank, world, port, n, chunk, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = stack.shard(n, rank, world, chunk)
    # the only cross-rank traffic: counters (pairs, iterations) and the barrier
    cnt = torch.tensor([len(mine), sum(mine)], dtype=torch.int64)
    dist.all_reduce(cnt)
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    dist.barrier()
    if rank == 0:
        q.put((cnt.tolist(), sorted(i for g in gathered for i in g)))
    dist.destroy_process_group()


def test_gloo_two_ranks_cover_every_pair_once():
    n, world, chunk = 255, 2, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    cnt, union = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert cnt == [n, n * (n - 1) // 2]
    assert union == list(range(n))


def _queue_worker(rank, world, port, n, q):
    import threading
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    store = dist.distributed_c10d._get_default_store()
    if rank == 0:
        store.set("stack_q", "0")
    dist.barrier()
    wq = stack.WorkQueue(n, store)
    got = [[] for _ in range(2)]

    def pull(j):
        while (i := wq.pop()) is not None:
            got[j].append(i)

    ts = [threading.Thread(target=pull, args=(j,)) for j in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    gathered = [None] * world
    dist.all_gather_object(gathered, got[0] + got[1])
    if rank == 0:
        q.put(gathered)
    dist.destroy_process_group()


def test_work_queue_two_ranks_two_threads_each_item_once():
    """bench.py --workload stack: chunks pulled from one atomic counter on the
    distributed store by every thread of every rank -- each handed out exactly once."""
    n, world = 97, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_queue_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    allitems = sorted(i for g in gathered for i in g)
    assert allitems == list(range(n))


def test_work_queue_local_counter():
    wq = stack.WorkQueue(5)
    assert [wq.pop() for _ in range(7)] == [0, 1, 2, 3, 4, None, None]
