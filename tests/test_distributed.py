"""Multi-rank path of bench.py on CPU (gloo, world_size 2 and 3).

Stripes are independent, so ranks shard them round-robin with no data-path
collective; the only cross-rank operations are the timing
barrier and the max-reduce of elapsed time.  Each rank here codes its own
stripes with the CPU oracle (test infrastructure: no GPU in this container)
and the union is checked against a single-process run: every stripe coded
exactly once, identical bytes.  The same ranks coding with the product
library on a GPU, and bench.py --gpus 2 itself, are in
tests/test_multirank_gpu.py (-m gpu).
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    import torch.distributed as dist
    from ecdata import fnv1a64, shard_seed, splitmix_bytes
    from oracle.oracle import Restatement, alloc_shards

    r, local, w = bench.dist_setup()
    assert (r, w) == (rank, world)
    o = Restatement()
    k, m, size = 6, 3, 1000
    M = o.vandermonde_coding_matrix(k, m)
    mine = {}
    for s in bench.stripes_for_rank(total, rank, world):
        data = alloc_shards(k, size)
        for j in range(k):
            data[j][:size] = splitmix_bytes(size, shard_seed(2, s, j))
        coding = alloc_shards(m, size)
        o.matrix_encode(k, m, M, data, coding, size)
        mine[s] = [fnv1a64(c[:size]) for c in coding]
    bench.barrier(world)
    t = bench.max_over_ranks(float(rank + 1), world)
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    dist.destroy_process_group()
    q.put((rank, t, gathered))


@pytest.mark.parametrize("world", [2, 3])
def test_round_robin_sharding_and_max_reduce(world):
    total = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, gathered in results:
        assert t == float(world)  # max over ranks of (rank + 1)
        merged = {}
        for part in gathered:
            assert not (set(part) & set(merged)), "a stripe was coded twice"
            merged.update(part)
        assert sorted(merged) == list(range(total))
    # single-process reference for the same stripes
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from ecdata import fnv1a64, shard_seed, splitmix_bytes
    from oracle.oracle import Restatement, alloc_shards
    o = Restatement()
    k, m, size = 6, 3, 1000
    M = o.vandermonde_coding_matrix(k, m)
    for s in range(total):
        data = alloc_shards(k, size)
        for j in range(k):
            data[j][:size] = splitmix_bytes(size, shard_seed(2, s, j))
        coding = alloc_shards(m, size)
        o.matrix_encode(k, m, M, data, coding, size)
        assert merged[s] == [fnv1a64(c[:size]) for c in coding]
