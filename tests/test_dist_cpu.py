"""Multi-process plumbing of bench.py on CPU (gloo, world_size 2): each rank
takes its own disjoint set of sequence seeds (weak scaling, no collective on
the data path), the timed region is bracketed by barriers, and rank 0 reports
the MAX time over ranks and the SUM of per-rank work."""
import os
import socket

import pytest
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    w, r, local, dist = bench.dist_setup()
    assert (w, r, local) == (world, rank, rank)
    seeds = bench.sequence_seeds(r, 4)
    bench.barrier(dist)
    t = bench.allreduce_max(dist, float(rank + 1))
    s = bench.allreduce_sum(dist, float(len(seeds)))
    allseeds = [None] * world
    dist.all_gather_object(allseeds, seeds)
    out[rank] = (t, s, allseeds)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_bench_dist_plumbing_gloo(world):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    for rank in range(world):
        t, s, allseeds = out[rank]
        assert t == float(world)           # max over ranks
        assert s == 4.0 * world            # total sequences
        flat = [x for seeds in allseeds for x in seeds]
        assert len(flat) == len(set(flat)) == 4 * world   # disjoint shards
