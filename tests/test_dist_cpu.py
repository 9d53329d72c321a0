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


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus 2` with no launcher env starts 2 ranks itself (gloo
    rendezvous on 127.0.0.1, no GPU call in the parent): world size 2 on every
    rank, disjoint sequence seeds, the total counted over ranks (--dry-run stops
    each rank before it touches a GPU)."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    out = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--seq", "3", "--dry-run"],
                         env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 and d["total_sequences"] == 6 for d in lines)
    seeds = [s for d in lines for s in d["seeds"]]
    assert len(seeds) == len(set(seeds)) == 6


def test_bench_gpus_flag_must_match_launcher():
    """Under a launcher, --gpus N must equal the world size it started."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--dry-run"], env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode != 0 and "--gpus 2" in out.stderr


def _plan_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import svo_amd as S
    w, r, local, dist = bench.dist_setup()
    mine = S.host_cpu_plan(local, w)                   # no GPU: split the node by rank
    numa = S.host_cpu_plan(local, w, [0] * w)          # both GPUs on NUMA node 0
    allp = [None] * world
    dist.all_gather_object(allp, (mine, numa))
    out[rank] = allp
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_host_cpu_plan_disjoint_per_rank_gloo(world):
    """Each rank's RANSAC pool gets its own cores (svo_host_cpu_plan): with one
    process per GPU on a node the ranks' sets are disjoint, non-empty, inside
    the allowed CPUs, and NUMA-node-local when the GPUs' node is given."""
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < world:
        pytest.skip("fewer CPUs than ranks")
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_plan_worker, args=(world, port, out), nprocs=world, join=True)
    plans = out[0]
    for k in range(2):
        sets = [set(p[k]) for p in plans]
        assert all(sets) and all(s <= set(allowed) for s in sets)
        assert not set.intersection(*sets)
    assert set().union(*(set(p[0]) for p in plans)) == set(allowed)   # the whole node is used
