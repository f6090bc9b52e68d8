"""Data-parallel plumbing on CPU with the gloo backend, world_size 2: the flat-gradient bucketed
all-reduce averages exactly, and rank shards of the synthetic stream are disjoint."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "eeg-multimodal_amd"), str(root)]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eegfusion.trainer import GradReducer
    from data import WindowDataset
    g = torch.arange(1000, dtype=torch.float32) * (rank + 1)
    GradReducer(bucket_elems=128)(g)                         # 8 buckets
    ds = WindowDataset(12, shard=rank, num_shards=world)
    q.put((rank, g.tolist(), ds.idx))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_reducer_and_sharding_gloo():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (g, idx)) for r, g, idx in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = (torch.arange(1000, dtype=torch.float32) * 1.5).tolist()
    assert res[0][0] == expect and res[1][0] == expect
    assert set(res[0][1]).isdisjoint(res[1][1]) and len(res[0][1]) + len(res[1][1]) == 12
