"""Two ranks on one GPU (gloo over device tensors; RCCL needs one GPU per rank): a real PriGumbel
step with the overlapped GradReducer leaves every rank with the exact average of the ranks' local
gradients over the whole model range — the hooks fired inside the HIP backward cover every used
parameter, in the same order on both ranks, and no range is reduced twice."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


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
    try:
        from eegfusion.modules import PriGumbelModel
        from eegfusion.trainer import GradReducer, PriGumbelTrainer
        torch.cuda.set_device(0)

        def step(reducer):
            torch.manual_seed(3)
            m = PriGumbelModel(1.0, contract="W", dropout=0.0).cuda()
            # lr 0: pass 1's DP step must not differ between the local and the reduced run (the
            # averaged DP gradient would move DP differently and change pass 2's gradients)
            tr = PriGumbelTrainer(m.engine, lr=0.0, reducer=reducer, consume_grads=False)
            g = torch.Generator(device="cuda").manual_seed(100 + rank)       # rank-specific shard
            eeg = torch.randn(2, 64, 256, generator=g, device="cuda")
            act = torch.randn(2, 32, generator=g, device="cuda") * 0.5
            labels = torch.tensor([rank, 1 - rank], device="cuda")
            tr.step({"eeg": eeg, "act": act}, labels)
            torch.cuda.synchronize()
            lo, hi = m.arena.model_range
            return m.arena.grad[lo:hi].clone(), reducer

        local, _ = step(GradReducer())                       # world 1: rank-local gradients
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        reduced, red = step(GradReducer(bucket_elems=8 << 20))
        dist.all_reduce(local)                               # reference: one synchronous reduce
        local.mul_(1.0 / world)
        err = float((reduced - local).abs().max())
        q.put((rank, err, float(local.abs().max()), len(red.log), red.log[:3]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e), 0.0, 0, []))


def test_overlapped_reducer_two_ranks_one_gpu():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=100) for _ in range(world))}
    for p in procs:
        p.join(timeout=30)
    for r in range(world):
        err, scale, n, head = res[r]
        assert not isinstance(err, str), err
        assert scale > 0 and err <= 1e-6 * scale, (r, err, scale)
        assert n == res[0][2] and head == res[0][3]
