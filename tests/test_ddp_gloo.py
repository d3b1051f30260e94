"""Data-parallel gradient all-reduce (stfunet.ddp.GradAllReduce), world_size 2 on
CPU with the gloo backend.

The HIP model cannot run here, so a stand-in "program" with the same
interface (``flat`` = FlatParams, ``grad_ready_hook``) replays a backward that
finishes parameter blocks in reverse flat order, as UNetProgram.backward does.
Checks: every rank ends with the rank-average of the gradients, buckets are
launched while "backward" is still running (more than one bucket), and a second
step reuses the hook state correctly.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Prog:
    def __init__(self, module):
        from stfunet.flat import FlatParams
        self.flat = FlatParams(module)
        self.flat.ensure()
        self.grad_ready_hook = None


class _Model(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.blocks = torch.nn.ModuleList([torch.nn.Linear(64, 64) for _ in range(6)])
        self._program = None

    @property
    def program(self):
        if self._program is None:
            self._program = _Prog(self)
        return self._program


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from stfunet.ddp import GradAllReduce
    torch.manual_seed(0)
    model = _Model()
    ddp = GradAllReduce(model, bucket_mb=0.02)        # ~5k floats -> several buckets
    prog = model.program
    results = []
    for step in range(2):
        prog.flat.fresh_grad()
        g = torch.Generator().manual_seed(100 * step + rank)
        expect = []
        for r in range(world):
            gr = torch.Generator().manual_seed(100 * step + r)
            expect.append(torch.randn(prog.flat.numel, generator=gr))
        mine = torch.randn(prog.flat.numel, generator=g)
        # reverse-order "backward": each block's grads land, then the hook fires
        launched = []
        for blk in reversed(model.blocks):
            first = next(blk.parameters())
            i = prog.flat.index[id(first)]
            lo = prog.flat.offsets[i]
            hi = prog.flat.offsets[i + 2] if i + 2 < len(prog.flat.offsets) else prog.flat.numel
            prog.flat.grad[lo:hi] = mine[lo:hi]
            prog.grad_ready_hook(lo)
            launched.append(len(ddp.works))
        prog.grad_ready_hook(0)
        ddp.finish()
        avg = sum(expect) / world
        ok = torch.allclose(prog.flat.grad, avg, atol=1e-6)
        results.append((ok, max(launched) >= 2))
    q.put((rank, results))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_two_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, results in out:
        for ok, overlapped in results:
            assert ok, f"rank {rank}: gradients are not the rank average"
            assert overlapped, f"rank {rank}: buckets were not launched during backward"
