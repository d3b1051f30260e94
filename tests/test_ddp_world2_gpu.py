"""Data parallelism through the REAL programs at world size 2 on one GPU.

Two spawned ranks share the box's one MI355X and talk over gloo (the driver's 8-GPU
runs use RCCL, one GPU per rank; gloo all-reduces device tensors the same way as far
as stfunet.ddp is concerned: async suffix buckets launched from the HIP backward's
grad_ready_hook, finish() before AdamW).  For UNet and STFLSTMUNet:

* each rank trains on its own batch with GradAllReduce; after backward + finish() its
  flat gradient must equal, bit for bit, (g_0 + g_1) / 2 where g_r is the local
  (no-DDP) gradient of rank r's batch from the same initial weights -- each rank
  recomputes both local gradients itself, the kernels being deterministic;
* buckets went out while the backward ran (more than one per step);
* after AdamW the parameters are identical on both ranks (all-gathered and compared),
  while the BatchNorm running statistics differ (per-rank BN, like torch DDP);
* four DDP steps on native plans (stfunet/plan.py: the second step records, the rest replay
  with the hook running between backward segments) end with exactly the parameters and
  losses of four eager DDP steps (STF_PLAN=0), and the same on both ranks.
"""
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


def _make(which):
    from stfunet import STFLSTMUNet, UNet
    torch.manual_seed(0)
    if which == "unet":
        return UNet(in_channels=8, num_classes=2, base_c=16).cuda().train()
    return STFLSTMUNet(in_channels=1, num_classes=2, time_steps=4).cuda().train()


def _batch(which, seed):
    from stfunet.synthetic import dce_batch
    if which == "unet":
        x, t = dce_batch(2, 8, 128, 128, seed=seed, device="cuda")
        return x.flatten(1, 2), t
    return dce_batch(2, 4, 128, 128, seed=seed, device="cuda", mask_hw=(64, 64))


def _local_grad(which, batch):
    from stfunet import engine
    model = _make(which)
    loss = engine.criterion(model(batch[0]), batch[1])
    loss.backward()
    return model.program.flat.grad.detach().clone()


def _ddp_steps(which, rank, batches, steps, plan_on):
    from stfunet import engine
    from stfunet.ddp import GradAllReduce
    from stfunet.optim import AdamW
    os.environ["STF_PLAN"] = "1" if plan_on else "0"
    try:
        model = _make(which)
        opt = AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
        ddp = GradAllReduce(model, bucket_mb=0.5)
        losses = []
        for i in range(steps):
            x, t = batches[(rank + i) % len(batches)]
            loss = engine.criterion(model(x), t)
            opt.zero_grad()
            loss.backward()
            ddp.finish()
            opt.step()
            losses.append(loss.detach().clone())
        torch.cuda.synchronize()
        model.program.grad_ready_hook = None
        return (torch.stack(losses), model.program.flat.data.detach().clone(),
                model.program.runtime.bwd is not None)
    finally:
        os.environ.pop("STF_PLAN", None)


def _plan_steps(which, rank, world, batches):
    le, pe, _ = _ddp_steps(which, rank, batches, 4, False)
    lp, pp, replayed = _ddp_steps(which, rank, batches, 4, True)
    ps = [torch.empty_like(pp) for _ in range(world)]
    dist.all_gather(ps, pp)
    return dict(plan_replayed=replayed, plan_losses_equal=bool(torch.equal(le, lp)),
                plan_params_equal=bool(torch.equal(pe, pp)),
                plan_params_equal_ranks=all(torch.equal(ps[0], o) for o in ps[1:]))


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from stfunet import engine
    from stfunet.ddp import GradAllReduce
    from stfunet.optim import AdamW
    res = {}
    try:
        for which in ("unet", "stf"):
            batches = [_batch(which, 500 + r) for r in range(world)]
            expect = sum(_local_grad(which, b) for b in batches) / world
            model = _make(which)
            opt = AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
            ddp = GradAllReduce(model, bucket_mb=0.5)
            x, t = batches[rank]
            loss = engine.criterion(model(x), t)
            opt.zero_grad()
            loss.backward()
            launched = len(ddp.works)
            ddp.finish()
            g = model.program.flat.grad.detach().clone()
            opt.step()
            torch.cuda.synchronize()
            p = model.program.flat.data.detach().clone()
            ps = [torch.empty_like(p) for _ in range(world)]
            dist.all_gather(ps, p)
            rm = torch.cat([b.detach().flatten() for n, b in model.named_buffers() if "running_mean" in n])
            rms = [torch.empty_like(rm) for _ in range(world)]
            dist.all_gather(rms, rm)
            model.program.grad_ready_hook = None
            res[which] = dict(grad_equal=bool(torch.equal(g, expect)),
                              grad_maxdiff=float((g - expect).abs().max()),
                              launched=launched,
                              params_equal=all(torch.equal(ps[0], o) for o in ps[1:]),
                              running_stats_differ=not torch.equal(rms[0], rms[1]),
                              loss=float(loss))
            res[which].update(_plan_steps(which, rank, world, batches))
    except Exception as e:  # report, do not hang the peer
        res["error"] = repr(e)
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_world2_real_programs():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in out.items():
        assert "error" not in res, (rank, res)
        for which in ("unet", "stf"):
            r = res[which]
            assert r["grad_equal"], (rank, which, r)
            assert r["launched"] > 1, (rank, which, r)
            assert r["params_equal"], (rank, which, r)
            assert r["running_stats_differ"], (rank, which, r)
            assert r["plan_replayed"] and r["plan_losses_equal"] and r["plan_params_equal"], (rank, which, r)
            assert r["plan_params_equal_ranks"], (rank, which, r)
    assert out[0]["unet"]["loss"] != out[1]["unet"]["loss"]      # the ranks really had different batches
