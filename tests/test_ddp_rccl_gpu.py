"""The data-parallel gradient path on RCCL (torch "nccl") on the GPU, world size 1.

The driver's multi-GPU runs use one rank per GPU over RCCL; a one-GPU box can still run
the same code path with a single rank: bucket hooks firing from inside the HIP backward
(UNet: from the program's block loop; STF: after joining its weight-gradient side
stream), async all-reduces of flat-gradient suffixes on RCCL's stream, finish() before
the optimizer.  With one rank every all-reduce is the identity, so the gradients must
equal, bit for bit, those of the same step without the hook -- any race between the
buckets and the gradient kernels (a bucket reduced before its gradients are final)
shows up as a mismatch.  The N > 1 arithmetic (rank averaging) is covered on CPU by
tests/test_ddp_gloo.py.
"""
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def rccl():
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device(DEV, 0))
    yield
    dist.destroy_process_group()


def _grads_after_steps(make, x, t, use_ddp, steps=2):
    from stfunet import engine
    from stfunet.ddp import GradAllReduce
    from stfunet.optim import AdamW
    torch.manual_seed(0)
    model = make().to(DEV).train()
    opt = AdamW(model.parameters(), lr=1e-3)
    ddp = GradAllReduce(model, bucket_mb=0.25) if use_ddp else None    # small buckets: many per step
    out = []
    for _ in range(steps):
        loss = engine.criterion(model(x), t)
        opt.zero_grad()
        loss.backward()
        n = len(ddp.works) if ddp is not None else 0
        if ddp is not None:
            ddp.finish()
        out.append(([p.grad.detach().clone() for p in model.parameters()], n))
        opt.step()
    torch.cuda.synchronize()
    if ddp is not None:
        model.program.grad_ready_hook = None
    return out


@pytest.mark.parametrize("which", ["unet", "stf"])
def test_rccl_buckets_match_local_step(rccl, which):
    from stfunet import STFLSTMUNet, UNet
    from stfunet.synthetic import dce_batch
    if which == "unet":
        make = lambda: UNet(in_channels=8, num_classes=2, base_c=16)        # noqa: E731
        x, t = dce_batch(4, 8, 128, 128, seed=11, device=DEV)
        x = x.flatten(1, 2)
    else:
        make = lambda: STFLSTMUNet(in_channels=1, num_classes=2, time_steps=4)   # noqa: E731
        x, t = dce_batch(2, 4, 128, 128, seed=12, device=DEV, mask_hw=(64, 64))
    ref = _grads_after_steps(make, x, t, False)
    got = _grads_after_steps(make, x, t, True)
    for (g_ref, _), (g_got, launched) in zip(ref, got):
        assert launched > 1, launched                     # buckets went out while backward ran
        for a, b in zip(g_ref, g_got):
            assert torch.equal(a, b)
