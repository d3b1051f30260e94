"""A training step replayed as a HIP graph (stfunet.graph.TrainStepGraph) is the same
step: after eager warm-up steps, capture + replay gives bit-identical parameters,
running statistics and loss to running that step eagerly (same kernels, same
buffers' contents; side streams of the STF LSTMs forked and joined inside the capture)."""
import pytest
import torch

from oracle.cases import dce_case
from oracle.init import canonical_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _make(kind, seed):
    from stfunet import STFLSTMUNet, UNet, engine
    from stfunet.optim import AdamW
    if kind == "unet":
        m = UNet(in_channels=8, num_classes=2, base_c=8)
    else:
        m = STFLSTMUNet(time_steps=4)
    m.load_state_dict(canonical_state_dict(m.state_dict(), seed=seed))
    m = m.to(DEV).train()
    opt = AdamW(m.parameters(), lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4, eps=1e-8, capturable=True)
    return m, opt, engine.create_lr_scheduler(opt, 4, 3, warmup=True)


def _batches(kind):
    out = []
    for i in range(3):
        if kind == "unet":
            x5, t = dce_case(40 + i, 2, 8, 64, 64)
            out.append((x5.flatten(1, 2).to(DEV), t.to(DEV)))
        else:
            x5, t = dce_case(40 + i, 2, 4, 64, 64)
            out.append((x5.to(DEV), t[:, ::2, ::2].contiguous().to(DEV)))
    return out


@pytest.mark.parametrize("kind", ["unet", "stf"])
def test_graph_replay_matches_eager(kind):
    from stfunet import engine
    from stfunet.graph import TrainStepGraph
    data = _batches(kind)

    def eager_step(m, opt, sched, x, t):
        loss = engine.criterion(m(x), t)
        opt.zero_grad()
        loss.backward()
        opt.step()
        sched.step()
        return loss

    m1, o1, s1 = _make(kind, 3)
    for x, t in data:
        l1 = eager_step(m1, o1, s1, x, t)
    m2, o2, s2 = _make(kind, 3)
    for x, t in data[:2]:
        eager_step(m2, o2, s2, x, t)
    g = TrainStepGraph(m2, o2, engine.criterion, *data[0]).capture()
    l2 = g.step(*data[2])
    s2.step()
    torch.cuda.synchronize()
    assert torch.equal(l1, l2)
    sd1, sd2 = m1.state_dict(), m2.state_dict()
    for k in sd1:
        assert torch.equal(sd1[k], sd2[k]), k
