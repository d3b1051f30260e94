"""Digest of one UNet and one STF training step (logits, loss, flat gradient, BN running stats)
on fixed seeded inputs, for checking that two builds of the library (STF_LIB=...) compute the
same bits.  Usage: python tools/lib_digest.py  -> one line per model: sha256 prefixes."""
import hashlib
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from oracle.init import canonical_state_dict
from stfunet import STFLSTMUNet, UNet
from stfunet.loss import criterion
from stfunet.synthetic import dce_batch


def h(t):
    return hashlib.sha256(t.detach().float().cpu().contiguous().numpy().tobytes()).hexdigest()[:16]


def run(name, m, x, t):
    m.load_state_dict(canonical_state_dict(m.state_dict(), seed=0))
    m = m.cuda().train()
    for _ in range(3):                          # eager, recorded and replayed steps
        for p in m.parameters():
            p.grad = None
        out = m(x)["out"]
        loss = criterion({"out": out}, t)
        loss.backward()
    torch.cuda.synchronize()
    g = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    rs = torch.cat([b.reshape(-1).float() for n, b in m.named_buffers() if "running" in n])
    print(f"{name}: logits {h(out)} loss {loss.item():.9g} grads {h(g)} running {h(rs)}", flush=True)


x, t = dce_batch(8, 8, 128, 128, seed=3, device="cuda")
run("unet", UNet(in_channels=8, num_classes=2, base_c=64), x.flatten(1, 2), t)
x, t = dce_batch(2, 4, 128, 128, seed=4, device="cuda")
run("stf", STFLSTMUNet(time_steps=4), x, t[:, ::2, ::2].contiguous())
