"""Diagnostic: per-parameter relative gradient error of stfunet.UNet vs the fp32 oracle."""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from oracle import loss as o_loss, unet as o_unet
from oracle.cases import dce_case
from oracle.init import canonical_state_dict
from stfunet.unet import UNet
from stfunet.loss import criterion


def run(base_c, size):
    m = UNet(8, 2, base_c)
    sd = canonical_state_dict(m.state_dict(), seed=0)
    m.load_state_dict(sd)
    m = m.cuda().train()
    x5, t = dce_case(1, 2, 8, size, size)
    x = x5.flatten(1, 2)
    p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    out_ref = o_unet.forward(p, x, True)["out"]
    lref = o_loss.criterion(out_ref, t)
    lref.backward()
    out = m(x.cuda())["out"]
    loss = criterion({"out": out}, t.cuda())
    loss.backward()
    print(f"base_c={base_c} size={size} loss {loss.item():.6f} ref {lref.item():.6f} "
          f"logits rel {((out.detach().cpu()-out_ref.detach()).norm()/out_ref.norm()).item():.4e}")
    named = dict(m.named_parameters())
    for k, v in reversed(list(p.items())):
        if v.grad is None or k.endswith(("0.bias", "3.bias")) and not k.startswith(("up", "out")):
            continue
        g = named[k].grad.cpu()
        r = ((g - v.grad).norm() / v.grad.norm()).item()
        print(f"  {k:28s} rel {r:.4e}")


for bc, sz in ((8, 64), (32, 64), (64, 128)):
    run(bc, sz)
