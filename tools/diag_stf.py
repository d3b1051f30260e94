"""Diagnostic: STFLSTMUNet (gfx950) vs the fp32 oracle -- logits, loss, per-param grad error."""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import numpy as np
import torch
from oracle import loss as o_loss, stf as o_stf
from oracle.init import canonical_state_dict
from stfunet import STFLSTMUNet
from stfunet.loss import criterion

torch.set_num_threads(16)
for pk in (False, True):
    g = np.load(os.path.join(os.path.dirname(HERE), "tests/golden", "stf_pk_t4.npz" if pk else "stf_t4.npz"))
    m = STFLSTMUNet(use_pk_maps=pk, time_steps=4)
    sd = canonical_state_dict(m.state_dict(), seed=0)
    m.load_state_dict(sd)
    m = m.cuda().train()
    x, t = torch.from_numpy(g["x"]), torch.from_numpy(g["target"])
    out = m(x.cuda())["out"]
    loss = criterion({"out": out}, t.cuda())
    loss.backward()
    p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    ref = o_stf.forward(p, x, True, use_pk_maps=pk)["out"]
    lref = o_loss.criterion(ref, t)
    lref.backward()
    print(f"pk={pk} loss {loss.item():.6f} oracle {lref.item():.6f} golden {float(g['loss']):.6f} "
          f"logits rel {((out.detach().cpu()-ref.detach()).norm()/ref.norm()).item():.3e}")
    named = dict(m.named_parameters())
    msd = m.state_dict()
    worst = []
    for k, v in p.items():
        if "running" in k:
            r = ((msd[k].cpu() - v.detach()).norm() / v.detach().norm().clamp_min(1e-12)).item()
            if r > 1e-2:
                print("   running", k, r)
            continue
        if v.grad is None:
            continue
        gg = named[k].grad.cpu()
        r = ((gg - v.grad).norm() / v.grad.norm().clamp_min(1e-20)).item()
        worst.append((r, k))
    worst.sort(reverse=True)
    for r, k in worst[:25]:
        print(f"   {k:45s} rel {r:.3e}")
    print("   median rel", np.median([r for r, _ in worst]))
    nbt = [int(v) for k, v in msd.items() if k.endswith("num_batches_tracked")]
    print("   num_batches_tracked set:", sorted(set(nbt)))
