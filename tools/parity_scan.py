"""Whole-model parity scan: gfx950 path vs the fp32 oracle and vs its bf16-storage
emulation, at several input sizes (the golden fixtures pin the oracle to the reference at
64x64; larger inputs give the BatchNorm groups more samples per statistic).
    python tools/parity_scan.py [--unet] [--fp16]
--fp16: the model runs on the fp16 library and the emulation rounds to fp16; the loss is
scaled by 1024 before the backward (GradScaler-style) and the gradients unscaled."""
import os
import sys
import time
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import numpy as np
import torch
from oracle import loss as o_loss, stf as o_stf, stf_bf16 as o_stf_bf16, unet as o_unet, unet_bf16 as o_unet_bf16
from oracle.cases import dce_case
from oracle.init import canonical_state_dict
from stfunet import STFLSTMUNet, UNet
from stfunet.loss import criterion

torch.set_num_threads(16)
UN = "--unet" in sys.argv
F16 = "--fp16" in sys.argv
SCALE = 1024.0 if F16 else 1.0
import oracle.unet_bf16 as o_q
o_q.STORE = torch.float16 if F16 else torch.bfloat16


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def oracle(fwd, sd, x, t):
    p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    out = fwd(p, x)["out"]
    loss = o_loss.criterion(out, t)
    (loss * SCALE).backward()
    for v in p.values():
        if v.grad is not None:
            v.grad.div_(SCALE)
    return p, out.detach(), loss.item()


sizes = [(4, 64), (4, 128), (4, 256)] if not UN else [(8, 64), (8, 128), (8, 256)]
for T, S in sizes:
    t0 = time.time()
    if UN:
        m = UNet(in_channels=8, num_classes=2, base_c=64)
        x5, t = dce_case(1, 2, 8, S, S)
        x = x5.flatten(1, 2)
        f32 = lambda p, x: o_unet.forward(p, x, training=True)          # noqa: E731
        emu = lambda p, x: o_unet_bf16.forward(p, x, training=True)     # noqa: E731
    else:
        m = STFLSTMUNet(time_steps=T)
        x, t = dce_case(1, 2, T, S, S)
        t = t[:, ::2, ::2].contiguous()
        f32 = lambda p, x: o_stf.forward(p, x, True)                    # noqa: E731
        emu = lambda p, x: o_stf_bf16.forward(p, x, True)               # noqa: E731
    sd = canonical_state_dict(m.state_dict(), seed=0)
    m.load_state_dict(sd)
    m = m.cuda().train()
    m.storage_dtype = torch.float16 if F16 else torch.bfloat16
    out = m(x.cuda())["out"]
    loss = criterion({"out": out}, t.cuda())
    (loss * SCALE).backward()
    for q_ in m.parameters():
        q_.grad.div_(SCALE)
    p32, o32, l32 = oracle(f32, sd, x, t)
    pem, oem, lem = oracle(emu, sd, x, t)
    named = dict(m.named_parameters())
    gh, ge = [], []
    for k, v in p32.items():
        if v.grad is None or v.grad.norm() == 0:
            continue
        gh.append(rel(named[k].grad, v.grad))
        ge.append(rel(pem[k].grad, v.grad))
    print(f"T={T} {S}x{S}: logits hip-f32 {rel(out, o32):.3e}  emu-f32 {rel(oem, o32):.3e}  hip-emu {rel(out, oem):.3e}"
          f" | loss hip {loss.item():.6f} f32 {l32:.6f} emu {lem:.6f}"
          f" | grad rel median hip {np.median(gh):.3e} emu {np.median(ge):.3e}, max hip {max(gh):.3e} emu {max(ge):.3e}"
          f"  ({time.time() - t0:.0f} s)", flush=True)
