"""Where the host enqueue time of one eager training step goes (the GPU held by a spin
kernel so launches never wait for a full queue): baseline, Python GC off, the share inside
the C-ABI calls (ctypes + HIP launch), and the share of the operand checks.
    python tools/host_breakdown.py [--model stf|unet] [--steps 9]"""
import argparse
import gc
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
# STF_PKG_ROOT: import the package from another tree (same-box A/B of host-side changes)
sys.path[:0] = [os.path.dirname(HERE), os.environ.get("STF_PKG_ROOT", os.path.join(os.path.dirname(HERE), "stf-unet_amd"))]
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="stf")
ap.add_argument("--steps", type=int, default=9)
ap.add_argument("--time-steps", type=int, default=8)
a = ap.parse_args()
from stfunet import _lib, engine, nhwc, STFLSTMUNet, UNet
from stfunet.optim import AdamW
from stfunet.synthetic import dce_batch

dev = torch.device("cuda")
torch.manual_seed(0)
if a.model == "unet":
    model, B, half = UNet(in_channels=8, num_classes=2, base_c=64).to(dev), 64, None
else:
    model, B, half = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=a.time_steps).to(dev), 16, (128, 128)
model.train()
opt = AdamW(model.parameters(), lr=1e-3)
x, t = dce_batch(B, a.time_steps, 256, 256, seed=1, device=dev, mask_hw=half)
x = engine.preprocess_input(x, model)


def step():
    loss = engine.criterion(model(x), t)
    opt.zero_grad()
    loss.backward()
    opt.step()


for _ in range(4):
    step()
torch.cuda.synchronize()
c0 = time.perf_counter()
torch.cuda._sleep(10_000_000)
torch.cuda.synchronize()
cyc_per_ms = 10_000_000 / ((time.perf_counter() - c0) * 1e3)


def held(n=a.steps):
    """median host enqueue (ms) of one step while a 60 ms spin holds the GPU"""
    out = []
    for _ in range(n):
        torch.cuda.synchronize()
        torch.cuda._sleep(int(60 * cyc_per_ms))
        h0 = time.perf_counter()
        step()
        out.append((time.perf_counter() - h0) * 1e3)
    torch.cuda.synchronize()
    out.sort()
    return out[len(out) // 2], out[0]


base = held()
gc.disable()
nogc = held()
gc.enable()
acc = [0.0, 0]
orig_call = _lib.call


def timed_call(name, *args):
    c = time.perf_counter()
    orig_call(name, *args)
    acc[0] += time.perf_counter() - c
    acc[1] += 1


_lib.call = timed_call
for mod in (nhwc,):
    mod.call = timed_call
import stfunet.stf_lstm_unet as _s, stfunet.unet as _u, stfunet.loss as _l, stfunet.optim as _o
for mod in (_s, _u, _l, _o):
    if hasattr(mod, "call"):
        mod.call = timed_call
acc[:] = [0.0, 0]
wrapped = held()
n_steps = a.steps
calls_ms = acc[0] * 1e3 / n_steps
ncalls = acc[1] / n_steps
_lib.call = orig_call
for mod in (nhwc, _s, _u, _l, _o):
    if hasattr(mod, "call"):
        mod.call = orig_call
orig_check = nhwc.Feat.check
nhwc.Feat.check = lambda self: None
nocheck = held()
nhwc.Feat.check = orig_check
print(f"{a.model}: host enqueue median {base[0]:.2f} ms (min {base[1]:.2f}); GC off {nogc[0]:.2f} (min {nogc[1]:.2f}); "
      f"C-ABI calls {calls_ms:.2f} ms over {ncalls:.0f} calls/step (wrapped step {wrapped[0]:.2f}); "
      f"without Feat.check {nocheck[0]:.2f}")
