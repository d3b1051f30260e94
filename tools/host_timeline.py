"""Host vs GPU timeline of one synced training step (the bench loop: forward, criterion,
zero_grad, backward, optimizer step, loss.item()): at each phase boundary the host time since
the step start and the GPU time (an event on the current stream) since the same point.  Where
GPU time ~= host time the GPU was waiting for the host to enqueue; where GPU >> host the host
is ahead.  Also the main-stream idle inferred per phase.
    python tools/host_timeline.py [--model stf|unet] [--config 3|4] [--steps 8]"""
import argparse
import os
import sys
import time
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="stf")
ap.add_argument("--time-steps", type=int, default=8)
ap.add_argument("--steps", type=int, default=8)
a = ap.parse_args()
from stfunet import STFLSTMUNet, UNet, engine
from stfunet.optim import AdamW
from stfunet.synthetic import dce_batch

dev = torch.device("cuda")
torch.manual_seed(0)
if a.model == "unet":
    model, B, half = UNet(in_channels=8, num_classes=2, base_c=64).to(dev), 64, None
else:
    model, B, half = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=a.time_steps).to(dev), 16, (128, 128)
model.train()
opt = AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
x, t = dce_batch(B, a.time_steps, 256, 256, seed=1, device=dev, mask_hw=half)
x = engine.preprocess_input(x, model)
names = ["forward", "criterion", "zero_grad", "backward", "opt.step", "item"]


def step(rec):
    ev, ht = [], []

    def mark():
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.append(e)
        ht.append(time.perf_counter())
    mark()
    out = model(x)
    mark()
    loss = engine.criterion(out, t)
    mark()
    opt.zero_grad()
    mark()
    loss.backward()
    mark()
    opt.step()
    mark()
    v = loss.item()
    mark()
    torch.cuda.synchronize()
    if rec is not None:
        rec.append(([(ht[i] - ht[0]) * 1e3 for i in range(len(ht))],
                    [ev[0].elapsed_time(ev[i]) for i in range(len(ev))]))
    return v


for _ in range(5):
    step(None)
rec = []
for _ in range(a.steps):
    step(rec)
rec.sort(key=lambda r: r[1][-1])
h, g = rec[len(rec) // 2]
print(f"{a.model}: median step host {h[-1]:.3f} ms, GPU {g[-1]:.3f} ms (event to event)")
for i, n in enumerate(names):
    print(f"  after {n:10s} host {h[i + 1]:8.3f} ms   GPU {g[i + 1]:8.3f} ms   host phase {h[i + 1] - h[i]:7.3f} ms")
