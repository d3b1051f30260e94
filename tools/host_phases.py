"""Host time of one synced training step (bench.py's loop: the host reads the loss after every
step, as train_one_epoch does), by phase -- what the GPU waits for between the loss read that ends
step k and the first launch of step k+1 (the input copy of the forward plan replay).
    python tools/host_phases.py [--model unet|stf] [--steps 20]"""
import argparse
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="unet")
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
from stfunet import engine, plan, STFLSTMUNet, UNet
from stfunet.optim import AdamW
from stfunet.synthetic import dce_batch

dev = torch.device("cuda")
torch.manual_seed(0)
if a.model == "unet":
    model, B, T, half = UNet(in_channels=8, num_classes=2, base_c=64).to(dev), 64, 8, None
else:
    model, B, T, half = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=8).to(dev), 16, 8, (128, 128)
opt = AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
sched = engine.create_lr_scheduler(opt, 100, 10, warmup=True)
x, t = dce_batch(B, T, 256, 256, seed=1, device=dev, mask_hw=half)
x = engine.preprocess_input(x, model)

marks = {}
rt = model.program.runtime
orig_fwd, orig_bwd = rt.forward, rt.backward


def fwd(*args, **kw):
    marks["fwd_in"] = time.perf_counter()
    r = orig_fwd(*args, **kw)
    marks["fwd_out"] = time.perf_counter()
    return r


def bwd(*args, **kw):
    marks["bwd_in"] = time.perf_counter()
    r = orig_bwd(*args, **kw)
    marks["bwd_out"] = time.perf_counter()
    return r


rt.forward, rt.backward = fwd, bwd
rows = []
for i in range(a.steps + 6):
    m = {"start": time.perf_counter()}
    out = model(x)
    m["model"] = time.perf_counter()
    loss = engine.criterion(out, t)
    m["criterion"] = time.perf_counter()
    opt.zero_grad()
    m["zero_grad"] = time.perf_counter()
    loss.backward()
    m["backward"] = time.perf_counter()
    opt.step()
    m["opt"] = time.perf_counter()
    sched.step()
    m["sched"] = time.perf_counter()
    loss.item()
    m["item"] = time.perf_counter()
    m.update(marks)
    if i >= 6:
        rows.append(m)
order = ["start", "fwd_in", "fwd_out", "model", "criterion", "zero_grad", "bwd_in", "bwd_out", "backward", "opt",
         "sched", "item"]
print(f"{a.model}: plans {'on' if plan.enabled() else 'off'}, {len(rows)} synced steps, median host time per phase:")
for p, q in zip(order, order[1:]):
    d = statistics.median((r[q] - r[p]) * 1e6 for r in rows)
    print(f"  {p:>9s} -> {q:<9s} {d:9.1f} us")
gap = statistics.median((r["fwd_in"] - r["start"]) * 1e6 for r in rows)
print(f"  host time from the loss read to the forward plan replay: {gap:.1f} us (+ the replay's input copy)")
