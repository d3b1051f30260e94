"""Host-side cost of one training step: CPU enqueue time per step (no sync) vs wall
time per step (synced), bench.py's model/data/optimizer, no kernel timer.
    python tools/host_step.py [--model stf] [--steps 20]"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="unet")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--time-steps", type=int, default=8)
a = ap.parse_args()
from stfunet import engine, STFLSTMUNet, UNet
from stfunet.optim import AdamW
from stfunet.synthetic import dce_batch

dev = torch.device("cuda")
torch.manual_seed(0)
if a.model == "unet":
    model, B, T, half = UNet(in_channels=8, num_classes=2, base_c=64).to(dev), 64, 8, None
else:
    T = a.time_steps
    model, B, half = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=T).to(dev), 16, (128, 128)
model.train()
opt = AdamW(model.parameters(), lr=1e-3)
x, t = dce_batch(B, T, 256, 256, seed=1, device=dev, mask_hw=half)
x = engine.preprocess_input(x, model)


def step():
    loss = engine.criterion(model(x), t)
    opt.zero_grad()
    loss.backward()
    opt.step()


for _ in range(5):
    step()
torch.cuda.synchronize()
cpu = []
t0 = time.perf_counter()
for _ in range(a.steps):
    c0 = time.perf_counter()
    step()
    cpu.append(time.perf_counter() - c0)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / a.steps
cpu.sort()
print(f"{a.model}: wall {wall * 1e3:.2f} ms/step, host enqueue median {cpu[len(cpu) // 2] * 1e3:.2f} ms "
      f"(min {cpu[0] * 1e3:.2f}, max {cpu[-1] * 1e3:.2f})")
