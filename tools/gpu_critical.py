"""GPU-side time of one eager training step with the host out of the way: a spin kernel
(torch.cuda._sleep) holds the main stream while the host enqueues the whole step, so the
GPU then runs the step back to back with the streams and events of the eager program.
Event e0 after the spin, e1 after the optimizer: e0 -> e1 = the step's GPU critical path.
    python tools/gpu_critical.py [--model stf|unet] [--steps 5] [--spin-ms 40]"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="stf")
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--spin-ms", type=float, default=40.0)
ap.add_argument("--time-steps", type=int, default=8)
a = ap.parse_args()
from stfunet import engine, STFLSTMUNet, UNet
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
    return loss


for _ in range(4):
    step()
torch.cuda.synchronize()
# calibrate the spin: cycles per ms
c0 = time.perf_counter()
torch.cuda._sleep(10_000_000)
torch.cuda.synchronize()
cyc_per_ms = 10_000_000 / ((time.perf_counter() - c0) * 1e3)
gpu, host, wall = [], [], []
for _ in range(a.steps):
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    torch.cuda._sleep(int(a.spin_ms * cyc_per_ms))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    h0 = time.perf_counter()
    step()
    h1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    gpu.append(e0.elapsed_time(e1))
    host.append((h1 - h0) * 1e3)
    wall.append((time.perf_counter() - w0) * 1e3)
gpu.sort()
host.sort()
print(f"{a.model}: GPU critical path {gpu[len(gpu) // 2]:.3f} ms/step (min {gpu[0]:.3f}); host enqueue "
      f"{host[len(host) // 2]:.3f} ms (must stay under the {a.spin_ms:.0f} ms spin: "
      f"{'ok' if host[-1] < a.spin_ms else 'SPIN TOO SHORT'})")
