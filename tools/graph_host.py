"""Host cost of a HIP-graph replay of the STF step: the time the replay() call itself takes on
the host (no sync) vs the synced wall time per replay.
    python tools/graph_host.py [--steps 20]"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
from stfunet import engine, STFLSTMUNet
from stfunet.graph import TrainStepGraph
from stfunet.optim import AdamW
from stfunet.synthetic import dce_batch

dev = torch.device("cuda")
model = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=8).to(dev).train()
opt = AdamW(model.parameters(), lr=1e-3, capturable=True)
x, t = dce_batch(16, 8, 256, 256, seed=1, device=dev, mask_hw=(128, 128))
for _ in range(4):
    loss = engine.criterion(model(x), t)
    opt.zero_grad()
    loss.backward()
    opt.step()
loss = None
torch.cuda.synchronize()
g = TrainStepGraph(model, opt, engine.criterion, x, t).capture()
for _ in range(3):
    g.step()
torch.cuda.synchronize()
host = []
t0 = time.perf_counter()
for _ in range(a.steps):
    c0 = time.perf_counter()
    g.graph.replay()
    host.append(time.perf_counter() - c0)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
host.sort()
print(f"graph replay: host per replay() median {host[len(host) // 2] * 1e3:.3f} ms (min {host[0] * 1e3:.3f}, "
      f"max {host[-1] * 1e3:.3f}); loop {1e3 * (t1 - t0) / a.steps:.3f} ms/step, wall incl. drain "
      f"{1e3 * (t2 - t0) / a.steps:.3f} ms/step")
# synced one at a time: GPU time of one replay with nothing queued behind it
w = []
for _ in range(5):
    torch.cuda.synchronize()
    c0 = time.perf_counter()
    g.graph.replay()
    torch.cuda.synchronize()
    w.append(time.perf_counter() - c0)
print(f"one replay synced: {min(w) * 1e3:.3f} ms (median {sorted(w)[2] * 1e3:.3f})")
