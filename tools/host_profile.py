"""cProfile of the host side of N training steps (bench.py's model/data/optimizer):
where the Python/ctypes enqueue time of a step goes.
    python tools/host_profile.py [--model stf] [--steps 5] [--top 30]"""
import argparse
import cProfile
import os
import pstats
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="stf")
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--top", type=int, default=30)
a = ap.parse_args()
from stfunet import engine, STFLSTMUNet, UNet
from stfunet.optim import AdamW
from stfunet.synthetic import dce_batch

dev = torch.device("cuda")
if a.model == "unet":
    model, B, half = UNet(in_channels=8, num_classes=2, base_c=64).to(dev), 64, None
else:
    model, B, half = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=8).to(dev), 16, (128, 128)
model.train()
opt = AdamW(model.parameters(), lr=1e-3)
sched = engine.create_lr_scheduler(opt, 100, 10, warmup=True)
x, t = dce_batch(B, 8, 256, 256, seed=1, device=dev, mask_hw=half)
x = engine.preprocess_input(x, model)


def step():
    loss = engine.criterion(model(x), t)
    opt.zero_grad()
    loss.backward()
    opt.step()
    sched.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
# backward on this thread, so that cProfile sees the programs' backward schedule too
torch.autograd.set_multithreading_enabled(False)
pr = cProfile.Profile()
pr.enable()
for _ in range(a.steps):
    step()
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(a.top)
st.sort_stats("cumulative").print_stats(a.top)
