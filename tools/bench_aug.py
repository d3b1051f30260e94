"""Training-augmentation throughput at cfg3's input (B=16 samples x T=8 DCE frames + mask,
256x256 uint8 sources, get_transform(train) parameters -> 224^2 crops):

* device: DeviceAugment end to end (host draws + tables + one pinned H2D copy + the three
  kernels), wall clock per batch, and the kernels alone (HIP events on the launch stream)
* CPU: the reference's per-frame Pillow pipeline on one core, as its DataLoader workers
  run it (Pillow resize / transpose / rotate, numpy crop, to_tensor + normalize via torch),
  and the numpy restatement (oracle/augment.py, the "port")

Prints one JSON line (samples/s)."""
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "stf-unet_amd")]
import numpy as np
import torch

from stfunet.augment import DeviceAugment

B, T, H = 16, 8, 256
rng = np.random.default_rng(0)
frames = [rng.integers(0, 256, (T, H, H), dtype=np.uint8) for _ in range(B)]
masks = [(rng.random((H, H)) < 0.3).astype(np.uint8) for _ in range(B)]
aug = DeviceAugment(seed=1, device="cuda")

for _ in range(3):
    aug(frames, masks)
torch.cuda.synchronize()
N = 30
t0 = time.perf_counter()
for _ in range(N):
    x, t = aug(frames, masks)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / N

params = [aug.draw_sample(T, H, H) for _ in range(B)]
s = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(2):
    aug(frames, masks, params)
torch.cuda.synchronize()
# kernels only: stage once, time repeated launches of the same staged batch
st = aug(frames, masks, params, launch=False)
aug.launch(st)
torch.cuda.synchronize()
e0.record(s)
for _ in range(N):
    aug.launch(st)
e1.record(s)
torch.cuda.synchronize()
ms = [e0.elapsed_time(e1) / N]
gpu_stream = float(np.median(ms)) / 1e3

from PIL import Image                                           # noqa: E402
from oracle import augment as A                                 # noqa: E402


def pil_sample(fr, m, p):
    out = []
    for img in list(fr) + [m]:
        im = Image.fromarray(img)
        rs = Image.BILINEAR if len(out) < T else Image.NEAREST
        im = im.resize((p["w2"], p["h2"]), rs)
        if p["hflip"]:
            im = im.transpose(Image.FLIP_LEFT_RIGHT)
        if p["vflip"]:
            im = im.transpose(Image.FLIP_TOP_BOTTOM)
        if p["angle"] is not None:
            im = im.rotate(p["angle"], resample=rs, expand=False)
        a = A.crop(np.array(im), 224, p["h0"], p["w0"])
        out.append(A.normalize(a) if len(out) < T else a.astype(np.int64))
    return out


torch.set_num_threads(1)
t0 = time.perf_counter()
for b in range(B):
    pil_sample(frames[b], masks[b], params[b][0])
pil = (time.perf_counter() - t0) / B
t0 = time.perf_counter()
for b in range(4):
    A.sample(frames[b], masks[b], params[b])
port = (time.perf_counter() - t0) / 4
print(json.dumps({
    "metric": "augmented samples/s (T=8 frames + mask, 256^2 -> 224^2)", "batch": B,
    "device_wall_samples_per_s": round(B / wall, 1), "device_stream_samples_per_s": round(B / gpu_stream, 1),
    "device_ms_per_batch_wall": round(wall * 1e3, 3), "device_ms_per_batch_stream": round(gpu_stream * 1e3, 3),
    "cpu_pillow_1core_samples_per_s": round(1 / pil, 1), "cpu_port_1core_samples_per_s": round(1 / port, 2)}))
