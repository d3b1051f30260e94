"""Per-launch census of one training step's GEMM-shaped launches (stf_igemm / stf_wgrad) in issue
order: shape, device kernel, stream, duration (HIP events on the launching stream; side-stream
launches overlap the main stream, so their times are shared-machine numbers).
    python tools/gemm_census.py [--model unet|stf] [--config 2|3|4] [--top N]"""
import argparse
import os
import sys
from collections import defaultdict
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="stf")
ap.add_argument("--time-steps", type=int, default=8)
ap.add_argument("--batch", type=int, default=None)
ap.add_argument("--top", type=int, default=40)
a = ap.parse_args()
from stfunet import STFLSTMUNet, UNet, engine, nhwc
from stfunet.optim import AdamW
from stfunet.synthetic import dce_batch
dev = torch.device("cuda")
if a.model == "unet":
    b = a.batch or 64
    m = UNet(in_channels=a.time_steps, num_classes=2, base_c=64).to(dev)
    x, t = dce_batch(b, a.time_steps, 256, 256, seed=1, device=dev)
    x = x.flatten(1, 2)
else:
    b = a.batch or 16
    m = STFLSTMUNet(time_steps=a.time_steps).to(dev)
    x, t = dce_batch(b, a.time_steps, 256, 256, seed=1, device=dev, mask_hw=(128, 128))
m.train()
opt = AdamW(m.parameters(), lr=1e-3)
for i in range(3):
    if i == 2:
        nhwc.TIMER = nhwc.KernelTimer(log=True)
    loss = engine.criterion(m(x), t)
    opt.zero_grad()
    loss.backward()
    opt.step()
torch.cuda.synchronize()
log = nhwc.TIMER.log
nhwc.TIMER = None
main = torch.cuda.current_stream().stream_id
rows = [(desc, fam, e0.elapsed_time(e1) * 1e3, sid, fl) for desc, fam, e0, e1, sid, fl in log]
print(f"{len(rows)} launches; main stream {sum(r[2] for r in rows if r[3] == main) / 1e3:.3f} ms, "
      f"side streams {sum(r[2] for r in rows if r[3] != main) / 1e3:.3f} ms")
agg = defaultdict(lambda: [0, 0.0, 0.0])
for desc, fam, us, sid, fl in rows:
    k = (desc, fam[:48], "main" if sid == main else "side")
    agg[k][0] += 1
    agg[k][1] += us
    agg[k][2] += fl
print(f"{'us total':>9} {'n':>3} {'TF/s':>6}  stream  shape / kernel")
for (desc, fam, st), (n, us, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
    print(f"{us:9.1f} {n:3d} {fl / (us * 1e-6) / 1e12 if us > 0 else 0:6.0f}  {st:5}  {desc}  |  {fam}")
