"""List every implicit-GEMM / wgrad launch of one STF (or UNet) training step with its
shape, chosen device kernel and FLOPs, aggregated (launch counts per shape).  Weight
gradients run inline (STF_WGRAD_SIDE=0) so that the events bracket them.
    python tools/stf_shapes.py [--unet]"""
import os
import sys
from collections import defaultdict
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
os.environ["STF_WGRAD_SIDE"] = "0"
import torch
from stfunet import nhwc, engine, STFLSTMUNet, UNet
from stfunet.synthetic import dce_batch

log = defaultdict(lambda: [0, 0.0])
evs = defaultdict(list)
TIME = False
orig_igemm, orig_wgrad = nhwc.igemm, nhwc.wgrad


def igemm(src, wgt, nout, dst, R, S, stride, pad, transposed=False, **kw):
    e0 = torch.cuda.Event(enable_timing=True); e0.record()
    r = orig_igemm(src, wgt, nout, dst, R, S, stride, pad, transposed=transposed, **kw)
    e1 = torch.cuda.Event(enable_timing=True); e1.record()
    Hd, Wd = (dst.H // 2, dst.W // 2) if kw.get("scatter2x2") else (dst.H, dst.W)
    fl = 2.0 * src.N * Hd * Wd * nout * R * S * src.C / (stride * stride if transposed else 1)
    key = (f"igemm {src.N}x{src.H}x{src.W}x{src.C} -> {Hd}x{Wd}x{nout} k{R}s{stride}"
           f"{' T' if transposed else ''}{' sc' if kw.get('scatter2x2') else ''}{' lstm' if kw.get('lstm') else ''}"
           f"{' bnr' if kw.get('bnr') else ''}")
    if TIME:
        log[key][0] += 1
        log[key][1] += fl
        evs[key].append((e0, e1))
    return r


def wgrad(dy, x, R, S, stride, pad, out, **kw):
    e0 = torch.cuda.Event(enable_timing=True); e0.record()
    r = orig_wgrad(dy, x, R, S, stride, pad, out, **kw)
    e1 = torch.cuda.Event(enable_timing=True); e1.record()
    key = f"wgrad dy {dy.N}x{dy.H}x{dy.W}x{dy.C} x {x.H}x{x.W}x{x.C} k{R}s{stride}"
    if TIME:
        log[key][0] += 1
        log[key][1] += 2.0 * dy.N * dy.H * dy.W * dy.C * R * S * x.C
        evs[key].append((e0, e1))
    return r


nhwc.igemm, nhwc.wgrad = igemm, wgrad
dev = torch.device("cuda")
if "--unet" in sys.argv:
    model, B, half = UNet(in_channels=8, num_classes=2, base_c=64).to(dev), 64, None
else:
    model, B, half = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=8).to(dev), 16, (128, 128)
model.train()
x, t = dce_batch(B, 8, 256, 256, seed=1, device=dev, mask_hw=half)
x = engine.preprocess_input(x, model)
for it in range(3):
    TIME = it == 2
    for p in model.parameters():
        p.grad = None
    loss = engine.criterion(model(x), t)
    loss.backward()
    torch.cuda.synchronize()
tot = 0.0
for k, (n, fl) in sorted(log.items(), key=lambda kv: -sum(a.elapsed_time(b) for a, b in evs[kv[0]])):
    ms = sum(a.elapsed_time(b) for a, b in evs[k])
    tot += ms
    print(f"{n:3d} x {fl / n / 1e9:8.2f} GF {ms / n * 1e3:8.1f} us {fl / ms / 1e9:7.1f} TF/s  {k}")
print(f"total {tot:.3f} ms (each launch timed alone: events between launches)")
