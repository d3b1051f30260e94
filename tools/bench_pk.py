"""PK-map fit throughput (stf_tofts_fit) on one synthetic 256x256 slice, 8 time points,
with the reference's schedule (batches of 1,024 tissue pixels, 100 epochs), beside the
fp32 CPU oracle on a bounded sample.  Prints one JSON line.
    python tools/bench_pk.py [H] [--cpu-pixels N]"""
import json
import os
import sys
import time
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import numpy as np
import torch
from stfunet.pk import ToftsModelFitter

H = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 256
cpu_px = int(sys.argv[sys.argv.index("--cpu-pixels") + 1]) if "--cpu-pixels" in sys.argv else 4096
T = 8
g = torch.Generator().manual_seed(7)
yy, xx = torch.meshgrid(torch.arange(H), torch.arange(H), indexing="ij")
tissue = (((yy - H / 2) / (0.45 * H)) ** 2 + ((xx - H / 2) / (0.42 * H)) ** 2) < 1
t = torch.arange(T, dtype=torch.float32)
P = int(tissue.sum())
curves = (0.2 + 0.6 * torch.rand(P, 1, generator=g)) * (1 - torch.exp(-(0.05 + 0.25 * torch.rand(P, 1, generator=g)) * t))
curves = (curves + 0.01 * torch.randn(P, T, generator=g)).contiguous()
f = ToftsModelFitter()
cur = curves.cuda()
f.fit_curves(cur[:1024], epochs=2)            # warm-up (tables, code object)
torch.cuda.synchronize()
s = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
f.fit_curves(cur)
e1.record(s)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
nv = f._tables(f.time_points)[4].cpu()
terms = 100 * int(nv.sum()) * P                  # exp terms (Tofts convolution) evaluated in the fit
# CPU oracle on a bounded sample: one batch of cpu_px pixels for 2 epochs, per pixel-epoch
from oracle import pk as o_pk
threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
threads = min(threads, 16)
torch.set_num_threads(threads)
t0 = time.perf_counter()
o_pk.fit(curves[:cpu_px], t, batch=1024, epochs=4)
cpu_s = time.perf_counter() - t0
cpu_px_per_s = cpu_px * 4 / cpu_s / 100           # whole 100-epoch pixel fits per second
print(json.dumps({
    "metric": "PK-map fit (extended Tofts, 100 epochs per-pixel Adam) tissue pixels/s",
    "value": round(P / (ms / 1e3), 1), "unit": "pixels/s", "slice": [H, H], "tissue_pixels": P, "time_points": T,
    "batches": (P + 1023) // 1024, "ms": round(ms, 3), "exp_terms": terms,
    "gexp_per_s": round(terms / (ms / 1e3) / 1e9, 1),
    "cpu_baseline": {"value": round(cpu_px_per_s, 2), "unit": "pixels/s", "cores": threads, "kind": "port",
                     "sample": f"oracle fp32 fit of {cpu_px} pixels (4 batches of 1024) x 4 epochs ({cpu_s:.3f} s), per 100-epoch fit"}}))
