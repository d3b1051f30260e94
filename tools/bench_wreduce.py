#!/usr/bin/env python3
"""Micro-bench of stf_wgrad_reduce over the split plans the UNet / STF steps use (set STF_LIB to
time another build of the library).  Prints one line per (splits, Nout, Cs, taps) case."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "stf-unet_amd"))
import torch  # noqa: E402
from stfunet._lib import call, stream  # noqa: E402

CASES = [(512, 64, 64, 9), (256, 64, 64, 9), (256, 64, 128, 9), (128, 128, 128, 9), (64, 256, 256, 9),
         (32, 256, 256, 9), (16, 512, 512, 9), (8, 512, 512, 9), (4, 1024, 512, 9), (4, 512, 512, 9),
         (2, 1024, 1024, 9), (14, 512, 512, 9)]
dev = torch.device("cuda")
tot_ms = 0.0
for splits, nout, cs, taps in CASES:
    total = nout * cs * taps
    ws = torch.randn(splits * total, device=dev)
    out = torch.empty(total, device=dev)
    for _ in range(3):
        call("stf_wgrad_reduce", ws.data_ptr(), splits, nout, 3, 3, cs, out.data_ptr(), stream())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        call("stf_wgrad_reduce", ws.data_ptr(), splits, nout, 3, 3, cs, out.data_ptr(), stream())
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    ref = ws.view(splits, nout, taps, cs).double().sum(0).permute(0, 2, 1).reshape(-1).float()
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    tot_ms += us / 1e3
    print(f"splits {splits:4d} Nout {nout:5d} Cs {cs:5d}: {us:8.2f} us  {splits * total * 4 / us / 1e3:7.1f} GB/s  "
          f"max rel err {err:.1e}", flush=True)
print(f"TOTAL {tot_ms:.3f} ms")
