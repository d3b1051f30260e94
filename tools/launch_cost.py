"""Host cost of the launch paths: a plan replay vs its op count, and single library calls.
    python tools/launch_cost.py [--config 3]"""
import argparse
import ctypes
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "stf-unet_amd"))

import torch  # noqa: E402


def per_call(fn, n=2000):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / n * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    a = ap.parse_args()
    from stfunet import STFLSTMUNet, _lib, engine, nhwc
    from stfunet.optim import AdamW
    from stfunet.synthetic import dce_batch
    dev = torch.device("cuda")
    lib = _lib.load()
    s = _lib.stream()
    buf = torch.zeros(1024, device=dev)
    src = torch.randn(64, 64, device=dev)
    dst = torch.empty(64, 64, device=dev)
    side = torch.cuda.Stream()
    print(f"stf_memset (hipMemsetAsync)      {per_call(lambda: lib.stf_memset(buf.data_ptr(), 0, 4096, s)):7.2f} us")
    print(f"stf_copy_rows (1 kernel)         "
          f"{per_call(lambda: lib.stf_copy_rows(src.data_ptr(), 64, dst.data_ptr(), 64, 64, 64, s)):7.2f} us")
    print(f"stf_stream_wait (record+wait)    "
          f"{per_call(lambda: lib.stf_stream_wait(side.cuda_stream, torch.cuda.current_stream().cuda_stream)):7.2f} us")
    print(f"torch zero_ (1 kernel)           {per_call(lambda: buf.zero_()):7.2f} us")
    # a plan of the tiny kernel replayed
    from stfunet.plan import Plan
    p = Plan()
    p.record(lambda: [lib.stf_copy_rows(src.data_ptr(), 64, dst.data_ptr(), 64, 64, 64, s) for _ in range(500)])
    print(f"plan replay, 500 tiny kernels    {per_call(lambda: p.replay(), 20) / 500:7.2f} us per op")
    p2 = Plan()
    p2.record(lambda: [lib.stf_stream_wait(side.cuda_stream, torch.cuda.current_stream().cuda_stream)
                       for _ in range(500)])
    print(f"plan replay, 500 stream waits    {per_call(lambda: p2.replay(), 20) / 500:7.2f} us per op")
    # the STF step's plans
    torch.manual_seed(0)
    m = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=8).to(dev).train()
    opt = AdamW(m.parameters(), lr=1e-3)
    x, t = dce_batch(16, 8, 256, 256, seed=0, device=dev, mask_hw=(128, 128))
    for i in range(3):
        loss = engine.criterion(m(x), t)
        opt.zero_grad()
        loss.backward()
        opt.step()
    rt = m.program.runtime
    for name, pl in (("forward", rt.fwd), ("backward", rt.bwd)):
        us = per_call(lambda: pl.replay(), 10)
        print(f"STF cfg3 {name} plan: {pl.n} ops, replay host {us / 1e3:.3f} ms = {us / pl.n:.2f} us per op")


if __name__ == "__main__":
    main()
