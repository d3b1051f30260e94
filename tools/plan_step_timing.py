"""Where a plan-replayed training step spends its time, without a profiler in the way.

Per step: host time to enqueue (forward / criterion / backward / optimizer, no sync),
and the GPU time of each phase from HIP events on the main stream (the host runs ahead
of the GPU with plans, so consecutive events measure the GPU's own critical path).
    python tools/plan_step_timing.py --config 3 [--steps 20]
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "stf-unet_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 4, 5])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    a = ap.parse_args()
    from stfunet import STFLSTMUNet, UNet, engine
    from stfunet.optim import AdamW
    from stfunet.synthetic import dce_batch
    cfg = {2: ("unet", 64, 256, 8, False), 3: ("stf", 16, 256, 8, False), 4: ("stf", 16, 256, 16, False),
           5: ("stf", 4, 512, 32, True)}[a.config]
    which, B, hw, T, pk = cfg
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = (UNet(in_channels=T, num_classes=2, base_c=64) if which == "unet" else
             STFLSTMUNet(in_channels=1, num_classes=2, time_steps=T, use_pk_maps=pk)).to(dev).train()
    fp16 = a.config == 5
    model.storage_dtype = torch.float16 if fp16 else torch.bfloat16
    scaler = torch.amp.GradScaler("cuda") if fp16 else None
    opt = AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
    half = (hw // 2, hw // 2) if which == "stf" else None
    batches = [dce_batch(B, T, hw, hw, seed=i, device=dev, pk_channels=3 if pk else 0, mask_hw=half) for i in range(2)]
    batches = [(engine.preprocess_input(x, model), t) for x, t in batches]
    evs = []

    def step(i, record):
        x, t = batches[i % 2]
        e = [torch.cuda.Event(enable_timing=True) for _ in range(5)] if record else None
        h = [time.perf_counter()]
        if e:
            e[0].record()
        with torch.amp.autocast("cuda", enabled=fp16):
            out = model(x)
        h.append(time.perf_counter())
        if e:
            e[1].record()
        with torch.amp.autocast("cuda", enabled=fp16):
            loss = engine.criterion(out, t)
        opt.zero_grad()
        if e:
            e[2].record()
        h.append(time.perf_counter())
        (scaler.scale(loss) if scaler else loss).backward()
        h.append(time.perf_counter())
        if e:
            e[3].record()
        if scaler:
            scaler.step(opt)
            scaler.update()
        else:
            opt.step()
        if e:
            e[4].record()
        h.append(time.perf_counter())
        if e:
            evs.append((e, h))

    for i in range(a.warmup):
        step(i, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i, True)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    names = ["forward", "criterion", "backward", "optimizer"]
    gpu = [sum(e[k].elapsed_time(e[k + 1]) for e, _ in evs[2:]) / len(evs[2:]) for k in range(4)]
    host = [sum((h[k + 1] - h[k]) * 1e3 for _, h in evs[2:]) / len(evs[2:]) for k in range(4)]
    step_gpu = sum(evs[k][0][0].elapsed_time(evs[k + 1][0][0]) for k in range(2, len(evs) - 1)) / (len(evs) - 3)
    print(f"config {a.config} ({which}, B={B}, {hw}^2, T={T}{', PK' if pk else ''}), plan={os.environ.get('STF_PLAN', '1')}: "
          f"wall {wall:.3f} ms/step, GPU step (event to event) {step_gpu:.3f} ms")
    for n, g, hh in zip(names, gpu, host):
        print(f"  {n:10s} GPU {g:7.3f} ms   host enqueue {hh:7.3f} ms")
    print(f"  host enqueue total {sum(host):.3f} ms; GPU phases total {sum(gpu):.3f} ms")


if __name__ == "__main__":
    main()
