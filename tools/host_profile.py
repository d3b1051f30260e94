"""Where the host time of a plan-replayed training step goes (cProfile of N steps after warm-up).
    python tools/host_profile.py [--config 3] [--steps 10]"""
import argparse
import cProfile
import os
import pstats
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "stf-unet_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3, choices=[2, 3])
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    from stfunet import STFLSTMUNet, UNet, engine
    from stfunet.optim import AdamW
    from stfunet.synthetic import dce_batch
    dev = torch.device("cuda")
    torch.manual_seed(0)
    if a.config == 2:
        m, B, half = UNet(in_channels=8, num_classes=2, base_c=64), 64, None
    else:
        m, B, half = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=8), 16, (128, 128)
    m = m.to(dev).train()
    opt = AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    x, t = dce_batch(B, 8, 256, 256, seed=0, device=dev, mask_hw=half)
    x = engine.preprocess_input(x, m)

    def step():
        loss = engine.criterion(m(x), t)
        opt.zero_grad()
        loss.backward()
        opt.step()

    for _ in range(4):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(30)


if __name__ == "__main__":
    main()
