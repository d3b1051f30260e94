"""evaluate() per-batch metric cost at cfg2's output (64 x 2 x 256^2 logits): the fused
stf_eval_counts pass vs the reference's metric classes run with torch ops on the same
GPU tensors (softmax + argmax + bincount + per-class sums with a host sync per class)."""
import os
import sys
import time
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from stfunet import engine

B, K, H = 64, 2, 256
logits = torch.randn(B, K, H, H, device="cuda")
target = torch.randint(0, K, (B, H, H), device="cuda")


def fused():
    cm, dc = engine.ConfusionMatrix(K), engine.DiceCoefficient(K, ignore_index=255)
    engine.eval_update(logits, target, cm, dc)
    return cm, dc


def torch_ops():
    cm, dc = engine.ConfusionMatrix(K), engine.DiceCoefficient(K, ignore_index=255)
    cm.update(target.flatten(), logits.argmax(1).flatten())
    p = torch.softmax(logits, 1).argmax(1)        # the reference's DiceCoefficient.update
    keep = target != 255
    p, t = (p * keep).view(-1), (target * keep).view(-1)
    for c in range(K):
        u = (p == c).float().sum() + (t == c).float().sum()
        if u > 0:                                  # host sync, as in the reference
            pass
    return cm, dc


for name, fn in (("fused stf_eval_counts", fused), ("torch ops (reference style)", torch_ops)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    print(f"{name:30s} {(time.perf_counter() - t0) / 20 * 1e6:8.1f} us per batch (wall, incl. host)")
