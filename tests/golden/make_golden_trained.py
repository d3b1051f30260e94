"""Trained-weight Dice fixture, produced by running the REFERENCE training code (build container only).

    python tests/golden/make_golden_trained.py  [--ref /root/reference]

Why: at initialisation the logits sit near 0, so a handful of argmax flips move Dice by ~1e-3 and
"Dice equal to the reference" says nothing about the kernels.  After training the predictions are
confident and Dice is a meaningful parity point.

What it does (reference modules imported by path, as in ``make_golden.py``):

1. ``src/unet.py`` ``UNet(in_channels=8, num_classes=2, base_c=8)`` from ``oracle.init``'s canonical
   weights (seed 0), trained by the reference's own ``train_one_epoch`` (``train_and_eval.py:377-411``:
   ``criterion`` = CE + Dice, ``torch.optim.AdamW(fused=True)`` with ``train.py:230-237``'s
   hyper-parameters, ``create_lr_scheduler`` per iteration) for ``EPOCHS`` x ``STEPS`` steps of
   ``dce_case`` batches ([B=4, T=8, 1, 64, 64], seeds 1000+).
2. Parameters rounded to bf16 (stored as uint16 bit patterns, ~1 MB); BatchNorm running statistics
   kept in fp32.  The reference model is reloaded with exactly those values.
3. The reference's ``evaluate`` (``train_and_eval.py:316-374``: eval-mode forward, ConfusionMatrix,
   DiceCoefficient(ignore_index=255)) over ``EVAL_BATCHES`` held-out batches (seeds 2000+) gives the
   golden Dice / confusion matrix; the per-pixel argmax and the logit margin (|l1 - l0|) are stored
   so a test can count flipped pixels and see how close to the boundary they were.

Output: ``tests/golden/unet_trained.npz`` (no pickles).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import load_reference  # noqa: E402
from oracle.cases import dce_case  # noqa: E402
from oracle.init import canonical_state_dict  # noqa: E402

BASE_C, B, T, HW = 8, 4, 8, 64
EPOCHS, STEPS = 12, 50
EVAL_BATCHES = 4


def train_batches(epoch):
    return [dce_case(1000 + epoch * STEPS + i, B, T, HW, HW) for i in range(STEPS)]


def eval_batches():
    return [dce_case(2000 + i, B, T, HW, HW) for i in range(EVAL_BATCHES)]


def to_bf16_bits(t):
    u = t.detach().float().contiguous().view(torch.int32).numpy().astype(np.int64) & 0xFFFFFFFF
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF          # round to nearest even (finite values)
    return r.astype(np.uint16)


def from_bf16_bits(bits, shape):
    return torch.from_numpy((bits.astype(np.uint32) << 16).view(np.float32).reshape(shape).copy())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    a = ap.parse_args()
    torch.set_num_threads(8)
    unet_mod, _, tae, _ = load_reference(a.ref)

    model = unet_mod.UNet(in_channels=8, num_classes=2, base_c=BASE_C)
    model.load_state_dict(canonical_state_dict(model.state_dict(), seed=0))
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-3,
                            betas=(0.9, 0.999), weight_decay=1e-4, eps=1e-8, fused=True)
    sched = tae.create_lr_scheduler(opt, STEPS, EPOCHS, warmup=True)
    losses = []
    for ep in range(EPOCHS):
        mean_loss, lr = tae.train_one_epoch(model, opt, train_batches(ep), torch.device("cpu"), ep, 2,
                                            lr_scheduler=sched, print_freq=1000)
        losses.append(mean_loss)
        print(f"epoch {ep}: mean loss {mean_loss:.4f} lr {lr:.2e}", flush=True)

    res = {}
    sd = model.state_dict()
    for k, v in sd.items():
        if v.is_floating_point() and "running" not in k:
            res["bf16." + k] = to_bf16_bits(v)
            sd[k] = from_bf16_bits(res["bf16." + k], v.shape)
        else:
            res["state." + k] = v.numpy().copy()
    model.load_state_dict(sd)

    ev = eval_batches()
    metrics = tae.evaluate(model, ev, torch.device("cpu"), num_classes=2)
    model.eval()
    preds, margins = [], []
    with torch.no_grad():
        for x5, _ in ev:
            lo = model(tae.preprocess_input(x5, model))["out"]
            preds.append(lo.argmax(1).numpy().astype(np.uint8))
            margins.append((lo[:, 1] - lo[:, 0]).abs().numpy().astype(np.float32))
    pred = np.concatenate(preds)
    res.update(
        dice=np.array(metrics["dice"]),
        confmat=metrics["confusion_matrix"].mat.numpy(),
        pred_bits=np.packbits(pred.reshape(-1)),
        pred_shape=np.array(pred.shape),
        margin=np.concatenate(margins).astype(np.float16),
        train_losses=np.array(losses),
        config=np.array([BASE_C, B, T, HW, EPOCHS, STEPS, EVAL_BATCHES]),
    )
    np.savez_compressed(os.path.join(a.out, "unet_trained.npz"), **res)
    m = np.concatenate(margins)
    print(json.dumps({"dice": metrics["dice"], "confmat": metrics["confusion_matrix"].mat.tolist(),
                      "margin_lt_1e-2": int((m < 1e-2).sum()), "margin_lt_1e-1": int((m < 1e-1).sum()),
                      "pixels": int(m.size)}, indent=1))


if __name__ == "__main__":
    main()
