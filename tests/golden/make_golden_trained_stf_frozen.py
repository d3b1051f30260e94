"""STF Dice fixture at CONFIDENT trained weights, produced by the REFERENCE's own training code
(build container only).

    python tests/golden/make_golden_trained_stf_frozen.py  [--ref /root/reference]

``src/stf_lstm_unet.py`` ``STFLSTMUNet(in_channels=1, num_classes=2, time_steps=4)`` (imported by
path with the standard BasicBlock ResNet-34 stand-in for the absent torchvision, as in
``make_golden.py``) starts from ``oracle.init``'s canonical weights (seed 0).  Its ResNet-34
encoder (``conv1``, ``bn1``, ``layer1..4``: 21 M of its 27 M parameters) is FROZEN at that init
(``requires_grad = False``; ``train.py:230-231`` hands AdamW only the parameters that require
grad), so the encoder weights are regenerable from the seed and need not be committed; the
LSTMs, decoders, ``upconv1``, ``final_res`` and ``final`` are trained by the reference's own
``train_one_epoch`` (``train_and_eval.py:377-411``: CE + Dice, ``torch.optim.AdamW(fused=True)``
with ``train.py:230-237``'s hyper-parameters, the per-iteration ``create_lr_scheduler``) for
``EPOCHS`` x ``STEPS`` steps of ``dce_case`` batches ([B=4, T=4, 1, 64, 64], seeds 6000+,
half-resolution 32^2 targets).  Training mode also advances the encoder's BatchNorm running
statistics, so those are committed too (fp32, small).

The fixture then holds what the reference's own ``evaluate`` (``train_and_eval.py:316-374``)
reports on ``EVAL_BATCHES`` held-out batches (seeds 7000+, 16 x 4 x 32^2 = 65,536 output pixels):
the Dice, the confusion matrix, the per-pixel argmax and |logit margin| -- and the trained
parameters rounded to bf16 (``bf16.<key>``, uint16 bit patterns), with the reference's evaluation
run on exactly those rounded weights, so a 16-bit implementation is compared at identical weights.

Output: ``tests/golden/stf_trained_frozen.npz`` (no pickles).
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
sys.path.insert(0, os.path.join(REPO, "stf-unet_amd"))
sys.path.insert(0, HERE)

from make_golden import load_reference  # noqa: E402
from oracle.cases import dce_case  # noqa: E402
from oracle.init import canonical_state_dict  # noqa: E402

B, T, HW = 4, 4, 64
EPOCHS, STEPS = 10, 40
EVAL_BATCHES = 16
ENCODER = ("conv1.", "bn1.", "layer1.", "layer2.", "layer3.", "layer4.")


def train_batches(epoch):
    return [dce_case(6000 + epoch * STEPS + i, B, T, HW, HW, target_hw=(HW // 2, HW // 2)) for i in range(STEPS)]


def eval_batches():
    return [dce_case(7000 + i, B, T, HW, HW, target_hw=(HW // 2, HW // 2)) for i in range(EVAL_BATCHES)]


def to_bf16_bits(t):
    """Round-to-nearest-even fp32 -> bf16, as uint16 bit patterns."""
    u = t.detach().float().contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).numpy().astype(np.uint16)


def from_bf16_bits(bits, shape):
    return torch.from_numpy((bits.astype(np.uint32) << 16).view(np.float32).reshape(shape).copy())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    _, stf_mod, tae, _ = load_reference(a.ref)
    model = stf_mod.STFLSTMUNet(in_channels=1, num_classes=2, time_steps=T)
    model.load_state_dict(canonical_state_dict(model.state_dict(), seed=0))
    for k, p in model.named_parameters():
        if k.startswith(ENCODER):
            p.requires_grad_(False)
    trained = [k for k, p in model.named_parameters() if p.requires_grad]
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-3,
                            betas=(0.9, 0.999), weight_decay=1e-4, eps=1e-8, fused=True)
    sched = tae.create_lr_scheduler(opt, STEPS, EPOCHS, warmup=True)
    losses = []
    for ep in range(EPOCHS):
        mean_loss, lr = tae.train_one_epoch(model, opt, train_batches(ep), torch.device("cpu"), ep, 2,
                                            lr_scheduler=sched, print_freq=1000)
        losses.append(mean_loss)
        print(f"epoch {ep}: mean loss {mean_loss:.4f} lr {lr:.2e}", flush=True)
    # round the trained parameters to bf16 and evaluate the reference on exactly those weights
    res = {}
    sd = model.state_dict()
    for k in trained:
        bits = to_bf16_bits(sd[k])
        res["bf16." + k] = bits
        sd[k] = from_bf16_bits(bits, tuple(sd[k].shape))
    for k, v in sd.items():
        if "running" in k:
            res["state." + k] = v.numpy().astype(np.float32)
        if "num_batches_tracked" in k:
            res["state." + k] = np.array(int(v))
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
    pred, margin = np.concatenate(preds), np.concatenate(margins)
    res.update(
        dice=np.array(metrics["dice"]),
        confmat=metrics["confusion_matrix"].mat.numpy(),
        pred_bits=np.packbits(pred.reshape(-1)),
        pred_shape=np.array(pred.shape),
        margin=margin.astype(np.float16),
        train_losses=np.array(losses),
        trained_keys=np.array(trained),
        config=np.array([B, T, HW, EPOCHS, STEPS, EVAL_BATCHES]),
    )
    np.savez_compressed(os.path.join(a.out, "stf_trained_frozen.npz"), **res)
    print(json.dumps({"dice": metrics["dice"], "confmat": metrics["confusion_matrix"].mat.tolist(),
                      "trained_params": int(sum(sd[k].numel() for k in trained)),
                      "margin_median": float(np.median(margin)),
                      "margin_lt_1e-2": int((margin < 1e-2).sum()), "margin_lt_1e-1": int((margin < 1e-1).sum()),
                      "pixels": int(margin.size), "losses": losses}, indent=1))


if __name__ == "__main__":
    main()
