"""Optimizer / LR-schedule restatement (test infrastructure).

* ``adamw_step``: ``torch.optim.AdamW(lr, betas=(0.9, 0.999), weight_decay=1e-4,
  eps=1e-8)`` as built at ``train.py:230-237`` (decoupled decay, bias-corrected,
  PyTorch's evaluation order: p *= 1 - lr*wd; m, v update;
  p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)).
* ``lr_factor``: the ``LambdaLR`` lambda of ``create_lr_scheduler``
  (``train_utils/train_and_eval.py:414-438``): linear warm-up from
  ``warmup_factor`` over ``warmup_epochs * num_step`` iterations, then
  ``(1 - progress) ** 0.9``.
"""
import math

import torch


def adamw_step(params, grads, exp_avg, exp_avg_sq, step, lr=1e-3, betas=(0.9, 0.999),
               eps=1e-8, weight_decay=1e-4):
    """In-place AdamW over lists of fp32 tensors; ``step`` is the 1-based count."""
    b1, b2 = betas
    bc1 = 1.0 - b1 ** step
    bc2 = 1.0 - b2 ** step
    for p, g, m, v in zip(params, grads, exp_avg, exp_avg_sq):
        p.mul_(1.0 - lr * weight_decay)
        m.lerp_(g, 1.0 - b1)
        v.mul_(b2).addcmul_(g, g, value=1.0 - b2)
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(m, denom, value=-lr / bc1)


def lr_factor(x, num_step, epochs, warmup=True, warmup_epochs=1, warmup_factor=1e-3):
    if not warmup:
        warmup_epochs = 0
    w = warmup_epochs * num_step
    if warmup and x <= w:
        alpha = float(x) / w
        return warmup_factor * (1 - alpha) + alpha
    return (1 - (x - w) / ((epochs - warmup_epochs) * num_step)) ** 0.9
