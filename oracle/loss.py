"""Vectorised restatement of the reference training criterion (test infrastructure).

Reference: ``criterion`` ``train_utils/train_and_eval.py:299-313`` =
``cross_entropy(x, target, ignore_index=-100)`` + ``dice_loss(x, build_target(target),
multiclass=True, ignore_index=-100)`` with

* ``build_target``           ``dice_coefficient_loss.py:5-17`` (one-hot, NCHW; with
  ignore_index < 0 no masking happens)
* ``dice_coeff``             ``dice_coefficient_loss.py:20-39``:
  per image ``(2*sum(p*t) + eps) / (sum(p) + sum(t) + eps)``, eps = 1e-6, and when
  ``sum(p) + sum(t) == 0`` the denominator sum becomes ``2*inter`` (:34-35);
  averaged over the batch
* ``multiclass_dice_coeff``  ``dice_coefficient_loss.py:42-48``: mean over classes
* ``dice_loss``              ``dice_coefficient_loss.py:51-55``: ``1 - coeff(softmax(x))``

The per-image Python loop and the host-synchronising ``if`` of the reference
are replaced by reductions and a ``torch.where`` (same value).
"""
import torch
import torch.nn.functional as F

DICE_EPS = 1e-6


def dice_terms(logits, target, num_classes=2):
    """Per (image, class) sums: inter = sum p*t, psum = sum p, tsum = sum t."""
    p = torch.softmax(logits.float(), dim=1)
    t = F.one_hot(target, num_classes).permute(0, 3, 1, 2).to(p.dtype)
    inter = (p * t).flatten(2).sum(-1)
    psum = p.flatten(2).sum(-1)
    tsum = t.flatten(2).sum(-1)
    return inter, psum, tsum


def dice_coeff_from_terms(inter, psum, tsum, eps=DICE_EPS):
    sets = psum + tsum
    sets = torch.where(sets == 0, 2 * inter, sets)
    per = (2 * inter + eps) / (sets + eps)          # [B, C]
    return per.mean(0).mean()                       # batch mean, then class mean


def criterion(logits, target, num_classes=2, ignore_index=-100):
    """CE + multiclass Dice loss; ``logits`` [B,C,H,W], ``target`` int64 [B,H,W]."""
    ce = F.cross_entropy(logits.float(), target, ignore_index=ignore_index)
    inter, psum, tsum = dice_terms(logits, target, num_classes)
    return ce + (1.0 - dice_coeff_from_terms(inter, psum, tsum))
