"""Evaluation-metric restatement (test infrastructure).

* ``confusion_matrix``: ``ConfusionMatrix.update`` ``train_and_eval.py:30-39``
  (rows = target class, cols = predicted class; target outside [0, n) ignored).
* ``dice_per_class``: ``DiceCoefficient.update`` ``train_and_eval.py:80-118``:
  argmax(softmax(out)); with ignore_index, pred and target are *multiplied* by the
  keep-mask (so ignored pixels count as class 0, :87-90); per class
  2|P&T| / (|P|+|T|), and 1.0 when the class is absent from both (:104-107).
  ``DiceCoefficient.value`` = mean over classes of the per-batch average (:120-138).
"""
import numpy as np
import torch


def confusion_matrix(target, pred, n):
    t = target.flatten().to(torch.int64)
    p = pred.flatten().to(torch.int64)
    k = (t >= 0) & (t < n)
    return torch.bincount(n * t[k] + p[k], minlength=n * n).reshape(n, n)


def dice_per_class(logits, target, num_classes=2, ignore_index=None):
    pred = torch.argmax(torch.softmax(logits, dim=1), dim=1)      # :84-85
    if ignore_index is not None:
        keep = (target != ignore_index)
        pred = pred * keep
        target = target * keep
    pred = pred.flatten()
    target = target.flatten()
    out = []
    for c in range(num_classes):
        pc = (pred == c)
        tc = (target == c)
        union = pc.sum().item() + tc.sum().item()
        inter = (pc & tc).sum().item()
        out.append(2.0 * inter / union if union > 0 else 1.0)
    return np.array(out, dtype=np.float64)
