"""Training criterion on the gfx950 loss kernels.

Mirrors ``criterion`` (train_utils/train_and_eval.py:299-313): for every output
head, cross-entropy + multiclass Dice loss on the softmax
(train_utils/dice_coefficient_loss.py:5-55), ``losses['out'] + 0.5 *
losses['aux']`` when an aux head is present.  The reference's per-image Python
loop and its ``if sets_sum == 0`` host sync (dice_coefficient_loss.py:24-35)
become two kernels with a branch-free empty-set rule; the scalar loss stays on
the device.
"""
import torch

from . import _lib
from .nhwc import _p
from ._lib import call, stream


class _CEDice(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        logits = logits.detach().contiguous().float()
        target = target.contiguous()
        if target.dtype != torch.int64:
            target = target.long()
        N, K, H, W = logits.shape
        assert target.shape == (N, H, W), f"target {tuple(target.shape)} vs logits {tuple(logits.shape)}"
        terms = torch.empty(_lib.load().stf_loss_scratch_floats(N, K), dtype=torch.float32, device=logits.device)
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        call("stf_loss_fwd", _p(logits), _p(target), N, H, W, K, _p(terms), _p(loss), stream())
        ctx.save_for_backward(logits, target, terms)
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        logits, target, terms = ctx.saved_tensors
        N, K, H, W = logits.shape
        go = grad_out.detach().float().contiguous().reshape(1)
        dl = torch.empty_like(logits)
        call("stf_loss_bwd", _p(logits), _p(target), N, H, W, K, _p(terms), _p(go), _p(dl), stream())
        return dl, None


def ce_dice_loss(logits, target):
    if not logits.is_cuda:
        raise RuntimeError("stfunet loss kernels need a ROCm device (no CPU fallback)")
    return _CEDice.apply(logits, target)


def criterion(inputs, target, loss_weight=None, num_classes: int = 2, dice: bool = True, ignore_index: int = -100):
    """Same signature and reduction as the reference ``criterion``.

    Supported configuration is the one the reference trains with
    (train_and_eval.py:395): no class weights, Dice on, ignore_index -100
    (targets never hold it: the reference's one-hot would fail on it).
    """
    if loss_weight is not None or not dice or ignore_index >= 0:
        raise NotImplementedError("stfunet.criterion implements the reference training configuration "
                                  "(loss_weight=None, dice=True, ignore_index=-100)")
    losses = {name: ce_dice_loss(x, target) for name, x in inputs.items()}
    if len(losses) == 1:
        return losses["out"]
    return losses["out"] + 0.5 * losses["aux"]
