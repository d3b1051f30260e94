"""Fused evaluation counts (stf_eval_counts via engine.eval_update / evaluate) vs the
reference metric classes' semantics (oracle/metrics.py, pinned by
tests/golden/metrics_kat.npz): confusion matrix and Dice bit-exact (integer counts)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_eval_counts_known_answers():
    from stfunet import engine
    g = np.load(os.path.join(GOLDEN, "metrics_kat.npz"))
    cm = engine.ConfusionMatrix(2)
    dc = engine.DiceCoefficient(2, ignore_index=255)
    engine.eval_update(torch.from_numpy(g["logits"]).cuda(), torch.from_numpy(g["target"]).cuda(), cm, dc)
    assert np.array_equal(cm.mat.cpu().numpy(), g["confmat"])
    engine.eval_update(torch.from_numpy(g["logits_absent"]).cuda(), torch.from_numpy(g["target_absent"]).cuda(),
                       cm, dc)
    assert np.allclose(dc.compute().cpu().numpy(), g["dice_per_class"], atol=1e-6)
    assert abs(dc.value.item() - float(g["dice_value"])) < 1e-6


@pytest.mark.parametrize("K,ignore_frac,ties", [(2, 0.1, False), (4, 0.0, True), (3, 0.3, True)])
def test_eval_counts_random(K, ignore_frac, ties):
    from oracle import metrics as o_metrics
    from stfunet import engine
    torch.manual_seed(K)
    B, H, W = 3, 37, 53
    logits = torch.randn(B, K, H, W)
    if ties:                                    # exact ties: the first maximum wins
        logits[:, 1] = logits[:, 0]
    target = torch.randint(0, K, (B, H, W))
    target[torch.rand(B, H, W) < ignore_frac] = 255
    cm = engine.ConfusionMatrix(K)
    dc = engine.DiceCoefficient(K, ignore_index=255)
    engine.eval_update(logits.cuda(), target.cuda(), cm, dc)
    ref_cm = o_metrics.confusion_matrix(target, logits.argmax(1), K)
    assert torch.equal(cm.mat.cpu(), ref_cm)
    ref_d = o_metrics.dice_per_class(logits, target, K, ignore_index=255)
    assert np.allclose(dc.compute().cpu().numpy(), ref_d, atol=1e-6)


def test_eval_dice_uses_softmax_argmax_on_near_ties():
    """DiceCoefficient.update argmaxes torch.softmax(output, 1) (train_and_eval.py:84-85)
    while the confusion matrix argmaxes the logits (:331).  Logits one ulp apart round to
    the same fp32 probability, so the two predictions differ there: engine.eval_update must
    follow each (the Dice pass is fed the device softmax, the very op the reference runs)."""
    from oracle import metrics as o_metrics
    from stfunet import engine
    torch.manual_seed(7)
    B, K, H, W = 2, 2, 64, 48
    x0 = torch.randn(B, H, W) * 3
    x1 = torch.nextafter(x0, torch.full_like(x0, float("inf")))      # class 1 wins argmax(x) by one ulp
    far = torch.rand(B, H, W) < 0.5
    x1 = torch.where(far, x0 + torch.randn(B, H, W), x1)             # half the pixels: ordinary margins
    logits = torch.stack([x0, x1], 1).cuda()
    target = torch.randint(0, K, (B, H, W)).cuda()
    target[:, :4] = 255
    sm_pred = torch.softmax(logits, 1).argmax(1)
    assert (sm_pred != logits.argmax(1)).any(), "fixture has no softmax-rounded ties"
    cm = engine.ConfusionMatrix(K)
    dc = engine.DiceCoefficient(K, ignore_index=255)
    engine.eval_update(logits, target, cm, dc)
    assert torch.equal(cm.mat.cpu(), o_metrics.confusion_matrix(target.cpu(), logits.argmax(1).cpu(), K))
    ref_d = o_metrics.dice_per_class(logits, target, K, ignore_index=255)
    assert np.allclose(dc.compute().cpu().numpy(), ref_d, atol=1e-6)    # one flipped pixel: ~2e-4
    tdc = engine.DiceCoefficient(K, ignore_index=255)                # the torch-op class, same answer
    tdc.update(logits, target)
    assert np.allclose(tdc.compute().cpu().numpy(), ref_d, atol=1e-7)
