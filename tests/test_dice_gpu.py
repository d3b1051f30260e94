"""Dice parity at trained weights (BASELINE north star: "Dice within 1e-4 on fixed seed").

Fixture: ``tests/golden/unet_trained.npz`` -- the reference trained UNet(in=8, base_c=8) with its own
``train_one_epoch`` (12 x 50 steps, B=4, 64^2 DCE stacks), rounded its parameters to bf16 and ran its
own ``evaluate`` (eval-mode forward, DiceCoefficient(ignore_index=255), ConfusionMatrix) on 4 held-out
batches: Dice 0.9908.  At these weights predictions are confident (9 of 65,536 pixels have a logit
margin |l1 - l0| < 1e-2), so Dice compares the kernels, not rounding noise at the decision boundary.

Tolerances:
  evaluate() on the gfx950 path, bf16 and fp16 storage: |Dice - Dice_ref| <= 1e-4; every pixel whose
      argmax differs from the reference's had a reference margin < 0.1 (a flip elsewhere is a bug).
  training from the same canonical init with the same batches and schedule on the gfx950 path
      (bf16 storage, stfunet AdamW): the trajectory is not bitwise (16-bit storage; gradients at
      initialisation are hypersensitive), so the trained model's Dice is held to
      |Dice - Dice_ref| <= 5e-3 -- the statistical parity of two training runs.
"""
import numpy as np
import pytest
import torch

import _trained

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(tr, storage):
    from stfunet.unet import UNet
    m = UNet(in_channels=8, num_classes=2, base_c=tr["base_c"])
    m.load_state_dict(_trained.shaped(tr["state"], m.state_dict()))
    m.storage_dtype = storage
    return m.to(DEV)


@pytest.mark.parametrize("storage", [torch.bfloat16, torch.float16])
def test_trained_dice_vs_reference(storage):
    from stfunet import engine
    tr = _trained.load()
    m = _model(tr, storage)
    res = engine.evaluate(m, tr["eval"], torch.device(DEV), num_classes=2)
    preds = []
    with torch.no_grad():
        for x5, _ in tr["eval"]:
            preds.append(m(engine.preprocess_input(x5, m).to(DEV))["out"].argmax(1).cpu().numpy())
    flips = np.concatenate(preds) != tr["pred"]
    worst = float(tr["margin"][flips].max()) if flips.any() else 0.0
    print(f"{storage}: dice {res['dice']:.7f} ref {tr['dice']:.7f} |d| {abs(res['dice'] - tr['dice']):.2e} "
          f"flipped pixels {int(flips.sum())} (max ref margin {worst:.3g})")
    assert abs(res["dice"] - tr["dice"]) <= 1e-4
    assert worst < 0.1
    # each flipped pixel moves one count between the two columns of its target's row
    assert np.abs(res["confusion_matrix"].mat.cpu().numpy() - tr["confmat"]).sum() == 2 * int(flips.sum())


def test_training_from_same_seed_reaches_reference_dice():
    from oracle.init import canonical_state_dict
    from stfunet import engine
    from stfunet.optim import AdamW
    from stfunet.unet import UNet
    tr = _trained.load()
    m = UNet(in_channels=8, num_classes=2, base_c=tr["base_c"])
    m.load_state_dict(canonical_state_dict(m.state_dict(), seed=0))
    m = m.to(DEV)
    opt = AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, betas=(0.9, 0.999),
                weight_decay=1e-4, eps=1e-8)
    sched = engine.create_lr_scheduler(opt, tr["steps"], tr["epochs"], warmup=True)
    for ep in range(tr["epochs"]):
        loss, _ = engine.train_one_epoch(m, opt, tr["train_batches"](ep), torch.device(DEV), ep, 2,
                                         lr_scheduler=sched, print_freq=10 ** 6)
    res = engine.evaluate(m, tr["eval"], torch.device(DEV), num_classes=2)
    print(f"trained on gfx950: last-epoch loss {loss:.4f}, dice {res['dice']:.5f} vs reference {tr['dice']:.5f}")
    assert abs(res["dice"] - tr["dice"]) <= 5e-3


def test_stf_training_from_same_seed_reaches_reference_dice():
    """STF twin (tests/golden/stf_trained.npz, make_golden_trained_stf.py): the reference's own
    train_one_epoch trained STFLSTMUNet(T=4) from the canonical init for 8 x 40 steps of seeded
    [4, 4, 1, 64, 64] DCE stacks (32^2 targets) and its evaluate() scored Dice 0.98091 on 4
    held-out batches.  The same reference run differing only in the CPU thread count (reduction
    order: 3, 1, 5 threads) scored 0.98035 / 0.98071 / 0.97945, and with its model under
    bf16 autocast (a 16-bit trajectory of the reference itself; 8 and 3 threads) 0.98042 / 0.98022:
    the reference's own run-to-run band is [0.97945, 0.98091] (1.46e-3 wide).  The gfx950 path
    (bf16 storage, stfunet AdamW, engine.train_one_epoch / evaluate) trains from the same init on
    the same batches and must land inside that band widened by 1e-3 on each side (round 3: +-5e-3)."""
    import numpy as np
    import os
    from conftest import GOLDEN
    from oracle.cases import dce_case
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet, engine
    from stfunet.optim import AdamW
    z = np.load(os.path.join(GOLDEN, "stf_trained.npz"))
    b, t, hw, epochs, steps, n_eval = (int(v) for v in z["config"])
    tgt = (hw // 2, hw // 2)
    m = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=t)
    m.load_state_dict(canonical_state_dict(m.state_dict(), seed=0))
    m = m.to(DEV)
    opt = AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4,
                eps=1e-8)
    sched = engine.create_lr_scheduler(opt, steps, epochs, warmup=True)
    for ep in range(epochs):
        batches = [dce_case(3000 + ep * steps + i, b, t, hw, hw, target_hw=tgt) for i in range(steps)]
        loss, _ = engine.train_one_epoch(m, opt, batches, torch.device(DEV), ep, 2, lr_scheduler=sched,
                                         print_freq=10 ** 6)
    ev = [dce_case(4000 + i, b, t, hw, hw, target_hw=tgt) for i in range(n_eval)]
    res = engine.evaluate(m, ev, torch.device(DEV), num_classes=2)
    ref = float(z["dice"])
    band = z["band_dice"].astype(float)
    print(f"STF trained on gfx950: last-epoch loss {loss:.4f} (reference {float(z['train_losses'][-1]):.4f}), "
          f"dice {res['dice']:.5f} vs reference {ref:.5f} (reference band {band.min():.5f}..{band.max():.5f} over "
          f"{', '.join(str(n) for n in z['band_names'])})")
    assert band.min() - 1e-3 <= res["dice"] <= band.max() + 1e-3


def _stf_fixed(z, storage):
    """STFLSTMUNet(T=4) at the canonical init with the fixture's fixed eval-mode BatchNorm state
    and head-bias shift (make_golden_trained_stf.py fixed_weight_eval), on the device, eval mode."""
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet
    b, t, hw, n = (int(v) for v in z["fixed_config"])
    m = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=t)
    sd = canonical_state_dict(m.state_dict(), seed=0)
    gen = torch.Generator().manual_seed(7)
    for k, v in sd.items():
        if "running_mean" in k:
            sd[k] = torch.rand(v.shape, generator=gen) - 0.5
        if "running_var" in k:
            sd[k] = torch.rand(v.shape, generator=gen) * 1.5 + 0.5
    sd["final.bias"][1] += torch.tensor(z["fixed_bias_shift"])
    m.load_state_dict(sd)
    m.storage_dtype = storage
    return m.to(DEV).eval(), (b, t, hw, n)


@pytest.mark.parametrize("storage", [torch.bfloat16, torch.float16])
def test_stf_fixed_weight_dice_vs_reference(storage):
    """STF Dice at FIXED weights against the reference's own evaluate() (VERDICT r03 missing #1;
    tests/golden/stf_trained.npz, fixed_*): the canonical-init model with a fixed eval-mode
    BatchNorm state and the head bias shifted so both classes are predicted, 4 held-out
    [4, 4, 1, 128, 128] batches (65,536 output pixels).

    At initialisation the logit margins are small (median |l1 - l0| ~2e-2), so Dice here counts
    pixels within storage rounding of the decision boundary: fp16 storage (the reference's --amp
    numerics) must give |dDice| <= 1e-4; bf16's 8-bit mantissa moves ~0.4 % of these pixels in the
    bf16-storage emulation itself (oracle/stf_bf16.py through the reference's evaluate(): dDice
    1.16e-4, in the fixture), so bf16 is held to 2x the emulation's |dDice| + 1e-4.  Either way every
    flipped pixel must have a reference margin < 0.1 (a flip elsewhere is a bug), and the confusion
    matrix is exactly the counts of the run's own argmax."""
    import os
    from conftest import GOLDEN
    from oracle.cases import dce_case
    from stfunet import engine
    z = np.load(os.path.join(GOLDEN, "stf_trained.npz"))
    m, (b, t, hw, n) = _stf_fixed(z, storage)
    ev = [dce_case(5000 + i, b, t, hw, hw, target_hw=(hw // 2, hw // 2)) for i in range(n)]
    res = engine.evaluate(m, ev, torch.device(DEV), num_classes=2)
    preds = []
    with torch.no_grad():
        for x5, _ in ev:
            preds.append(m(engine.preprocess_input(x5, m).to(DEV))["out"].argmax(1).cpu().numpy())
    shape = tuple(int(v) for v in z["fixed_pred_shape"])
    ref_pred = np.unpackbits(z["fixed_pred_bits"])[:int(np.prod(shape))].reshape(shape)
    flips = np.concatenate(preds) != ref_pred
    margin = z["fixed_margin"]
    worst = float(margin[flips].max()) if flips.any() else 0.0
    d = abs(res["dice"] - float(z["fixed_dice"]))
    print(f"STF fixed weights, {storage}: dice {res['dice']:.7f} ref {float(z['fixed_dice']):.7f} |d| {d:.2e}, "
          f"flipped pixels {int(flips.sum())} of {flips.size} (max ref margin {worst:.3g})")
    assert worst < 0.1
    # the confusion matrix is exactly the counts of this run's argmax (flips in both directions
    # within one target class cancel in it, so it moves by at most two counts per flip)
    tgt = np.concatenate([t.numpy() for _, t in ev]).reshape(-1)
    pred = np.concatenate(preds).reshape(-1)
    mine = np.bincount(2 * tgt + pred, minlength=4).reshape(2, 2)
    got = res["confusion_matrix"].mat.cpu().numpy()
    assert np.array_equal(got, mine), (got, mine)
    assert np.abs(got - z["fixed_confmat"]).sum() <= 2 * int(flips.sum())
    if storage == torch.float16:
        assert d <= 1e-4
    else:
        assert d <= 2 * float(z["fixed_emu_bf16_ddice"]) + 1e-4


@pytest.mark.parametrize("storage", [torch.bfloat16, torch.float16])
def test_stf_frozen_trained_dice_vs_reference(storage):
    """STF Dice at CONFIDENT trained weights against the reference's own evaluate() (VERDICT r04
    item 6; tests/golden/stf_trained_frozen.npz, make_golden_trained_stf_frozen.py): the reference
    trained STFLSTMUNet(T=4) with its ResNet-34 encoder frozen at the canonical init (regenerable from
    the seed) -- LSTMs, decoders, upconv1, final_res and final trained (6.1 M parameters, committed
    rounded to bf16, the reference evaluated on exactly those weights) -- then scored 16 held-out
    [4, 4, 1, 64, 64] batches (65,536 output pixels; median |logit margin| 9.3, 78 pixels < 0.1).
    bf16 and fp16 storage: |dDice| <= 1e-4, every flipped pixel at a reference margin < 0.1, and the
    confusion matrix exactly the counts of the run's own argmax."""
    import os
    from conftest import GOLDEN
    from oracle.cases import dce_case
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet, engine
    z = np.load(os.path.join(GOLDEN, "stf_trained_frozen.npz"))
    b, t, hw, _, _, n = (int(v) for v in z["config"])
    m = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=t)
    sd = canonical_state_dict(m.state_dict(), seed=0)
    for k, v in sd.items():
        if "bf16." + k in z.files:
            bits = z["bf16." + k].astype(np.uint32) << 16
            sd[k] = torch.from_numpy(bits.view(np.float32).reshape(v.shape).copy())
        elif "state." + k in z.files:
            sd[k] = torch.from_numpy(np.asarray(z["state." + k]).copy()).reshape(v.shape).to(v.dtype)
    assert sum(1 for k in sd if "bf16." + k in z.files) == len(z["trained_keys"])
    m.load_state_dict(sd)
    m.storage_dtype = storage
    m = m.to(DEV)
    ev = [dce_case(7000 + i, b, t, hw, hw, target_hw=(hw // 2, hw // 2)) for i in range(n)]
    res = engine.evaluate(m, ev, torch.device(DEV), num_classes=2)
    preds = []
    with torch.no_grad():
        for x5, _ in ev:
            preds.append(m(engine.preprocess_input(x5, m).to(DEV))["out"].argmax(1).cpu().numpy())
    shape = tuple(int(v) for v in z["pred_shape"])
    ref_pred = np.unpackbits(z["pred_bits"])[:int(np.prod(shape))].reshape(shape)
    flips = np.concatenate(preds) != ref_pred
    margin = z["margin"].astype(np.float32)
    worst = float(margin[flips].max()) if flips.any() else 0.0
    d = abs(res["dice"] - float(z["dice"]))
    print(f"STF frozen-encoder trained, {storage}: dice {res['dice']:.7f} ref {float(z['dice']):.7f} |d| {d:.2e}, "
          f"flipped pixels {int(flips.sum())} of {flips.size} (max ref margin {worst:.3g})")
    tgt = np.concatenate([tt.numpy() for _, tt in ev]).reshape(-1)
    pred = np.concatenate(preds).reshape(-1)
    mine = np.bincount(2 * tgt + pred, minlength=4).reshape(2, 2)
    assert np.array_equal(res["confusion_matrix"].mat.cpu().numpy(), mine)
    assert worst < 0.1
    assert d <= 1e-4
