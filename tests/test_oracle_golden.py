"""Pin the CPU oracle against fixtures produced by the reference itself.

Fixtures: ``tests/golden/*.npz`` written by ``tests/golden/make_golden.py``
(reference modules imported by path in the build container).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import loss as o_loss, metrics as o_metrics, optim as o_optim
from oracle import stf as o_stf, unet as o_unet
from oracle.cases import dce_case
from oracle.init import canonical_state_dict

torch.set_num_threads(min(8, os.cpu_count() or 1))


def _g(name):
    return np.load(os.path.join(GOLDEN, name))


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def _close(a, b, rtol, atol=1e-7):
    """||a-b|| <= rtol*||b|| + atol*sqrt(n); atol covers conv biases that feed a
    BatchNorm, whose exact gradient is 0 and whose computed value is rounding noise."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) <= rtol * np.linalg.norm(b) + atol * np.sqrt(b.size)


def _params(sd):
    return {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k)
            for k, v in sd.items()}


def _grads(p):
    return {k: v.grad for k, v in p.items() if v.grad is not None}


def test_unet_small_forward_backward():
    g = _g("unet_small.npz")
    p = _params(canonical_state_dict(o_unet.template_state_dict(8, 2, 4), seed=0))
    x = torch.from_numpy(g["x"]).flatten(1, 2)
    out = o_unet.forward(p, x, training=True)["out"]
    loss = o_loss.criterion(out, torch.from_numpy(g["target"]))
    loss.backward()
    assert _rel(out.detach(), g["logits"]) < 1e-5
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    grads = _grads(p)
    for k in g.files:
        if k.startswith("grad."):
            assert _close(grads[k[5:]], g[k], 1e-4), k
        if k.startswith("state."):
            assert _rel(p[k[6:]].detach(), g[k]) < 1e-5, k


def test_unet_small_two_train_steps():
    """Oracle AdamW + LambdaLR vs the reference ``train_one_epoch`` (2 steps)."""
    g = _g("unet_small.npz")
    sd = canonical_state_dict(o_unet.template_state_dict(8, 2, 4), seed=0)
    p = _params(sd)
    names = [k for k in p if p[k].requires_grad]
    m = [torch.zeros_like(p[k]) for k in names]
    v = [torch.zeros_like(p[k]) for k in names]
    batches = [(g["x"], g["target"]), (g["x_step2"], g["target_step2"])]
    base_lr = 1e-3
    losses = []
    for step, (x, t) in enumerate(batches, start=1):
        lr = base_lr * o_optim.lr_factor(step - 1, 2, 3)
        for k in names:
            p[k].grad = None
        out = o_unet.forward(p, torch.from_numpy(x).flatten(1, 2), training=True)["out"]
        loss = o_loss.criterion(out, torch.from_numpy(t))
        loss.backward()
        losses.append(loss.item())
        with torch.no_grad():
            o_optim.adamw_step([p[k] for k in names], [p[k].grad for k in names], m, v, step, lr=lr)
    assert abs(np.mean(losses) - float(g["epoch_mean_loss"])) < 1e-5
    assert abs(base_lr * o_optim.lr_factor(2, 2, 3) - float(g["epoch_last_lr"])) < 1e-12
    for k in names:
        if k.endswith((".0.bias", ".3.bias")) and not k.startswith("up"):
            # conv bias feeding a BatchNorm: its gradient is rounding noise, so Adam moves
            # it by up to +-lr per step in an arbitrary direction (reference included)
            assert np.abs(p[k].detach().numpy() - g["after2." + k]).max() <= 2 * base_lr, k
            continue
        assert _rel(p[k].detach(), g["after2." + k]) < 1e-4, k


def test_unet_full_width_128():
    g = _g("unet_full_128.npz")
    x, t = dce_case(3, 2, 8, 128, 128)
    p = _params(canonical_state_dict(o_unet.template_state_dict(8, 2, 64), seed=0))
    out = o_unet.forward(p, x.flatten(1, 2), training=True)["out"]
    loss = o_loss.criterion(out, t)
    loss.backward()
    assert abs(loss.item() - float(g["loss"])) < 1e-4
    assert _rel(out.detach()[:, :, ::16, ::16], g["logits_probe"]) < 1e-4
    grads = _grads(p)
    for k in g.files:
        if k.startswith("gradck."):
            ck = g[k]
            got = grads[k[7:]].double()
            # sum of |g| and sum of g^2 are stable; signed sum can cancel
            assert abs(got.abs().sum().item() - ck[1]) <= 1e-3 * abs(ck[1]) + 1e-6 * got.numel(), k


@pytest.mark.parametrize("pk", [False, True])
def test_stf_t4(pk):
    g = _g("stf_pk_t4.npz" if pk else "stf_t4.npz")
    tpl = o_stf.template_state_dict(use_pk_maps=pk)
    p = _params(canonical_state_dict(tpl, seed=0))
    out = o_stf.forward(p, torch.from_numpy(g["x"]), training=True, use_pk_maps=pk)["out"]
    loss = o_loss.criterion(out, torch.from_numpy(g["target"]))
    loss.backward()
    assert out.shape[-1] == g["x"].shape[-1] // 2          # reference H/2 output
    assert _rel(out.detach(), g["logits"]) < 1e-4
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    grads = _grads(p)
    for k in g.files:
        if k.startswith("gradck."):
            got = grads[k[7:]].double()
            ck = g[k]
            assert abs(got.abs().sum().item() - ck[1]) <= 2e-3 * abs(ck[1]) + 1e-6 * got.numel(), k
        if k.startswith("grad."):
            assert _close(grads[k[5:]], g[k], 2e-3), k
        if k.startswith("stateck."):
            got = p[k[8:]].detach().double()
            assert abs(got.sum().item() - g[k][0]) <= 1e-4 * abs(g[k][0]) + 1e-5, k


def test_criterion_known_answers():
    g = _g("criterion_kat.npz")
    loss = o_loss.criterion(torch.from_numpy(g["logits"]), torch.from_numpy(g["target"]))
    assert abs(loss.item() - float(g["loss"])) < 1e-6
    loss2 = o_loss.criterion(torch.from_numpy(g["logits_sat"]), torch.from_numpy(g["target_sat"]))
    assert abs(loss2.item() - float(g["loss_sat"])) < 1e-6


def test_metrics_known_answers():
    g = _g("metrics_kat.npz")
    logits, target = torch.from_numpy(g["logits"]), torch.from_numpy(g["target"])
    cm = o_metrics.confusion_matrix(target, logits.argmax(1), 2)
    assert np.array_equal(cm.numpy(), g["confmat"])
    d1 = o_metrics.dice_per_class(logits, target, 2, ignore_index=255)
    d2 = o_metrics.dice_per_class(torch.from_numpy(g["logits_absent"]),
                                  torch.from_numpy(g["target_absent"]), 2, ignore_index=255)
    assert np.allclose((d1 + d2) / 2, g["dice_per_class"], atol=1e-6)
    assert abs(((d1 + d2) / 2).mean() - float(g["dice_value"])) < 1e-6


def test_lr_table():
    g = _g("lr_table.npz")
    got = [o_optim.lr_factor(i, 10, 3) for i in range(30)]
    assert np.allclose(got, g["lr"], rtol=0, atol=1e-12)


def test_flop_count_matches_survey():
    # UNet 256^2 in=8 fwd 96.72 GFLOP/sample, 128^2 24.18
    assert abs(o_unet.train_flops_per_sample(8, 64, 256, 256) / 3 / 1e9 - 96.72) < 0.05
    assert abs(o_unet.train_flops_per_sample(8, 64, 128, 128) / 3 / 1e9 - 24.18) < 0.05


def test_pk_tofts_oracle_vs_reference():
    """oracle.pk (extended Tofts model + per-pixel Adam fit, pk_fitting.py:193-420)
    against the reference's own outputs (tests/golden/make_golden_pk.py): the model
    bit-exact, the 200-step fit within 1e-6 relative (analytic vs autograd gradients)."""
    from oracle import pk as o_pk
    g = np.load(os.path.join(GOLDEN, "pk_tofts.npz"))
    out, _ = o_pk.tofts(g["time_points"], torch.from_numpy(g["fwd_ktrans"]), torch.from_numpy(g["fwd_ve"]),
                        torch.from_numpy(g["fwd_vp"]))
    assert torch.equal(out, torch.from_numpy(g["fwd_out"]))
    maps = o_pk.fit_volume(g["images"], g["tissue"], torch.from_numpy(g["time_points"]))
    ref = torch.from_numpy(g["param_maps"])
    for k in range(3):
        assert ((maps[k] - ref[k]).norm() / ref[k].norm()).item() < 1e-6
        assert (maps[k] - ref[k]).abs().max().item() < 1e-6


def test_trained_unet_dice_oracle_vs_reference():
    """Trained-weight Dice (tests/golden/make_golden_trained.py: the reference trained UNet(base_c=8)
    with its own train_one_epoch, then its evaluate()): the fp32 oracle's eval-mode forward gives the
    same argmax on every pixel and the same Dice."""
    import _trained
    tr = _trained.load()
    p = _trained.shaped(tr["state"], o_unet.template_state_dict(8, 2, tr["base_c"]))
    preds, dices = [], []
    with torch.no_grad():
        for x5, t in tr["eval"]:
            out = o_unet.forward(p, x5.flatten(1, 2), training=False)["out"]
            preds.append(out.argmax(1).numpy())
            dices.append(o_metrics.dice_per_class(out, t, 2, ignore_index=255))
    assert np.array_equal(np.concatenate(preds), tr["pred"])
    assert abs(float(np.mean(dices, axis=0).mean()) - tr["dice"]) < 1e-6
    assert tr["dice"] > 0.98


def test_stf_size_fallback_matches_reference():
    """The restatement's DecoderBlock size fallback (bilinear, align_corners=True, on a size
    mismatch; src/stf_lstm_unet.py:56-57) against the reference run at 72 x 104 (make_golden.py
    gen_stf_size_fallback): train-mode logits, loss and every parameter gradient's checksum, in
    fp32 and through the bf16-storage emulation's structure (shapes)."""
    import oracle.unet_bf16 as o_q
    from oracle import stf_bf16 as o_emu
    g = _g("stf_t3_72x104.npz")
    tpl = o_stf.template_state_dict()                       # (no T in the parameter shapes)
    p = _params(canonical_state_dict(tpl, seed=0))
    x = torch.from_numpy(g["x"])
    out = o_stf.forward(p, x, training=True)["out"]
    loss = o_loss.criterion(out, torch.from_numpy(g["target"]))
    loss.backward()
    assert out.shape == g["logits"].shape == (1, 2, 36, 52)
    assert _rel(out.detach(), g["logits"]) < 1e-4
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    grads = _grads(p)
    for k in g.files:
        if k.startswith("gradck."):
            got = grads[k[7:]].double()
            assert abs(got.abs().sum().item() - g[k][1]) <= 2e-3 * abs(g[k][1]) + 1e-6 * got.numel(), k
    with torch.no_grad(), o_q.storage(torch.bfloat16):
        emu = o_emu.forward({k: v.detach() for k, v in p.items()}, x, True)["out"]
    assert emu.shape == out.shape and _rel(emu, g["logits"]) < 0.3


def test_stf_frozen_trained_oracle_argmax_vs_reference():
    """tests/golden/stf_trained_frozen.npz (make_golden_trained_stf_frozen.py: the reference trained
    STFLSTMUNet(T=4) with its ResNet-34 encoder frozen at the canonical init): the fp32 restatement at
    the committed weights (canonical encoder + bf16 trained parameters + BatchNorm running statistics)
    reproduces the reference's per-pixel argmax on all 65,536 held-out pixels -- the fixture the GPU
    Dice test (tests/test_dice_gpu.py) is held to is consistent with the oracle."""
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    z = _g("stf_trained_frozen.npz")
    b, t, hw, _, _, n = (int(v) for v in z["config"])
    sd = canonical_state_dict(o_stf.template_state_dict(), seed=0)
    for k, v in sd.items():
        if "bf16." + k in z.files:
            sd[k] = torch.from_numpy((z["bf16." + k].astype(np.uint32) << 16).view(np.float32).reshape(v.shape).copy())
        elif "state." + k in z.files:
            sd[k] = torch.from_numpy(np.asarray(z["state." + k]).copy()).reshape(v.shape).to(v.dtype)
    preds = []
    with torch.no_grad():
        for i in range(n):
            x5, _ = dce_case(7000 + i, b, t, hw, hw, target_hw=(hw // 2, hw // 2))
            preds.append(o_stf.forward(sd, x5, False)["out"].argmax(1).numpy())
    shape = tuple(int(v) for v in z["pred_shape"])
    ref = np.unpackbits(z["pred_bits"])[:int(np.prod(shape))].reshape(shape)
    assert np.array_equal(np.concatenate(preds), ref)
    assert float(z["dice"]) > 0.95
