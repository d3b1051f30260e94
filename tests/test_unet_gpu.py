"""Model-level parity of ``stfunet.UNet`` (gfx950 kernels, bf16 storage / fp32
accumulation) with the fp32 CPU oracle and the reference-generated fixtures.

Tolerances (also in DESIGN.md, "Parity"):
  logits                 relative L2 <= 3e-2 vs the fp32 oracle
  loss                   |d| <= 1e-2
  running stats          relative L2 <= 2e-2
  parameter gradients    err_hip <= 2 * err_bf16emu + 0.03, where err_* is the relative
                         L2 distance to the fp32 oracle and bf16emu is
                         oracle/unet_bf16.py (same storage precision, fp32 math).
                         The deep gradients of this net are ill-conditioned: bf16
                         storage alone moves the bottleneck's by ~40 %, so a fixed
                         small tolerance cannot be met by any bf16 implementation;
                         the band catches wrong kernels (errors of O(1)) while
                         accepting rounding.  Conv biases that feed a BatchNorm have
                         an exact gradient of 0 and are checked in absolute terms.
  after 2 AdamW steps    |p_hip - p_oracle| <= 2 * (lr_1 + lr_2) elementwise
                         (an Adam step moves each element by ~lr * sign(m))
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import loss as o_loss, optim as o_optim, unet as o_unet, unet_bf16 as o_unet_bf16
from oracle.cases import dce_case
from oracle.init import canonical_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _bn_fed_bias(k):
    return k.endswith((".0.bias", ".3.bias")) and not k.startswith(("up", "out_conv"))


def _model(base_c, seed=0, in_channels=8):
    from stfunet.unet import UNet
    m = UNet(in_channels=in_channels, num_classes=2, base_c=base_c)
    sd = canonical_state_dict(m.state_dict(), seed=seed)
    m.load_state_dict(sd)
    return m.to(DEV), sd


def _oracle(sd, x, t, fwd=o_unet.forward):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    out = fwd(p, x, training=True)["out"]
    loss = o_loss.criterion(out, t)
    loss.backward()
    return p, out.detach(), loss.item()


@pytest.mark.parametrize("base_c,size", [(8, 64), (64, 64)])
def test_unet_forward_backward_vs_oracle(base_c, size):
    from stfunet.loss import criterion
    model, sd = _model(base_c)
    x5, t = dce_case(1, 2, 8, size, size)
    x = x5.flatten(1, 2)
    p, ref_out, ref_loss = _oracle(sd, x, t)
    pe, _, _ = _oracle(sd, x, t, o_unet_bf16.forward)
    model.train()
    out = model(x.to(DEV))["out"]
    loss = criterion({"out": out}, t.to(DEV))
    loss.backward()
    assert rel(out.detach(), ref_out) < 3e-2
    assert abs(loss.item() - ref_loss) < 1e-2
    named = dict(model.named_parameters())
    bad = []
    for k, v in p.items():
        if v.grad is None:
            continue
        got = named[k].grad
        if _bn_fed_bias(k):
            scale = v.grad.abs().max().item() + p[k.replace("bias", "weight")].grad.abs().mean().item()
            if got.abs().max().item() > 0.05 * scale + 1e-5:
                bad.append((k, "bias", got.abs().max().item()))
            continue
        e_hip, e_emu = rel(got, v.grad), rel(pe[k].grad, v.grad)
        if e_hip > 2 * e_emu + 0.03:
            bad.append((k, e_hip, e_emu))
    assert not bad, bad
    msd = model.state_dict()
    for k in sd:
        if "running" in k:
            assert rel(msd[k], p[k].detach()) < 2e-2, k
        if "num_batches" in k:
            assert int(msd[k]) == 1


def test_unet_eval_mode_vs_oracle():
    model, sd = _model(8, seed=3)
    x5, _ = dce_case(2, 2, 8, 64, 64)
    x = x5.flatten(1, 2)
    with torch.no_grad():
        for k, v in model.state_dict().items():
            if "running_mean" in k:
                v.uniform_(-0.5, 0.5)
            if "running_var" in k:
                v.uniform_(0.5, 2.0)
    sd_now = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    model.eval()
    with torch.no_grad():
        out = model(x.to(DEV))["out"]
    ref = o_unet.forward(sd_now, x, training=False)["out"]
    assert rel(out, ref) < 3e-2
    # eval forward must not touch the running statistics
    for k, v in model.state_dict().items():
        assert torch.equal(v.cpu(), sd_now[k]), k


def test_unet_full_width_vs_golden():
    from stfunet.loss import criterion
    g = np.load(os.path.join(GOLDEN, "unet_full_128.npz"))
    model, _ = _model(64)
    x5, t = dce_case(3, 2, 8, 128, 128)
    model.train()
    out = model(x5.flatten(1, 2).to(DEV))["out"]
    loss = criterion({"out": out}, t.to(DEV))
    loss.backward()
    assert abs(loss.item() - float(g["loss"])) < 1e-2
    assert rel(out.detach()[:, :, ::16, ::16], g["logits_probe"]) < 3e-2
    # gradient magnitudes per parameter (sum |g|) against the reference
    for k, prm in model.named_parameters():
        ck = g["gradck." + k]
        if _bn_fed_bias(k):
            continue
        got = prm.grad.double().abs().sum().item()
        assert abs(got - ck[1]) <= 0.15 * ck[1], (k, got, ck[1])


def test_two_training_steps_vs_oracle():
    """engine.train_one_epoch + stfunet AdamW + LambdaLR vs the oracle loop."""
    from stfunet import engine
    from stfunet.optim import AdamW
    model, sd = _model(8, seed=5)
    batches = [dce_case(11, 2, 8, 64, 64), dce_case(12, 2, 8, 64, 64)]
    opt = AdamW([q for q in model.parameters() if q.requires_grad], lr=1e-3, betas=(0.9, 0.999),
                weight_decay=1e-4, eps=1e-8)
    sched = engine.create_lr_scheduler(opt, 2, 3, warmup=True)
    mean_loss, lr = engine.train_one_epoch(model, opt, batches, torch.device(DEV), 0, 2, lr_scheduler=sched,
                                           print_freq=100)
    p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    names = [k for k in p if p[k].requires_grad]
    m = [torch.zeros_like(p[k]) for k in names]
    v = [torch.zeros_like(p[k]) for k in names]
    losses, lrs = [], []
    for step, (x5, t) in enumerate(batches, start=1):
        for k in names:
            p[k].grad = None
        out = o_unet.forward(p, x5.flatten(1, 2), training=True)["out"]
        loss = o_loss.criterion(out, t)
        loss.backward()
        losses.append(loss.item())
        lrs.append(1e-3 * o_optim.lr_factor(step - 1, 2, 3))
        with torch.no_grad():
            o_optim.adamw_step([p[k] for k in names], [p[k].grad for k in names], m, v, step, lr=lrs[-1])
    assert abs(mean_loss - np.mean(losses)) < 1e-2
    assert abs(lr - 1e-3 * o_optim.lr_factor(2, 2, 3)) < 1e-12
    named = dict(model.named_parameters())
    bound = 2.2 * sum(lrs) + 1e-6
    for k in names:
        d = (named[k].detach().cpu() - p[k].detach()).abs().max().item()
        assert d <= bound, (k, d, bound)
    # and the moments were really updated through the flat kernel
    st = opt.state[named["out_conv.weight"]]
    assert int(st["step"].item()) == 2 and st["exp_avg"].abs().sum().item() > 0


def test_autocast_gradscaler_step():
    """The reference trains under torch.amp.autocast + GradScaler (train.py:240,
    train_and_eval.py:389-401): the drop-in must train identically there -- its
    forward is explicit bf16 kernels, logits stay fp32, the scaled gradient flows
    into the flat .grad views, unscale_/inf-check/step work on them."""
    from stfunet import engine
    from stfunet.optim import AdamW
    batches = [dce_case(21, 2, 8, 64, 64), dce_case(22, 2, 8, 64, 64)]
    finals = []
    for use_scaler in (False, True):
        model, _ = _model(8, seed=7)
        opt = AdamW(list(model.parameters()), lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4, eps=1e-8)
        sched = engine.create_lr_scheduler(opt, 2, 3, warmup=True)
        scaler = torch.amp.GradScaler("cuda") if use_scaler else None
        loss, _ = engine.train_one_epoch(model, opt, batches, torch.device(DEV), 0, 2, lr_scheduler=sched,
                                         print_freq=100, scaler=scaler)
        assert np.isfinite(loss)
        if scaler is not None:
            assert scaler.get_scale() == 65536.0 * 1.0          # no inf/nan step skipped
        finals.append((loss, {k: v.detach().clone() for k, v in model.named_parameters()}))
    (l0, p0), (l1, p1) = finals
    assert abs(l0 - l1) < 1e-3
    for k in p0:
        d = (p0[k] - p1[k]).abs().max().item()
        assert d <= 2.2 * 2e-3 + 1e-6, (k, d)


def test_checkpoint_resume_bitwise():
    """train.py:289-311 checkpoint dict {'model','optimizer','lr_scheduler','epoch','args'}
    through torch.save / torch.load(weights_only=True), resumed into a FRESH model,
    optimizer and scheduler (train.py:249-256): the next steps match an uninterrupted
    run bit for bit (deterministic kernels, flat optimizer state re-laid on load)."""
    import io
    from stfunet import engine
    from stfunet.optim import AdamW
    batches = [dce_case(31 + i, 2, 8, 64, 64) for i in range(4)]

    def make(seed):
        model, _ = _model(8, seed=seed)
        opt = AdamW(list(model.parameters()), lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4, eps=1e-8)
        return model, opt, engine.create_lr_scheduler(opt, 2, 3, warmup=True)

    model, opt, sched = make(9)
    engine.train_one_epoch(model, opt, batches[:2], torch.device(DEV), 0, 2, lr_scheduler=sched, print_freq=100)
    buf = io.BytesIO()
    torch.save({"model": model.state_dict(), "optimizer": opt.state_dict(), "lr_scheduler": sched.state_dict(),
                "epoch": 0, "args": {"lr": 1e-3, "epochs": 3}}, buf)
    engine.train_one_epoch(model, opt, batches[2:], torch.device(DEV), 1, 2, lr_scheduler=sched, print_freq=100)
    want = {k: v.detach().clone() for k, v in model.state_dict().items()}

    buf.seek(0)
    ck = torch.load(buf, weights_only=True, map_location=DEV)
    model2, opt2, sched2 = make(123)                   # different init: everything must come from ck
    model2.load_state_dict(ck["model"])
    opt2.load_state_dict(ck["optimizer"])
    sched2.load_state_dict(ck["lr_scheduler"])
    engine.train_one_epoch(model2, opt2, batches[2:], torch.device(DEV), ck["epoch"] + 1, 2, lr_scheduler=sched2,
                           print_freq=100)
    got = model2.state_dict()
    for k, v in want.items():
        assert torch.equal(got[k], v), k
    assert sched2.get_last_lr() == sched.get_last_lr()


def test_checkpoint_resume_bitwise_amp_scaler():
    """--amp variant of the resume contract: train_one_epoch with a GradScaler (autocast
    fp16, train_and_eval.py:389-404), checkpoint through engine.checkpoint_dict (train.py:
    304-311, which adds the 'scaler' key under --amp) and torch.save/load(weights_only=True),
    then engine.resume_from into a FRESH model, AdamW, LambdaLR and GradScaler (train.py:
    249-256): the next epoch matches the uninterrupted run bit for bit, the scaler's scale and
    growth tracker included.  A growth_interval of 2 makes the scale change inside the run."""
    import io
    from stfunet import engine
    from stfunet.optim import AdamW
    batches = [dce_case(51 + i, 2, 8, 64, 64) for i in range(6)]

    def make(seed):
        model, _ = _model(8, seed=seed)
        opt = AdamW(list(model.parameters()), lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4, eps=1e-8)
        scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 14, growth_interval=2)
        return model, opt, engine.create_lr_scheduler(opt, 3, 3, warmup=True), scaler

    model, opt, sched, scaler = make(9)
    dev = torch.device(DEV)
    engine.train_one_epoch(model, opt, batches[:3], dev, 0, 2, lr_scheduler=sched, print_freq=100, scaler=scaler)
    ck = engine.checkpoint_dict(model, opt, sched, 0, {"lr": 1e-3, "epochs": 3, "amp": True}, scaler=scaler)
    assert set(ck) == {"model", "optimizer", "lr_scheduler", "epoch", "args", "scaler"}
    buf = io.BytesIO()
    torch.save(ck, buf)
    engine.train_one_epoch(model, opt, batches[3:], dev, 1, 2, lr_scheduler=sched, print_freq=100, scaler=scaler)
    want = {k: v.detach().clone() for k, v in model.state_dict().items()}
    want_scaler = scaler.state_dict()

    buf.seek(0)
    ck = torch.load(buf, weights_only=True, map_location=DEV)
    model2, opt2, sched2, scaler2 = make(123)
    start = engine.resume_from(ck, model2, opt2, sched2, scaler2)
    assert start == 1 and scaler2.get_scale() == ck["scaler"]["scale"]
    engine.train_one_epoch(model2, opt2, batches[3:], dev, start, 2, lr_scheduler=sched2, print_freq=100,
                           scaler=scaler2)
    got = model2.state_dict()
    for k, v in want.items():
        assert torch.equal(got[k], v), k
    assert scaler2.state_dict() == want_scaler
    assert sched2.get_last_lr() == sched.get_last_lr()


def test_unet_eval_mode_backward_vs_oracle():
    """Backward through eval-mode BatchNorm (running statistics are constants: dy = gamma *
    invstd * g, conv biases get sum(dy) != 0) vs autograd of the fp32 oracle in eval mode;
    gradients within 2x the bf16-storage emulation's error + 0.02 (no batch-statistics
    amplification here).  Training-mode BN-fed conv biases: exactly 0."""
    from stfunet.loss import criterion
    model, sd = _model(8, seed=4)
    gen = torch.Generator().manual_seed(5)
    for k, v in sd.items():
        if "running_mean" in k:
            sd[k] = torch.rand(v.shape, generator=gen) - 0.5
        if "running_var" in k:
            sd[k] = torch.rand(v.shape, generator=gen) + 0.5
    model.load_state_dict(sd)
    x5, t = dce_case(6, 2, 8, 64, 64)
    x = x5.flatten(1, 2)
    p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    ref = o_unet.forward(p, x, training=False)["out"]
    o_loss.criterion(ref, t).backward()
    pe = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    o_loss.criterion(o_unet_bf16.forward(pe, x, training=False)["out"], t).backward()
    model.eval()
    out = model(x.to(DEV))["out"]
    criterion({"out": out}, t.to(DEV)).backward()
    assert rel(out.detach(), ref.detach()) < 1e-2
    bad = []
    for k, prm in model.named_parameters():
        e_hip, e_emu = rel(prm.grad, p[k].grad), rel(pe[k].grad, p[k].grad)
        if e_hip > 2 * e_emu + 0.02:
            bad.append((k, e_hip, e_emu))
    assert not bad, bad
    for k, v in model.state_dict().items():                 # eval never moves the statistics
        assert torch.equal(v.cpu(), sd[k]), k
    model.train()
    model.zero_grad()
    out = model(x.to(DEV))["out"]
    criterion({"out": out}, t.to(DEV)).backward()
    for k, prm in model.named_parameters():
        if _bn_fed_bias(k):
            assert torch.count_nonzero(prm.grad) == 0, k


@pytest.mark.parametrize("train,cin", [(True, 8), (False, 8), (True, 1), (False, 3)])
def test_unet_input_gradient_vs_oracle(train, cin):
    """d(loss)/d(input) (autograd of the input tensor, e.g. saliency maps) vs the fp32
    oracle, within 2x the bf16-storage emulation's error + 0.03; the parameter gradients
    of the same backward are unchanged by asking for it.  cin 1 / 3: the input is zero-padded
    to 8 channels, the padded channels' gradient dropped (configs[0] is a 1-channel UNet)."""
    from stfunet.loss import criterion
    model, sd = _model(8, seed=6, in_channels=cin)
    x5, t = dce_case(7, 2, 8, 64, 64)
    x = x5.flatten(1, 2)[:, :cin].contiguous()
    res = []
    for fwd in (o_unet.forward, o_unet_bf16.forward):
        p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
        xr = x.clone().requires_grad_()
        o_loss.criterion(fwd(p, xr, training=train)["out"], t).backward()
        res.append(xr.grad)
    model.train(train)
    xg = x.to(DEV).requires_grad_()
    criterion({"out": model(xg)["out"]}, t.to(DEV)).backward()
    assert xg.grad is not None and xg.grad.shape == x.shape and xg.grad.dtype == torch.float32
    e_hip, e_emu = rel(xg.grad, res[0]), rel(res[1], res[0])
    assert e_hip <= 2 * e_emu + 0.03, (e_hip, e_emu)
    g_with = {k: v.grad.clone() for k, v in model.named_parameters()}
    model.load_state_dict(sd)
    model.zero_grad()
    criterion({"out": model(x.to(DEV))["out"]}, t.to(DEV)).backward()
    for k, v in model.named_parameters():
        assert torch.equal(v.grad, g_with[k]), k
    n_packs = None          # per-call zero-padded dgrad weights stay out of the pack cache
    for _ in range(3):
        model.zero_grad()
        xg = x.to(DEV).requires_grad_()
        criterion({"out": model(xg)["out"]}, t.to(DEV)).backward()
        n = len(model.program.packs.bufs)
        assert n_packs is None or n == n_packs, (n, n_packs)
        n_packs = n


def test_gradient_accumulation_without_zero_grad():
    """Two backward passes without zero_grad accumulate (p.grad = g_a + g_b, as autograd
    does for nn.Modules), and stfunet's AdamW steps on the accumulated gradients exactly
    like torch.optim.AdamW(fused=False) on copies of them."""
    from stfunet.loss import criterion
    from stfunet.optim import AdamW
    model, sd = _model(8, seed=8)
    model.train()
    xa5, ta = dce_case(8, 2, 8, 64, 64)
    xb5, tb = dce_case(9, 2, 8, 64, 64)
    xa, xb = xa5.flatten(1, 2).to(DEV), xb5.flatten(1, 2).to(DEV)
    ta, tb = ta.to(DEV), tb.to(DEV)
    single = []
    for x, t in ((xa, ta), (xb, tb)):
        model.load_state_dict(sd)
        model.zero_grad(set_to_none=True)
        criterion({"out": model(x)["out"]}, t).backward()
        single.append({k: v.grad.clone() for k, v in model.named_parameters()})
    model.load_state_dict(sd)
    model.zero_grad(set_to_none=True)
    criterion({"out": model(xa)["out"]}, ta).backward()
    criterion({"out": model(xb)["out"]}, tb).backward()
    for k, v in model.named_parameters():
        assert torch.equal(v.grad, single[0][k] + single[1][k]), k
    ref = {k: v.detach().clone().requires_grad_() for k, v in model.named_parameters()}
    for k in ref:
        ref[k].grad = dict(model.named_parameters())[k].grad.clone()
    AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4).step()
    torch.optim.AdamW(list(ref.values()), lr=1e-3, weight_decay=1e-4, foreach=False).step()
    for k, v in model.named_parameters():
        assert torch.allclose(v.detach(), ref[k].detach(), rtol=0, atol=1e-6), k


def test_gradscaler_step_on_device_and_inf_skip():
    """Under GradScaler the optimizer takes the scaler's device scale and inf flag
    (_step_supports_amp_scaling, like the reference's AdamW(fused=True)): the update equals
    torch.optim.AdamW on the unscaled gradients, the gradients stay scaled after step(), an
    inf gradient skips the update and the step count, and the scaler backs off."""
    from stfunet.loss import criterion
    from stfunet.optim import AdamW
    model, _ = _model(8, seed=11)
    model.train()
    x5, t = dce_case(12, 2, 8, 64, 64)
    x, t = x5.flatten(1, 2).to(DEV), t.to(DEV)
    opt = AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
    scaler = torch.amp.GradScaler("cuda")
    named = dict(model.named_parameters())

    def backward():
        opt.zero_grad()
        scaler.scale(criterion({"out": model(x)["out"]}, t)).backward()

    # 1) an inf gradient: nothing moves, the step count stays 0, the scale halves
    backward()
    before = {k: v.detach().clone() for k, v in named.items()}
    named["out_conv.weight"].grad.view(-1)[0] = float("inf")
    scaler.step(opt)
    scaler.update()
    assert scaler.get_scale() == 32768.0
    for k, v in named.items():
        assert torch.equal(v.detach(), before[k]), k
    assert int(opt.state_dict()["state"][0]["step"]) == 0
    # 2) a finite step: torch.optim.AdamW on the unscaled copies, step count 1
    backward()
    scaled = {k: v.grad.clone() for k, v in named.items()}
    ref = {k: v.detach().clone().requires_grad_() for k, v in named.items()}
    for k in ref:
        ref[k].grad = scaled[k] / 32768.0
    scaler.step(opt)
    scaler.update()
    torch.optim.AdamW(list(ref.values()), lr=1e-3, weight_decay=1e-4, foreach=False).step()
    for k, v in named.items():
        assert torch.equal(v.grad, scaled[k]), k                 # still scaled, as with fused AdamW
        assert torch.allclose(v.detach(), ref[k].detach(), rtol=0, atol=1e-6), k
    assert int(opt.state_dict()["state"][0]["step"]) == 1
    # 3) unscale_ by the caller first (e.g. for gradient clipping): the scaler hands over no
    #    scale, only the inf flag; the update equals torch's on the unscaled gradients
    backward()
    scaler.unscale_(opt)
    unscaled = {k: v.grad.clone() for k, v in named.items()}
    ref = {k: v.detach().clone().requires_grad_() for k, v in named.items()}
    ref_opt = torch.optim.AdamW(list(ref.values()), lr=1e-3, weight_decay=1e-4, foreach=False)
    ref_opt.load_state_dict({"state": {i: {kk: (vv.clone() if torch.is_tensor(vv) else vv)
                                           for kk, vv in st.items()}
                                       for i, st in opt.state_dict()["state"].items()},
                             "param_groups": ref_opt.state_dict()["param_groups"]})
    for k in ref:
        ref[k].grad = unscaled[k]
    scaler.step(opt)
    scaler.update()
    ref_opt.step()
    for k, v in named.items():
        assert torch.allclose(v.detach(), ref[k].detach(), rtol=0, atol=1e-6), k
    assert int(opt.state_dict()["state"][0]["step"]) == 2
    # 4) a plain (unscaled) step afterwards continues the count on the host path
    backward()
    opt.step()
    assert int(opt.state_dict()["state"][0]["step"]) == 3
