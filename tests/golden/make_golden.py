"""Generate the golden fixtures by running the REFERENCE code (build container only).

    python tests/golden/make_golden.py  [--ref /root/reference]

Imports reference modules by file path (never executes the reference's package
``__init__`` files, which pull in torchvision/cv2 that this image lacks):

* ``src/unet.py``                                (UNet)
* ``src/stf_lstm_unet.py``                       (STFLSTMUNet) -- needs
  ``torchvision.models.resnet34``; torchvision is absent, so an in-memory
  stand-in providing a standard BasicBlock ResNet-34 with torchvision's module
  names is registered first (architecture restated, no torchvision code).
* ``train_utils/train_and_eval.py`` + ``dice_coefficient_loss.py`` under a
  synthetic ``train_utils`` parent package (``criterion``, ``train_one_epoch``,
  ``create_lr_scheduler``, ``ConfusionMatrix``, ``DiceCoefficient``).

Weights come from ``oracle.init.canonical_state_dict`` and inputs from its
splitmix64 stream, so only outputs (and small inputs) are stored.  Output files
are ``tests/golden/*.npz`` (no pickles) -- small enough to commit.
"""
import argparse
import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle.init import canonical_state_dict, uniform_stream  # noqa: E402
from oracle.cases import dce_case  # noqa: E402
from oracle import unet as o_unet, stf as o_stf  # noqa: E402


# ----------------------------------------------------------------------------- stand-in
def _install_resnet34_standin():
    """Register ``torchvision.models.resnet34`` = standard BasicBlock ResNet-34."""

    class BasicBlock(nn.Module):
        def __init__(self, inp, planes, stride):
            super().__init__()
            self.conv1 = nn.Conv2d(inp, planes, 3, stride, 1, bias=False)
            self.bn1 = nn.BatchNorm2d(planes)
            self.relu = nn.ReLU(inplace=True)
            self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
            self.bn2 = nn.BatchNorm2d(planes)
            self.downsample = None
            if stride != 1 or inp != planes:
                self.downsample = nn.Sequential(nn.Conv2d(inp, planes, 1, stride, bias=False),
                                                nn.BatchNorm2d(planes))

        def forward(self, x):
            idt = x if self.downsample is None else self.downsample(x)
            y = self.relu(self.bn1(self.conv1(x)))
            y = self.bn2(self.conv2(y))
            return self.relu(y + idt)

    class ResNet34(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
            self.bn1 = nn.BatchNorm2d(64)
            self.relu = nn.ReLU(inplace=True)
            self.maxpool = nn.MaxPool2d(3, 2, 1)
            inp = 64
            for li, (planes, n, stride) in enumerate(o_stf.RESNET34_LAYERS, start=1):
                blocks = []
                for b in range(n):
                    blocks.append(BasicBlock(inp, planes, stride if b == 0 else 1))
                    inp = planes
                setattr(self, f"layer{li}", nn.Sequential(*blocks))

    tv = types.ModuleType("torchvision")
    models = types.ModuleType("torchvision.models")
    models.resnet34 = lambda weights=None: ResNet34()
    tv.models = models
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = models


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference(ref):
    _install_resnet34_standin()
    unet = _load(os.path.join(ref, "src/unet.py"), "ref_src_unet")
    stf = _load(os.path.join(ref, "src/stf_lstm_unet.py"), "ref_src_stf")
    pkg = types.ModuleType("train_utils")
    pkg.__path__ = [os.path.join(ref, "train_utils")]
    sys.modules["train_utils"] = pkg
    dcl = _load(os.path.join(ref, "train_utils/dice_coefficient_loss.py"),
                "train_utils.dice_coefficient_loss")
    tae = _load(os.path.join(ref, "train_utils/train_and_eval.py"), "train_utils.train_and_eval")
    return unet, stf, tae, dcl


def _cksum(t):
    t = t.detach().double()
    return np.array([t.sum().item(), t.abs().sum().item(), (t * t).sum().item()])


# ----------------------------------------------------------------------------- cases
def gen_unet_small(unet_mod, tae, out):
    torch.manual_seed(0)
    model = unet_mod.UNet(in_channels=8, num_classes=2, base_c=4)
    sd = canonical_state_dict(model.state_dict(), seed=0)
    model.load_state_dict(sd)
    x5, tgt = dce_case(1, 2, 8, 64, 64)
    x = tae.preprocess_input(x5, model)
    model.train()
    outd = model(x)
    loss = tae.criterion(outd, tgt)
    loss.backward()
    res = {"x": x5.numpy(), "target": tgt.numpy(), "logits": outd["out"].detach().numpy(),
           "loss": np.array(loss.item())}
    for k, v in model.state_dict().items():
        if "running" in k or "num_batches" in k:
            res["state." + k] = v.numpy().copy()
    for k, p in model.named_parameters():
        res["grad." + k] = p.grad.numpy().copy()
    # two steps of the reference train_one_epoch (AdamW fused, LambdaLR)
    model.load_state_dict(sd)
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-3,
                            betas=(0.9, 0.999), weight_decay=1e-4, eps=1e-8, fused=True)
    sched = tae.create_lr_scheduler(opt, 2, 3, warmup=True)
    x5b, tgtb = dce_case(2, 2, 8, 64, 64)
    loader = [(x5, tgt), (x5b, tgtb)]
    mean_loss, lr = tae.train_one_epoch(model, opt, loader, torch.device("cpu"), 0, 2,
                                        lr_scheduler=sched, print_freq=100)
    res["x_step2"] = x5b.numpy()
    res["target_step2"] = tgtb.numpy()
    res["epoch_mean_loss"] = np.array(mean_loss)
    res["epoch_last_lr"] = np.array(lr)
    for k, v in model.state_dict().items():
        res["after2." + k] = v.numpy()
    np.savez_compressed(os.path.join(out, "unet_small.npz"), **res)
    return {"unet_small_loss": loss.item(), "epoch_mean_loss": mean_loss}


def gen_unet_full(unet_mod, tae, out):
    model = unet_mod.UNet(in_channels=8, num_classes=2, base_c=64)
    model.load_state_dict(canonical_state_dict(model.state_dict(), seed=0))
    x5, tgt = dce_case(3, 2, 8, 128, 128)
    model.train()
    outd = model(tae.preprocess_input(x5, model))
    loss = tae.criterion(outd, tgt)
    loss.backward()
    res = {"logits_cksum": _cksum(outd["out"]), "loss": np.array(loss.item()),
           "logits_probe": outd["out"].detach()[:, :, ::16, ::16].numpy()}
    for k, p in model.named_parameters():
        res["gradck." + k] = _cksum(p.grad)
    np.savez_compressed(os.path.join(out, "unet_full_128.npz"), **res)
    return {"unet_full_loss": loss.item()}


def gen_stf(stf_mod, tae, out, pk):
    kw = dict(in_channels=1, num_classes=2, time_steps=4, use_pk_maps=pk)
    model = stf_mod.STFLSTMUNet(**kw)
    sd = canonical_state_dict(model.state_dict(), seed=0)
    model.load_state_dict(sd)
    b = 1 if pk else 2
    x, tgt = dce_case(4 if pk else 5, b, 4 + (3 if pk else 0), 64, 64, target_hw=(32, 32))
    if pk:  # PK slots are smooth fields in [0, 1]
        x[:, 4:] = torch.from_numpy(((uniform_stream(6, 0, b * 3 * 64 * 64) + 1) / 2)
                                    .astype(np.float32).reshape(b, 3, 1, 64, 64))
    model.train()
    outd = model(x)
    loss = tae.criterion(outd, tgt)
    loss.backward()
    res = {"x": x.numpy(), "target": tgt.numpy(), "logits": outd["out"].detach().numpy(),
           "loss": np.array(loss.item())}
    for k, v in model.state_dict().items():
        if "running" in k or "num_batches" in k:
            res["stateck." + k] = _cksum(v.float())
    for k, p in model.named_parameters():
        res["gradck." + k] = _cksum(p.grad)
        if p.numel() <= 4096:
            res["grad." + k] = p.grad.numpy().copy()
    name = "stf_pk_t4.npz" if pk else "stf_t4.npz"
    np.savez_compressed(os.path.join(out, name), **res)
    return {name: loss.item()}


def gen_criterion(tae, dcl, out):
    g = torch.Generator().manual_seed(7)
    logits = torch.randn(3, 2, 8, 8, generator=g) * 2
    target = (torch.rand(3, 8, 8, generator=g) > 0.6).long()
    loss = tae.criterion({"out": logits}, target)
    # empty-set branch (dice_coefficient_loss.py:34-35): saturated softmax, no fg
    logits2 = torch.zeros(2, 2, 4, 4)
    logits2[:, 0] = 200.0
    logits2[:, 1] = -200.0
    target2 = torch.zeros(2, 4, 4, dtype=torch.long)
    loss2 = tae.criterion({"out": logits2}, target2)
    dt = dcl.build_target(target, 2, -100)
    coeff = dcl.multiclass_dice_coeff(torch.softmax(logits, 1), dt)
    np.savez_compressed(os.path.join(out, "criterion_kat.npz"), logits=logits.numpy(),
                        target=target.numpy(), loss=np.array(loss.item()),
                        logits_sat=logits2.numpy(), target_sat=target2.numpy(),
                        loss_sat=np.array(loss2.item()), dice_coeff=np.array(float(coeff)))


def gen_metrics(tae, out):
    g = torch.Generator().manual_seed(11)
    logits = torch.randn(2, 2, 16, 16, generator=g)
    target = (torch.rand(2, 16, 16, generator=g) > 0.5).long()
    target[0, :2, :] = 255                              # ignore band
    cm = tae.ConfusionMatrix(2)
    cm.update(target.flatten(), logits.argmax(1).flatten())
    dc = tae.DiceCoefficient(num_classes=2, ignore_index=255)
    dc.update(logits, target)
    # absent class -> Dice 1.0 branch (train_and_eval.py:104-107)
    t2 = torch.zeros(1, 4, 4, dtype=torch.long)
    l2 = torch.zeros(1, 2, 4, 4)
    l2[:, 0] = 1.0
    dc.update(l2, t2)
    np.savez_compressed(os.path.join(out, "metrics_kat.npz"), logits=logits.numpy(),
                        target=target.numpy(), confmat=cm.mat.numpy(),
                        dice_per_class=dc.compute().numpy(), dice_value=np.array(dc.value.item()),
                        logits_absent=l2.numpy(), target_absent=t2.numpy())


def gen_lr(tae, out):
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    sched = tae.create_lr_scheduler(opt, 10, 3, warmup=True)
    lrs = []
    for _ in range(30):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sched.step()
    np.savez_compressed(os.path.join(out, "lr_table.npz"), lr=np.array(lrs), num_step=10, epochs=3)


def gen_keys(unet_mod, stf_mod, out):
    """state_dict key order and shapes of the reference modules (the drop-in contract,
    SURVEY.md 8(b)): UNet (in 8 / 11) and STFLSTMUNet with and without PK maps."""
    mods = {"unet_in8": unet_mod.UNet(in_channels=8, num_classes=2, base_c=64),
            "unet_in11": unet_mod.UNet(in_channels=11, num_classes=2, base_c=64),
            "stf_t8": stf_mod.STFLSTMUNet(in_channels=1, num_classes=2, time_steps=8),
            "stf_t8_pk": stf_mod.STFLSTMUNet(in_channels=1, num_classes=2, time_steps=8, use_pk_maps=True)}
    res = {k: [[n, list(v.shape)] for n, v in m.state_dict().items()] for k, m in mods.items()}
    res["param_counts"] = {k: sum(p.numel() for p in m.parameters()) for k, m in mods.items()}
    res["stf_input_format"] = getattr(mods["stf_t8"], "input_format", None)
    with open(os.path.join(out, "state_dict_keys.json"), "w") as f:
        json.dump(res, f)


def gen_stf_size_fallback(stf_mod, tae, out):
    """STFLSTMUNet(T=3) at 72 x 104 (not divisible by 32): the reference's DecoderBlock resizes the
    transposed-conv outputs of decoder4 / decoder3 to the skips by bilinear interpolation
    (src/stf_lstm_unet.py:56-57).  Train-mode logits, loss and gradient checksums."""
    model = stf_mod.STFLSTMUNet(in_channels=1, num_classes=2, time_steps=3)
    model.load_state_dict(canonical_state_dict(model.state_dict(), seed=0))
    x, tgt = dce_case(7, 1, 3, 72, 104, target_hw=(36, 52))
    model.train()
    outd = model(x)
    loss = tae.criterion(outd, tgt)
    loss.backward()
    res = {"x": x.numpy(), "target": tgt.numpy(), "logits": outd["out"].detach().numpy(),
           "loss": np.array(loss.item())}
    for k, p in model.named_parameters():
        res["gradck." + k] = _cksum(p.grad)
    np.savez_compressed(os.path.join(out, "stf_t3_72x104.npz"), **res)
    return {"stf_t3_72x104.npz": loss.item()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", default=None, choices=["keys", "fallback"], help="regenerate one fixture only")
    a = ap.parse_args()
    torch.set_num_threads(8)
    unet_mod, stf_mod, tae, dcl = load_reference(a.ref)
    if a.only == "fallback":
        print(gen_stf_size_fallback(stf_mod, tae, a.out))
        return
    gen_keys(unet_mod, stf_mod, a.out)
    if a.only == "keys":
        return
    summary = {}
    summary.update(gen_unet_small(unet_mod, tae, a.out))
    summary.update(gen_unet_full(unet_mod, tae, a.out))
    summary.update(gen_stf(stf_mod, tae, a.out, pk=False))
    summary.update(gen_stf(stf_mod, tae, a.out, pk=True))
    summary.update(gen_stf_size_fallback(stf_mod, tae, a.out))
    gen_criterion(tae, dcl, a.out)
    gen_metrics(tae, a.out)
    gen_lr(tae, a.out)
    with open(os.path.join(a.out, "SUMMARY.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
