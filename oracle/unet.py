"""Functional fp32 CPU restatement of the reference 2-D U-Net (test infrastructure).

Follows ``src/unet.py`` of the reference:

* ``conv_block`` (= DoubleConv)  ``src/unet.py:10-18``
  Conv3x3(p=1, bias) -> BN -> ReLU -> Conv3x3(p=1, bias) -> BN -> ReLU
* encoder ``enc1..enc4`` + ``pool`` (MaxPool2d(2), = Down)  ``src/unet.py:20-25,40-45``
* ``bottleneck``  ``src/unet.py:26``
* ``up4..up1`` ConvTranspose2d(k=2, s=2) + ``cat([up, skip], 1)`` + ``dec*`` (= Up)
  ``src/unet.py:28-35,47-54``
* ``out_conv`` 1x1 (= OutConv)  ``src/unet.py:37,56``; returns ``{"out": logits}`` (:57)

Parameters are a flat dict keyed exactly like the reference ``state_dict``
(``enc1.0.weight``, ``enc1.1.running_mean``, ``up4.weight`` ...).
BatchNorm in training mode normalises with the biased batch variance and
updates running stats with the unbiased one (momentum 0.1, eps 1e-5) -- torch
defaults the reference inherits.
"""
from collections import OrderedDict

import torch
import torch.nn.functional as F

BN_EPS = 1e-5
BN_MOMENTUM = 0.1

_STAGES = ("enc1", "enc2", "enc3", "enc4", "bottleneck")
_DEC = ("dec4", "dec3", "dec2", "dec1")
_UP = ("up4", "up3", "up2", "up1")


def _double_conv_shapes(name, cin, cout, out):
    for conv_idx, bn_idx, ci in ((0, 1, cin), (3, 4, cout)):
        out[f"{name}.{conv_idx}.weight"] = (cout, ci, 3, 3)
        out[f"{name}.{conv_idx}.bias"] = (cout,)
        for leaf in ("weight", "bias", "running_mean", "running_var"):
            out[f"{name}.{bn_idx}.{leaf}"] = (cout,)
        out[f"{name}.{bn_idx}.num_batches_tracked"] = ()


def param_shapes(in_channels=8, num_classes=2, base_c=64):
    """(key -> shape) in the reference's state_dict registration order."""
    s = OrderedDict()
    widths = [base_c, base_c * 2, base_c * 4, base_c * 8, base_c * 16]
    cin = in_channels
    for name, w in zip(_STAGES, widths):
        _double_conv_shapes(name, cin, w, s)
        cin = w
    for level, (up, dec) in enumerate(zip(_UP, _DEC)):
        hi = widths[4 - level]
        lo = widths[3 - level]
        s[f"{up}.weight"] = (hi, lo, 2, 2)
        s[f"{up}.bias"] = (lo,)
        _double_conv_shapes(dec, hi, lo, s)
    s["out_conv.weight"] = (num_classes, base_c, 1, 1)
    s["out_conv.bias"] = (num_classes,)
    return s


def template_state_dict(in_channels=8, num_classes=2, base_c=64):
    return OrderedDict(
        (k, torch.zeros(v, dtype=torch.int64) if k.endswith("num_batches_tracked")
         else torch.zeros(v, dtype=torch.float32))
        for k, v in param_shapes(in_channels, num_classes, base_c).items())


def batch_norm(x, p, prefix, training):
    """BatchNorm2d; in training mode also advances running stats in ``p``."""
    return F.batch_norm(x, p[prefix + ".running_mean"], p[prefix + ".running_var"],
                        p[prefix + ".weight"], p[prefix + ".bias"],
                        training=training, momentum=BN_MOMENTUM, eps=BN_EPS)


def double_conv(x, p, name, training):
    y = F.conv2d(x, p[f"{name}.0.weight"], p[f"{name}.0.bias"], padding=1)
    y = F.relu(batch_norm(y, p, f"{name}.1", training))
    y = F.conv2d(y, p[f"{name}.3.weight"], p[f"{name}.3.bias"], padding=1)
    return F.relu(batch_norm(y, p, f"{name}.4", training))


def forward(p, x, training=True):
    """x: [B, Cin, H, W] fp32 (already ``preprocess_input``-flattened).

    Running statistics in ``p`` are updated in place when ``training``
    (the caller passes clones if it wants to keep the originals).
    """
    skips = []
    h = x
    for i, name in enumerate(_STAGES):
        if i > 0:
            h = F.max_pool2d(h, 2)
        h = double_conv(h, p, name, training)
        skips.append(h)
    h = skips.pop()                      # bottleneck output
    for up, dec in zip(_UP, _DEC):
        h = F.conv_transpose2d(h, p[f"{up}.weight"], p[f"{up}.bias"], stride=2)
        h = double_conv(torch.cat([h, skips.pop()], dim=1), p, dec, training)
    logits = F.conv2d(h, p["out_conv.weight"], p["out_conv.bias"])
    if training:
        for k in p:
            if k.endswith("num_batches_tracked"):
                p[k] += 1
    return {"out": logits}


def train_flops_per_sample(in_channels=8, base_c=64, H=256, W=256):
    """Algorithmic fwd FLOPs (2*MAC) of conv/convT/1x1 layers, x3 for training."""
    widths = [base_c, base_c * 2, base_c * 4, base_c * 8, base_c * 16]
    f = 0.0
    cin = in_channels
    h, w = H, W
    res = []
    for i, c in enumerate(widths):
        if i > 0:
            h, w = h // 2, w // 2
        f += 2 * h * w * c * 9 * (cin + c)
        res.append((h, w))
        cin = c
    for level in range(4):
        hi, lo = widths[4 - level], widths[3 - level]
        hh, ww = res[3 - level]
        f += 2 * (hh // 2) * (ww // 2) * hi * lo * 4      # convT 2x2
        f += 2 * hh * ww * lo * 9 * (hi + lo)               # DoubleConv
    f += 2 * H * W * base_c * 2
    return 3.0 * f
