"""bf16-storage (or fp16-storage) emulation of the UNet oracle (test infrastructure).

Same functional forward as ``oracle.unet`` (src/unet.py:39-57), but every tensor
the gfx950 path stores in bf16 is rounded to bf16 at the same place, in the
forward (conv inputs/weights, conv outputs, BN+ReLU outputs) and in the
backward (their gradients), with fp32 arithmetic everywhere else.

Why it exists: the deep-layer gradients of this U-Net at initialisation are
ill-conditioned -- fp32 vs fp64 alone differs by up to ~2 % (bottleneck), and
bf16 storage moves them by ~40 %.  So "kernel correct" is tested as: the HIP
path's gradient error against the fp32 oracle stays within the band this
emulation shows against the same oracle (tests/test_unet_gpu.py).
"""
import contextlib

import torch
import torch.nn.functional as F

from . import unet as o_unet

STORE = torch.bfloat16       # the emulated 16-bit storage type (``storage(dtype)`` switches it)


@contextlib.contextmanager
def storage(dtype):
    """Emulate fp16 storage (the gfx950 path's fp16 library) instead of bf16 inside the
    block; ``oracle.stf_bf16`` rounds through the same ``q``."""
    global STORE
    prev, STORE = STORE, dtype
    try:
        yield
    finally:
        STORE = prev


class _Q(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, round_grad):
        ctx.round_grad = round_grad
        return x.to(STORE).float()

    @staticmethod
    def backward(ctx, g):
        return (g.to(STORE).float() if ctx.round_grad else g), None


def q(x, round_grad=True):
    return _Q.apply(x, round_grad)


def _double_conv(x, p, name, training):
    y = q(F.conv2d(x, q(p[f"{name}.0.weight"], False), p[f"{name}.0.bias"], padding=1))
    y = q(F.relu(o_unet.batch_norm(y, p, f"{name}.1", training)))
    y = q(F.conv2d(y, q(p[f"{name}.3.weight"], False), p[f"{name}.3.bias"], padding=1))
    return q(F.relu(o_unet.batch_norm(y, p, f"{name}.4", training)))


def forward(p, x, training=True):
    skips = []
    h = q(x)
    for i, name in enumerate(o_unet._STAGES):
        if i > 0:
            h = F.max_pool2d(h, 2)
        h = _double_conv(h, p, name, training)
        skips.append(h)
    h = skips.pop()
    for up, dec in zip(o_unet._UP, o_unet._DEC):
        h = q(F.conv_transpose2d(h, q(p[f"{up}.weight"], False), p[f"{up}.bias"], stride=2))
        h = _double_conv(torch.cat([h, skips.pop()], 1), p, dec, training)
    return {"out": F.conv2d(h, p["out_conv.weight"], p["out_conv.bias"])}
