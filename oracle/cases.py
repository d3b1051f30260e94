"""Deterministic synthetic DCE cases shared by the golden generator and the tests.

Test infrastructure (see ``oracle/__init__.py``).
"""
import numpy as np
import torch

from .init import uniform_stream


def dce_case(seed, b, t, h, w, target_hw=None):
    """Deterministic DCE-like stack + disc masks from the splitmix64 stream.

    Background ~U(-1,1)*0.3; 1-2 discs per image whose intensity rises with t;
    normalised like train.py:147-148 (mean 0.709, std 0.127).
    """
    noise = uniform_stream(seed, 0, b * t * h * w).reshape(b, t, 1, h, w) * 0.3
    geo = (uniform_stream(seed, 1, b * 8).reshape(b, 8) + 1.0) / 2.0
    yy, xx = np.mgrid[0:h, 0:w]
    mask = np.zeros((b, h, w), np.int64)
    img = noise + 0.5
    for i in range(b):
        for d in range(2):
            cy, cx, r = geo[i, 3 * d] * h, geo[i, 3 * d + 1] * w, 3 + geo[i, 3 * d + 2] * h / 5
            disc = (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r
            mask[i][disc] = 1
            for tt in range(t):
                img[i, tt, 0][disc] += 0.25 * (tt + 1) / t
    img = ((img - 0.709) / 0.127).astype(np.float32)
    if target_hw is not None:
        sy, sx = h // target_hw[0], w // target_hw[1]
        mask = mask[:, ::sy, ::sx].copy()
    return torch.from_numpy(img), torch.from_numpy(mask)
