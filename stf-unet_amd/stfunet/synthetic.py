"""Seeded synthetic DCE-MRI stacks (BreaDM is not available here).

Shape contract of ``DriveDataset`` + ``collate_fn`` (my_dataset.py:15-244):
image [B, T, 1, H, W] fp32 normalised like train.py:147-148 (mean 0.709, std
0.127), mask [B, H, W] int64 in {0, 1}.  Each sample: background N(0.5, 0.3^2)
plus 1-3 discs (radius 6-40 px at 256^2, scaled with H) whose intensity rises by
0.25 per unit of normalised time (wash-in).  ``pk_channels`` appends smooth
random fields in [0, 1] on the T axis (the PK-map layout of
src/stf_lstm_unet.py:146-156).  ``mask_hw`` nearest-downsamples the mask (the
STF model predicts at H/2 x W/2).
"""
import torch


def dce_batch(batch, time_steps, height, width, seed=0, device="cuda", pk_channels=0, mask_hw=None):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    img = 0.5 + 0.3 * torch.randn(batch, time_steps, 1, height, width, generator=g, device=device)
    yy = torch.arange(height, device=device).view(1, height, 1).float()
    xx = torch.arange(width, device=device).view(1, 1, width).float()
    mask = torch.zeros(batch, height, width, dtype=torch.bool, device=device)
    scale = height / 256.0
    for _ in range(3):
        cy = torch.rand(batch, 1, 1, generator=g, device=device) * height
        cx = torch.rand(batch, 1, 1, generator=g, device=device) * width
        r = (6 + 34 * torch.rand(batch, 1, 1, generator=g, device=device)) * scale
        on = torch.rand(batch, 1, 1, generator=g, device=device) < 0.75
        disc = ((yy - cy) ** 2 + (xx - cx) ** 2 <= r * r) & on
        mask |= disc
    ramp = 0.25 * (torch.arange(1, time_steps + 1, device=device).float() / time_steps)
    img = img + mask.view(batch, 1, 1, height, width).float() * ramp.view(1, -1, 1, 1, 1)
    img = (img - 0.709) / 0.127
    if pk_channels:
        low = torch.rand(batch, pk_channels, 1, max(height // 32, 2), max(width // 32, 2), generator=g,
                         device=device)
        pk = torch.nn.functional.interpolate(low.flatten(1, 2), size=(height, width), mode="bilinear",
                                             align_corners=True).view(batch, pk_channels, 1, height, width)
        img = torch.cat([img, pk], dim=1)
    target = mask.long()
    if mask_hw is not None:
        target = target[:, :: height // mask_hw[0], :: width // mask_hw[1]].contiguous()
    return img.contiguous(), target


_SM1, _SM2, _SM3 = 0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB


def _splitmix_uniform(seed, stream, n):
    """n float64 values in [-1, 1) from the counter-based splitmix64 stream (seed, stream, i): the
    generator the parity fixtures were written with (platform-independent, bit-reproducible)."""
    import numpy as np
    m = np.uint64(0xFFFFFFFFFFFFFFFF)
    base = np.uint64((seed * 0x100000001B3 + stream * 0x9E3779B1) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        z = (np.arange(n, dtype=np.uint64) + (base << np.uint64(20))) + np.uint64(_SM1)
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(_SM2)) & m
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(_SM3)) & m
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 / 9007199254740992.0) - 1.0


def splitmix_dce_case(seed, batch, time_steps, height, width, target_hw=None):
    """Deterministic CPU DCE stack + disc mask of the fixture set (tests/golden/make_golden*.py):
    background 0.5 + U(-0.3, 0.3), two discs per image whose intensity rises by 0.25 t/T, normalised
    like train.py:147-148.  Returns (image [B, T, 1, H, W] fp32, mask [B, H, W] int64); ``target_hw``
    nearest-downsamples the mask (STF predicts at H/2)."""
    import numpy as np
    b, t, h, w = batch, time_steps, height, width
    img = _splitmix_uniform(seed, 0, b * t * h * w).reshape(b, t, 1, h, w) * 0.3 + 0.5
    geo = (_splitmix_uniform(seed, 1, b * 8).reshape(b, 8) + 1.0) / 2.0
    yy, xx = np.mgrid[0:h, 0:w]
    mask = np.zeros((b, h, w), np.int64)
    for i in range(b):
        for d in range(2):
            cy, cx, r = geo[i, 3 * d] * h, geo[i, 3 * d + 1] * w, 3 + geo[i, 3 * d + 2] * h / 5
            disc = (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r
            mask[i][disc] = 1
            for tt in range(t):
                img[i, tt, 0][disc] += 0.25 * (tt + 1) / t
    if target_hw is not None:
        mask = mask[:, :: h // target_hw[0], :: w // target_hw[1]].copy()
    return torch.from_numpy(((img - 0.709) / 0.127).astype(np.float32)), torch.from_numpy(mask)


def canonical_state_dict(template, seed=0):
    """Seeded, platform-independent weights with PyTorch's default-init distributions (the
    reference relies on them: src/unet.py:12, src/stf_lstm_unet.py:13,105,124): conv / convT /
    linear weights and biases U(-1/sqrt(fan_in), +), BatchNorm 1 / 0 / 0 / 1, LSTM U(-1/sqrt(H), +),
    every entry drawn from the splitmix64 stream (seed, key index, element index).  The weights
    the trained-Dice fixtures started from, so bench.py's Dice legs can restart that training
    without committing 27 M parameters (tests/test_surface_cpu.py pins it to the fixtures' init)."""
    import numpy as np
    keys = list(template.keys())
    out = {}
    for idx, key in enumerate(keys):
        t = template[key]
        prefix, _, leaf = key.rpartition(".")
        if leaf == "num_batches_tracked":
            out[key] = torch.zeros_like(t)
            continue
        if (prefix + ".running_mean") in template:            # BatchNorm
            out[key] = torch.ones_like(t) if leaf in ("weight", "running_var") else torch.zeros_like(t)
            continue
        if "_ih_l" in leaf or "_hh_l" in leaf:                 # nn.LSTM
            bound = 1.0 / np.sqrt(template[prefix + ".weight_hh_l0"].shape[1])
        else:
            shp = tuple((template.get(prefix + ".weight") if leaf == "bias" else t).shape)
            fan = shp[0] if len(shp) < 2 else int(np.prod(shp[1:]))
            bound = 1.0 / np.sqrt(fan)
        vals = _splitmix_uniform(seed, idx, t.numel()) * bound
        out[key] = torch.from_numpy(vals.astype(np.float32)).reshape(t.shape).to(t.dtype)
    return out
