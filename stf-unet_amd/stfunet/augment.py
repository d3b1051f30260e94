"""Paired training augmentation on the gfx950 kernels (``stf_augment_frames`` /
``stf_augment_masks``, csrc/augment.hip).

Replaces the reference's per-sample CPU pipeline -- ``get_transform`` (train.py:51-73)
over ``transforms.py:18-157``, applied frame by frame in ``DriveDataset.__getitem__``
(my_dataset.py:200-239) inside DataLoader workers -- with two launches per batch for
every frame of every sample and one for the masks.  Results are bit-identical to the
Pillow arithmetic the reference runs (oracle/augment.py, tests/golden/aug_pil.npz).

The host keeps what Pillow keeps on the CPU: the random draws (Python ``random``, the
reference's order: RandomResize ``randint``, two flip ``random()``, rotation
``random()`` [+ ``uniform``], crop ``randint`` x 2), the resize coefficient tables
(Pillow's ``precompute_coeffs`` / ``normalize_coeffs_8bpc``, cached per size pair), the
nearest-neighbour index tables and the rotation matrix.  One descriptor per frame goes
to the device with the sources (one uint8 arena, one copy).

``paired=False`` (default) reproduces the reference's behaviour: a fresh draw per
frame (frame 0 shares the mask's draw, my_dataset.py:211-218, PK maps draw their own,
:233-237), so loss / Dice curves are comparable with the reference's.  ``paired=True``
(opt-in fix) draws ONE parameter set per sample for all its frames, PK maps and its
mask -- the alignment the reference intends but does not implement.  No CPU fallback.

Random stream: ``seed=None`` draws from the global ``random`` module at draw time (as
the reference does; torch reseeds it in every DataLoader worker).  With a seed, a
private ``random.Random`` is used; inside a DataLoader worker it is re-created from
(seed, worker id, worker seed) on first use, so workers never replay one another's
parameter stream.
"""
import ctypes
import math
import random

import numpy as np
import torch

from ._lib import call, stream

MEAN, STD = 0.709, 0.127                 # train.py:146-148
HFLIP, VFLIP, ROTATE = 1, 2, 4           # include/stfunet.h STF_AUG_*
PB = 22


class AugFrame(ctypes.Structure):
    _fields_ = [("src", ctypes.c_int64), ("rs", ctypes.c_int64), ("out", ctypes.c_int64),
                ("H", ctypes.c_int), ("W", ctypes.c_int), ("H2", ctypes.c_int), ("W2", ctypes.c_int),
                ("cx", ctypes.c_int), ("cy", ctypes.c_int), ("kx", ctypes.c_int), ("ky", ctypes.c_int),
                ("oh", ctypes.c_int), ("ow", ctypes.c_int), ("h0", ctypes.c_int), ("w0", ctypes.c_int),
                ("flags", ctypes.c_int), ("fx", ctypes.c_int * 6), ("pad_", ctypes.c_int),
                ("m", ctypes.c_double * 6)]


# ------------------------------------------------------------------ Pillow tables (host)
_COEF, _NEAR = {}, {}


def bilinear_rows(insz, outsz):
    """int32 [outsz][ks + 2] rows {xmin, n, k_0..k_{ks-1}}: Pillow's bilinear resample
    windows and 22-bit weights, vectorised over the outputs (same double operations in
    the same order as Pillow's per-output loop)."""
    key = (insz, outsz)
    if key not in _COEF:
        scale = insz / outsz
        fs = max(scale, 1.0)
        support = fs
        ks = int(math.ceil(support)) * 2 + 1
        c = (np.arange(outsz, dtype=np.float64) + 0.5) * scale
        xmin = np.maximum(np.trunc(c - support + 0.5).astype(np.int64), 0)
        xmax = np.minimum(np.trunc(c + support + 0.5).astype(np.int64), insz) - xmin
        ww = np.zeros(outsz)
        w = np.zeros((outsz, ks))
        for x in range(ks):
            t = np.abs((x + xmin - c + 0.5) * (1.0 / fs))
            w[:, x] = np.where((x < xmax) & (t < 1.0), 1.0 - t, 0.0)
            ww = ww + w[:, x]                              # left-to-right, as Pillow sums
        w = np.where(ww[:, None] != 0.0, w / np.where(ww == 0.0, 1.0, ww)[:, None], w)
        k = np.trunc(np.where(w < 0, -0.5 + w * (1 << PB), 0.5 + w * (1 << PB))).astype(np.int32)
        rows = np.zeros((outsz, ks + 2), np.int32)
        rows[:, 0], rows[:, 1], rows[:, 2:] = xmin, xmax, k
        _COEF[key] = (rows.reshape(-1), ks)
    return _COEF[key]


def nearest_index(insz, outsz):
    """Pillow ImagingScaleAffine's index table: positions accumulate scale/2 + j*scale by
    repeated double addition (cumsum is the same sequential sum), truncated; -1 outside."""
    key = (insz, outsz)
    if key not in _NEAR:
        scale = insz / outsz
        pos = np.cumsum(np.concatenate([[scale * 0.5], np.full(outsz - 1, scale)]))
        idx = np.where(pos < 0, -1, np.trunc(pos)).astype(np.int64)
        _NEAR[key] = np.where((idx >= 0) & (idx < insz), idx, -1).astype(np.int32)
    return _NEAR[key]


def rotation(angle, w, h):
    """Image.rotate(angle, expand=False): inverse affine about the centre (double) and
    its 16.16 fixed-point form {a0, a1, a3, a4, xo, yo} (Pillow's nearest fast path)."""
    angle = angle % 360.0
    cx, cy = w / 2.0, h / 2.0
    r = -math.radians(angle)
    a, b, d, e = round(math.cos(r), 15), round(math.sin(r), 15), round(-math.sin(r), 15), round(math.cos(r), 15)
    c = a * -cx + b * -cy + 0.0 + cx
    f = d * -cx + e * -cy + 0.0 + cy
    m = (a, b, c, d, e, f)

    def fix(v):
        return math.floor(v * 65536.0 + 0.5)
    fx = (fix(a), fix(b), fix(d), fix(e), fix(c + b * 0.5 + a * 0.5), fix(f + e * 0.5 + d * 0.5))
    return m, fx


def resized_size(h, w, size):
    """torchvision F.resize with an int: short side -> size, long = int(size*long/short)."""
    if w <= h:
        return int(size * h / w), size
    return size, int(size * w / h)


class DeviceAugment:
    """``get_transform(train)`` (train.py:51-73) on the device.

    Call with a batch of samples: ``frames`` = list of uint8 [F][H][W] arrays (the T
    DCE frames, then PK maps if any), ``masks`` = list of uint8 [H][W] 0/1 labels
    (the dataset's ``//255``-style binarisation already applied); returns
    (x fp32 [B][F][1][oh][ow], target int64 [B][oh][ow]) on the device."""

    def __init__(self, train=True, base_size=256, crop_size=224, mean=MEAN, std=STD, hflip_prob=0.5,
                 vflip_prob=0.5, degrees=30, paired=False, seed=None, device=None):
        self.train, self.base, self.crop = train, base_size, crop_size
        self.mean, self.std = float(mean), float(std)
        self.hflip_prob, self.vflip_prob, self.degrees = hflip_prob, vflip_prob, degrees
        self.paired = paired
        self.seed = seed
        self._rng, self._rng_owner = None, None     # owner: worker id the generator belongs to
        self.device = torch.device(device) if device is not None else torch.device("cuda")

    @property
    def rng(self):
        """The generator draws come from (see the module docstring).  Never the module
        object itself is stored, so the instance pickles for spawn / forkserver workers."""
        if self.seed is None:
            return random
        info = torch.utils.data.get_worker_info()
        owner = None if info is None else info.id
        if self._rng is None or self._rng_owner != owner:
            key = self.seed if info is None else hash((self.seed, info.id, info.seed))
            self._rng, self._rng_owner = random.Random(key), owner
        return self._rng

    # ------------------------------------------------------------- draws (train.py:58-63 order)
    def draw(self, h, w):
        if not self.train:                                  # eval: RandomResize(crop_size) only
            h2, w2 = resized_size(h, w, self.crop)
            return dict(h2=h2, w2=w2, hflip=False, vflip=False, angle=None, crop=None, h0=0, w0=0)
        r = self.rng
        size = r.randint(int(0.5 * self.base), int(1.2 * self.base))
        h2, w2 = resized_size(h, w, size)
        hflip = r.random() < self.hflip_prob
        vflip = r.random() < self.vflip_prob
        angle = r.uniform(-self.degrees, self.degrees) if r.random() < 0.5 else None
        h0 = r.randint(0, max(h2, self.crop) - self.crop)
        w0 = r.randint(0, max(w2, self.crop) - self.crop)
        return dict(h2=h2, w2=w2, hflip=hflip, vflip=vflip, angle=angle, crop=self.crop, h0=h0, w0=w0)

    def draw_sample(self, n_frames, h, w):
        """Parameter sets for one sample's frames (index 0 also moves the mask)."""
        if self.paired:
            return [self.draw(h, w)] * n_frames
        return [self.draw(h, w) for _ in range(n_frames)]

    # ------------------------------------------------------------- launch
    def __call__(self, frames, masks, params=None, launch=True):
        """plan + to_device (+ launch)."""
        st = self.to_device(self.plan(frames, masks, params))
        return self.launch(st) if launch else st

    def plan(self, frames, masks, params=None):
        """Host half (numpy only, picklable: runs in DataLoader workers via
        ``DriveDataset.collate_fn``): draws, Pillow tables, descriptors, and ONE byte
        blob = [sources | int tables | descriptors] for a single H2D copy."""
        B = len(frames)
        if B == 0:
            raise ValueError("empty batch")
        frames = [np.ascontiguousarray(np.asarray(f, dtype=np.uint8)) for f in frames]
        masks = [np.ascontiguousarray(np.asarray(m, dtype=np.uint8)) for m in masks]
        F = frames[0].shape[0]
        if any(f.ndim != 3 or f.shape[0] != F for f in frames) or len(masks) != B:
            raise ValueError("frames must be B arrays of [F][H][W] with the same F, masks B arrays [H][W]")
        if params is None:
            params = [self.draw_sample(F, f.shape[1], f.shape[2]) for f in frames]

        # sources: all frames, then all masks, in one uint8 arena
        srcs, off = [], 0
        coef_parts, coef_off, coef_len = [], {}, 0
        near_parts, near_off, near_len = [], {}, 0

        def coef(insz, outsz):
            nonlocal coef_len
            if (insz, outsz) not in coef_off:
                rows, ks = bilinear_rows(insz, outsz)
                coef_off[(insz, outsz)] = (coef_len, ks)
                coef_parts.append(rows)
                coef_len += rows.size
            return coef_off[(insz, outsz)]

        def near(insz, outsz):
            nonlocal near_len
            if (insz, outsz) not in near_off:
                t = nearest_index(insz, outsz)
                near_off[(insz, outsz)] = near_len
                near_parts.append(t)
                near_len += t.size
            return near_off[(insz, outsz)]

        fdesc = (AugFrame * (B * F))()
        mdesc = (AugFrame * B)()
        out_hw, rs_off, max_rs, max_out = None, 0, 0, 0
        for b in range(B):
            _, H, W = frames[b].shape
            if masks[b].shape != (H, W):
                raise ValueError("mask and frames differ in size")
            for f in range(F):
                p = params[b][f]
                oh, ow = (p["crop"], p["crop"]) if p["crop"] is not None else (p["h2"], p["w2"])
                if out_hw is None:
                    out_hw = (oh, ow)
                elif out_hw != (oh, ow):
                    raise ValueError(f"augmented sizes differ within the batch: {out_hw} vs {(oh, ow)}")
                d = fdesc[b * F + f]
                cxo, kx = coef(W, p["w2"])
                cyo, ky = coef(H, p["h2"])
                d.src, d.rs, d.out = off + f * H * W, rs_off, (b * F + f) * oh * ow
                d.H, d.W, d.H2, d.W2, d.cx, d.cy, d.kx, d.ky = H, W, p["h2"], p["w2"], cxo, cyo, kx, ky
                d.oh, d.ow, d.h0, d.w0 = oh, ow, p["h0"], p["w0"]
                d.flags = self._flags(p)
                if d.flags & ROTATE:
                    m, _ = rotation(p["angle"], p["w2"], p["h2"])
                    d.m[:] = m
                rs_off += p["h2"] * p["w2"]
                max_rs, max_out = max(max_rs, p["h2"] * p["w2"]), max(max_out, oh * ow)
            srcs.append(frames[b].reshape(-1))
            off += F * H * W
        for b in range(B):
            _, H, W = frames[b].shape
            p = params[b][0]
            d = mdesc[b]
            d.src, d.out = off, b * out_hw[0] * out_hw[1]
            d.H, d.W, d.H2, d.W2 = H, W, p["h2"], p["w2"]
            d.cx, d.cy = near(W, p["w2"]), near(H, p["h2"])
            d.oh, d.ow, d.h0, d.w0 = out_hw[0], out_hw[1], p["h0"], p["w0"]
            d.flags = self._flags(p)
            if d.flags & ROTATE:
                _, fx = rotation(p["angle"], p["w2"], p["h2"])
                d.fx[:] = fx
            srcs.append(masks[b].reshape(-1))
            off += H * W

        for b in range(B):                                  # mask tables follow the coefficients
            mdesc[b].cx += coef_len
            mdesc[b].cy += coef_len

        def al(n):
            return (n + 15) // 16 * 16
        ints = np.concatenate(coef_parts + near_parts).astype(np.int32).view(np.uint8)
        dbytes = np.frombuffer(bytes(fdesc) + bytes(mdesc), np.uint8)
        o_int = al(off)
        o_desc = al(o_int + ints.size)
        blob = np.zeros(o_desc + dbytes.size, np.uint8)
        blob[:off] = np.concatenate(srcs)
        blob[o_int:o_int + ints.size] = ints
        blob[o_desc:] = dbytes
        return dict(blob=blob, o_int=o_int, o_desc=o_desc, mask_desc=ctypes.sizeof(fdesc), n=B * F, B=B, F=F,
                    out_hw=out_hw, rs_bytes=rs_off, max_rs=max_rs, max_out=max_out)

    def to_device(self, plan):
        """One pinned H2D copy of the plan's blob + the output buffers (main process)."""
        dev = self.device
        blob = torch.from_numpy(plan["blob"]).pin_memory().to(dev, non_blocking=True)
        base = blob.data_ptr()
        B, F, (oh, ow) = plan["B"], plan["F"], plan["out_hw"]
        # the pinned host copy is held by torch's host allocator until the copy completes;
        # device buffers are ordered on this stream
        return dict(blob=blob, src=base, ints=base + plan["o_int"], desc=base + plan["o_desc"],
                    mask_desc=plan["mask_desc"], n=plan["n"], B=B, max_rs=plan["max_rs"], max_out=plan["max_out"],
                    scratch=torch.empty(max(plan["rs_bytes"], 1), dtype=torch.uint8, device=dev),
                    x=torch.empty(B, F, 1, oh, ow, dtype=torch.float32, device=dev),
                    target=torch.empty(B, oh, ow, dtype=torch.int64, device=dev))

    def launch(self, st):
        """The three kernels over a batch on the device (``__call__(..., launch=False)``)."""
        s = stream()
        call("stf_augment_frames", st["src"], st["desc"], st["n"], st["ints"], st["scratch"].data_ptr(),
             st["max_rs"], st["max_out"], self.mean, self.std, st["x"].data_ptr(), s)
        call("stf_augment_masks", st["src"], st["desc"] + st["mask_desc"], st["B"], st["ints"], st["max_out"],
             st["target"].data_ptr(), s)
        return st["x"], st["target"]

    @staticmethod
    def _flags(p):
        fl = (HFLIP if p["hflip"] else 0) | (VFLIP if p["vflip"] else 0)
        if p["angle"] is not None and p["angle"] % 360.0 != 0.0:
            if p["angle"] % 90.0 == 0.0:                    # Pillow transposes these instead
                raise NotImplementedError("rotation by a multiple of 90 degrees (degrees < 90 never draws one)")
            fl |= ROTATE
        return fl
