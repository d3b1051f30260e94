"""Paired training augmentation, CPU restatement (TEST INFRASTRUCTURE ONLY).

Reference: ``train.py:51-73`` ``get_transform`` composes ``transforms.py``:

* ``RandomResize(128, 307)``   transforms.py:18-32  ``size = random.randint(lo, hi)``;
  torchvision ``F.resize(img, size)`` (short side -> size, long side
  ``int(size * long / short)``, returned unchanged when already that size), image
  BILINEAR, mask NEAREST -- both PIL ``Image.resize``
* ``RandomHorizontalFlip(0.5)`` / ``RandomVerticalFlip(0.5)``  :35-54  ``random.random()
  < p`` -> PIL transpose
* ``RandomRotation(30)``       :133-157  ``random.random() < 0.5`` -> ``angle =
  random.uniform(-30, 30)``; PIL ``Image.rotate(angle, BILINEAR / NEAREST,
  expand=False)`` (fill 0)
* ``RandomCrop(224)``          :57-115  zero pad bottom/right up to 224, then
  ``h0 = randint(0, h - 224)``, ``w0 = randint(0, w - 224)``
* ``ToTensor`` + ``Normalize`` :118-130  ``u8 / 255`` (fp32), ``(x - mean) / std`` (fp32)
  with mean 0.709, std 0.127 (train.py:146-148); the mask becomes int64
* eval: ``RandomResize(224)`` + ``ToTensor`` + ``Normalize`` (no crop)

The image arithmetic lives in Pillow (12.2.0 in this image), which the reference
reaches through torchvision's PIL backend; it is restated here from Pillow's
published algorithms and pinned bit-exactly against Pillow itself
(``tests/golden/make_golden_aug.py`` -> ``tests/golden/aug_pil.npz``):

* BILINEAR resize: ``ImagingResample`` -- separable, horizontal pass first, per-output
  windows ``[int(c - s + .5), int(c + s + .5))`` with support ``s = max(scale, 1)``,
  triangle weights normalised in double and quantised to 22-bit fixed point
  (``(int)(w * 2^22 +- .5)``), accumulator seeded with 2^21, clipped to uint8
  after EACH pass
* NEAREST resize: ``ImagingScaleAffine`` -- source index tables by INCREMENTAL double
  accumulation (``x0 = scale / 2``, ``+= scale`` per output), ``(int)`` truncation
* rotate: matrix from ``angle % 360`` (cos/sin rounded to 15 digits, about the
  image centre); BILINEAR = ``ImagingGenericTransform`` (double math, sample at pixel
  centres, edge clamping, uint8 TRUNCATION); NEAREST = the 16.16 fixed-point affine
  fast path (``FIX(v) = floor(v * 65536 + .5)``, ``>> 16``)

The torchvision glue (size rule, early return, to_tensor, normalize) is restated from
torchvision's documented behaviour; torchvision is absent here, so that part is
parity unpinned (it is index bookkeeping and two fp32 operations).

Random parameters follow the reference's draw order per ``Compose`` call, from a
Python ``random.Random`` (the module the reference uses).  The reference draws a
fresh parameter set for EVERY frame (my_dataset.py:211-218: frame 0 + mask, then each
further frame, then each PK map), misaligning frames from the mask; ``paired=True``
draws one set per sample (the fix SURVEY.md section 8(f) asks for), ``paired=False``
reproduces the reference.
"""
import math

import numpy as np
import torch

PB = 22                                   # PRECISION_BITS = 32 - 8 - 2 (8-bit images)
MEAN, STD = 0.709, 0.127                  # train.py:146-148
BASE, CROP, DEGREES = 256, 224, 30        # train.py:53-62


# ------------------------------------------------------------------ torchvision glue
def resized_size(h, w, size):
    """torchvision ``_compute_resized_output_size`` for an int size (short side)."""
    short, long_ = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long_ / short)
    return (new_long, new_short) if w <= h else (new_short, new_long)        # (h2, w2)


def normalize(u8, mean=MEAN, std=STD):
    """ToTensor + Normalize: fp32 (u8 / 255 - mean) / std (transforms.py:118-130)."""
    t = torch.from_numpy(np.ascontiguousarray(u8)).to(torch.float32).div(255)
    return t.sub_(torch.tensor(mean, dtype=torch.float32)).div_(torch.tensor(std, dtype=torch.float32)).numpy()


# ------------------------------------------------------------------ Pillow: resize
def resize_coeffs(insz, outsz):
    """Per-output (xmin, n) windows and 22-bit weights [outsz][ksize] (ImagingResample)."""
    scale = insz / outsz
    fs = scale if scale > 1.0 else 1.0
    support = 1.0 * fs                    # bilinear filter support 1
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((outsz, 2), np.int32)
    kk = np.zeros((outsz, ksize), np.int32)
    ss = 1.0 / fs
    for xx in range(outsz):
        c = (xx + 0.5) * scale
        xmin = max(int(c - support + 0.5), 0)
        xmax = min(int(c + support + 0.5), insz) - xmin
        w = []
        for x in range(xmax):
            t = abs((x + xmin - c + 0.5) * ss)
            w.append(1.0 - t if t < 1.0 else 0.0)
        ww = 0.0
        for v in w:
            ww += v
        for x, v in enumerate(w):
            v = v / ww if ww != 0.0 else v
            kk[xx, x] = int(-0.5 + v * (1 << PB)) if v < 0 else int(0.5 + v * (1 << PB))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(acc):
    return np.where(acc >= (1 << PB << 8), 255, np.where(acc <= 0, 0, acc >> PB)).astype(np.uint8)


def resize_bilinear(img, h2, w2):
    h, w = img.shape
    if (h, w) == (h2, w2):
        return img.copy()
    out = img
    if w2 != w:
        b, k = resize_coeffs(w, w2)
        acc = np.full((h, w2), 1 << (PB - 1), np.int64)
        for xx, (x0, n) in enumerate(b):
            for x in range(n):
                acc[:, xx] += out[:, x0 + x].astype(np.int64) * int(k[xx, x])
        out = _clip8(acc)
    if h2 != h:
        b, k = resize_coeffs(h, h2)
        acc = np.full((h2, out.shape[1]), 1 << (PB - 1), np.int64)
        for yy, (y0, n) in enumerate(b):
            for y in range(n):
                acc[yy, :] += out[y0 + y, :].astype(np.int64) * int(k[yy, y])
        out = _clip8(acc)
    return out


def nearest_table(insz, outsz):
    """ImagingScaleAffine's pretabulated source indices (-1 = outside)."""
    scale = insz / outsz
    o, tab = scale * 0.5, np.zeros(outsz, np.int32)
    for x in range(outsz):
        xi = -1 if o < 0 else int(o)
        tab[x] = xi if 0 <= xi < insz else -1
        o += scale
    return tab


def resize_nearest(img, h2, w2):
    h, w = img.shape
    if (h, w) == (h2, w2):
        return img.copy()
    xt, yt = nearest_table(w, w2), nearest_table(h, h2)
    out = img[np.clip(yt, 0, None)][:, np.clip(xt, 0, None)].copy()
    out[yt < 0, :] = 0
    out[:, xt < 0] = 0
    return out


# ------------------------------------------------------------------ Pillow: rotate
def rotate_matrix(angle, w, h):
    """Image.rotate's inverse affine (output pixel -> input position), expand=False."""
    angle = angle % 360.0
    cx, cy = w / 2.0, h / 2.0
    r = -math.radians(angle)
    m = [round(math.cos(r), 15), round(math.sin(r), 15), 0.0, round(-math.sin(r), 15), round(math.cos(r), 15), 0.0]
    a, b, c, d, e, f = m
    m[2], m[5] = a * -cx + b * -cy + c, d * -cx + e * -cy + f
    m[2] += cx
    m[5] += cy
    return m


def rotate_is_identity(angle):
    return angle % 360.0 == 0.0


def fix16(v):
    return math.floor(v * 65536.0 + 0.5)


def rotate_bilinear(img, m):
    h, w = img.shape
    ys, xs = np.meshgrid(np.arange(h, dtype=np.float64) + 0.5, np.arange(w, dtype=np.float64) + 0.5, indexing="ij")
    xx = m[0] * xs + m[1] * ys + m[2]
    yy = m[3] * xs + m[4] * ys + m[5]
    ok = (xx >= 0.0) & (xx < w) & (yy >= 0.0) & (yy < h)
    xx, yy = xx - 0.5, yy - 0.5
    x0, y0 = np.floor(xx).astype(np.int64), np.floor(yy).astype(np.int64)
    dx, dy = xx - x0, yy - y0
    src = img.astype(np.float64)
    xa, xb = np.clip(x0, 0, w - 1), np.clip(x0 + 1, 0, w - 1)
    r0 = np.clip(y0, 0, h - 1)
    r1ok = (y0 + 1 >= 0) & (y0 + 1 < h)
    r1 = np.clip(y0 + 1, 0, h - 1)
    v1 = src[r0, xa] + (src[r0, xb] - src[r0, xa]) * dx
    v2 = np.where(r1ok, src[r1, xa] + (src[r1, xb] - src[r1, xa]) * dx, v1)
    v = v1 + (v2 - v1) * dy
    return np.where(ok, v.astype(np.int64), 0).astype(np.uint8)      # (UINT8) truncation


def rotate_nearest(img, m):
    h, w = img.shape
    a0, a1, a3, a4 = fix16(m[0]), fix16(m[1]), fix16(m[3]), fix16(m[4])
    xo, yo = fix16(m[2] + m[1] * 0.5 + m[0] * 0.5), fix16(m[5] + m[4] * 0.5 + m[3] * 0.5)
    ys, xs = np.meshgrid(np.arange(h, dtype=np.int64), np.arange(w, dtype=np.int64), indexing="ij")
    xi = (xo + ys * a1 + xs * a0) >> 16
    yi = (yo + ys * a4 + xs * a3) >> 16
    ok = (xi >= 0) & (xi < w) & (yi >= 0) & (yi < h)
    return np.where(ok, img[np.clip(yi, 0, h - 1), np.clip(xi, 0, w - 1)], 0).astype(img.dtype)


# ------------------------------------------------------------------ crop
def crop(img, size, h0, w0):
    h, w = img.shape
    if h < size or w < size:
        img = np.pad(img, ((0, max(size - h, 0)), (0, max(size - w, 0))))
    return img[h0:h0 + size, w0:w0 + size]


# ------------------------------------------------------------------ parameters
def draw_train(rng, h, w, base=BASE, crop_size=CROP, degrees=DEGREES):
    """One ``Compose`` call's random draws (train.py:58-63 order) for an h x w input."""
    size = rng.randint(int(0.5 * base), int(1.2 * base))
    h2, w2 = resized_size(h, w, size)
    hflip = rng.random() < 0.5
    vflip = rng.random() < 0.5
    angle = rng.uniform(-degrees, degrees) if rng.random() < 0.5 else None
    ph, pw = max(h2, crop_size), max(w2, crop_size)
    h0 = rng.randint(0, ph - crop_size)
    w0 = rng.randint(0, pw - crop_size)
    return dict(h2=h2, w2=w2, hflip=hflip, vflip=vflip, angle=angle, crop=crop_size, h0=h0, w0=w0)


def eval_params(h, w, crop_size=CROP):
    h2, w2 = resized_size(h, w, crop_size)
    return dict(h2=h2, w2=w2, hflip=False, vflip=False, angle=None, crop=None, h0=0, w0=0)


def _geometry(img, p, bilinear):
    out = resize_bilinear(img, p["h2"], p["w2"]) if bilinear else resize_nearest(img, p["h2"], p["w2"])
    if p["hflip"]:
        out = out[:, ::-1]
    if p["vflip"]:
        out = out[::-1, :]
    out = np.ascontiguousarray(out)
    if p["angle"] is not None and not rotate_is_identity(p["angle"]):
        m = rotate_matrix(p["angle"], out.shape[1], out.shape[0])
        out = rotate_bilinear(out, m) if bilinear else rotate_nearest(out, m)
    if p["crop"] is not None:
        out = crop(out, p["crop"], p["h0"], p["w0"])
    return out


def frame(img, p, mean=MEAN, std=STD):
    """uint8 [H][W] frame -> fp32 [h][w] network input."""
    return normalize(_geometry(img, p, True), mean, std)


def frame_u8(img, p):
    return _geometry(img, p, True)


def mask(m, p):
    """uint8 [H][W] label (0/1 after the dataset's //255) -> int64 target."""
    return _geometry(m, p, False).astype(np.int64)


def sample(frames, m, params, mean=MEAN, std=STD):
    """frames [F][H][W] uint8 with one parameter set per frame (params[0] also moves the
    mask) -> (x fp32 [F][1][h][w], target int64 [h][w])."""
    x = np.stack([frame(f, p, mean, std) for f, p in zip(frames, params)])[:, None]
    return x, mask(m, params[0])
