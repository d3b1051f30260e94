"""PK-map generation: ``ToftsModelFitter`` on the gfx950 kernels (pk_fitting.py).

Same surface as the reference class (``pk_fitting.py:10-420``): ``population_aif``,
``modified_aif``, ``aif``, ``convert_signal_to_concentration``, ``preprocess_images``,
``extended_tofts_model_batch`` and ``fit_volume_gpu``.  The fit itself -- 100 epochs
of per-batch Adam over every tissue pixel, which the reference drives from Python in
batches of 1,024 (~25,600 kernel sequences per 256x256 slice) -- is ONE launch of
``stf_tofts_fit``: a thread per pixel runs the whole schedule (include/stfunet.h).
The host only builds the constant tables (time grid, AIF) with the same torch calls
as the reference, so the kernels see bit-identical inputs.

Differences: ``aif_method='auto'`` is not offered (the reference's
``get_auto_detected_aif`` references an undefined ``aif_concentration``,
pk_fitting.py:127, and cannot run); the tissue mask's 5x5 morphological open/close
(cv2.morphologyEx, absent from this image) is restated with numpy min/max filters
following OpenCV's documented border rule (erosion pads with the maximum, dilation
with the minimum) -- parity of the mask builder is unpinned; parameter PNGs are
written with PIL.  There is no CPU fallback: the fit and the model need the HIP
library on a ROCm device.
"""
import ctypes
import os

import numpy as np
import torch

from ._lib import call, stream
from .nhwc import _p

DT = 0.01
BATCH, EPOCHS, LR = 1024, 100, 0.005
BETAS, EPS = (0.9, 0.999), 1e-8
INIT = (0.05, 0.1, 0.01)                                   # pk_fitting.py:286-289
BOUNDS = (0.0, 1.0, 0.001, 0.5, 0.0, 0.2)                  # constrain_params, :303-307


def _morph(mask, k, erode):
    """Binary erosion (min filter) / dilation (max filter) with a k x k square;
    OpenCV's default border: erosion sees +inf outside, dilation -inf."""
    r = k // 2
    pad = np.pad(mask, r, mode="constant", constant_values=1 if erode else 0)
    H, W = mask.shape
    out = np.ones_like(mask) if erode else np.zeros_like(mask)
    for dy in range(k):
        for dx in range(k):
            win = pad[dy:dy + H, dx:dx + W]
            out = np.minimum(out, win) if erode else np.maximum(out, win)
    return out


class ToftsModelFitter:
    def __init__(self, time_points=None, device=None, aif_method="population"):
        self.device = device if device is not None else torch.device("cuda")
        tp = [0, 1, 2, 3, 4, 5, 6, 7] if time_points is None else time_points
        self.time_points = torch.tensor(tp, dtype=torch.float32, device=self.device)
        if aif_method not in ("population", "modified"):
            raise ValueError(f"aif_method {aif_method!r} not supported (population, modified)")
        self.aif_method = aif_method

    # ------------------------------------------------------------- AIF (:28-94)
    def population_aif(self, t, dose=0.1):
        a1, a2 = 3.99, 4.78
        m1, m2 = 0.144, 0.0111
        return dose * (a1 * torch.exp(-m1 * t) + a2 * torch.exp(-m2 * t))

    def modified_aif(self, t):
        a1, a2 = 3.99, 4.78
        m1, m2 = 0.144, 0.0111
        return a1 * torch.exp(-m1 * t) + a2 * torch.exp(-m2 * t)

    def aif(self, t):
        return self.population_aif(t) if self.aif_method == "population" else self.modified_aif(t)

    def convert_signal_to_concentration(self, signal_curves, baseline_indices=None):
        """(S - S0) / (S0 + 1e-6) with S0 the mean of the baseline frames (:131-155)."""
        idx = [0] if baseline_indices is None else baseline_indices
        base = torch.mean(signal_curves[:, idx], dim=1, keepdim=True)
        return (signal_curves - base) / (base + 1e-6)

    # ------------------------------------------------------------- preprocessing (:157-191)
    def preprocess_images(self, images):
        """images [T][H][W] -> (images / 255 on the device, tissue mask): first frame >
        0.15 * its mean, cleaned by a 5x5 open then close."""
        images = np.asarray(images)
        t = torch.tensor(images, dtype=torch.float32, device=self.device) / 255.0
        first = images[0]
        m = (first > np.mean(first) * 0.15).astype(np.uint8)
        m = _morph(_morph(m, 5, erode=True), 5, erode=False)          # MORPH_OPEN
        m = _morph(_morph(m, 5, erode=False), 5, erode=True)          # MORPH_CLOSE
        return t, torch.tensor(m.astype(bool), device=self.device)

    # ------------------------------------------------------------- tables
    def _tables(self, t):
        """The reference's constant tables (pk_fitting.py:198-203), built with the same
        torch calls (CPU, fp32) and moved to the device."""
        tc = t.detach().float().cpu()
        tau = torch.arange(0, tc[-1].item(), DT, dtype=torch.float32)
        nv = torch.tensor([int((tau < ti).sum()) for ti in tc], dtype=torch.int32)
        dev = self.device
        return (tc.to(dev), self.aif(tc).to(dev), tau.to(dev), self.aif(tau).to(dev), nv.to(dev), tau.numel())

    # ------------------------------------------------------------- model (:193-231)
    def extended_tofts_model_batch(self, t, Ktrans, ve, vp):
        tp, cpt, tau, cptau, nv, n = self._tables(t)
        kt, e, p = (v.detach().float().contiguous() for v in (Ktrans, ve, vp))
        if not kt.is_cuda:
            raise RuntimeError("stfunet.pk runs on the gfx950 HIP kernels only (no CPU fallback)")
        P, T = kt.shape[0], tp.shape[0]
        out = torch.empty(P, T, dtype=torch.float32, device=kt.device)
        call("stf_tofts_forward", _p(kt), _p(e), _p(p), P, T, _p(tp), _p(cpt), _p(tau), _p(cptau), _p(nv), n,
             DT, _p(out), stream())
        return out

    # ------------------------------------------------------------- fit (:233-420)
    def fit_curves(self, curves, batch=BATCH, epochs=EPOCHS, lr=LR):
        """Fit [P][T] tissue curves (row-major pixel order); returns params [3][P]."""
        curves = curves.detach().float().contiguous()
        if not curves.is_cuda:
            raise RuntimeError("stfunet.pk runs on the gfx950 HIP kernels only (no CPU fallback)")
        P, T = curves.shape
        tp, cpt, tau, cptau, nv, n = self._tables(self.time_points)
        assert T == tp.shape[0], "curve length != number of time points"
        nb = max(1, (P + batch - 1) // batch)
        b1, b2 = BETAS
        s = np.arange(1, epochs * nb + 1, dtype=np.float64)
        sched = np.stack([lr / (1.0 - b1 ** s), np.sqrt(1.0 - b2 ** s)], 1).astype(np.float32)
        sched = torch.from_numpy(sched).to(curves.device)
        params = torch.tensor(INIT, dtype=torch.float32, device=curves.device).view(3, 1).repeat(1, P).contiguous()
        bounds = (ctypes.c_float * 6)(*BOUNDS)               # host array (include/stfunet.h)
        call("stf_tofts_fit", _p(curves), P, T, _p(tp), _p(cpt), _p(tau), _p(cptau), _p(nv), n, DT, batch, epochs,
             _p(sched), b1, b2, EPS, bounds, _p(params), stream())
        return params

    def fit_volume_gpu(self, subtraction_images, output_dir=None, debug_output_dir=None):
        """[T][H][W] subtraction frames -> numpy param maps [3][H][W] (Ktrans, ve, vp)."""
        images, tissue = self.preprocess_images(subtraction_images)
        T, H, W = images.shape
        mask = tissue.reshape(-1)
        curves = images.permute(1, 2, 0).reshape(-1, T)[mask]
        params = self.fit_curves(curves)
        maps = torch.zeros(3, H * W, dtype=torch.float32, device=images.device)
        maps[:, mask] = params
        maps = maps.reshape(3, H, W).cpu().numpy()
        if output_dir is not None:
            self._save(maps, output_dir)
        return maps

    def _save(self, maps, output_dir):
        from PIL import Image
        os.makedirs(output_dir, exist_ok=True)
        for k, name in enumerate(("ktrans", "ve", "vp")):
            pm = maps[k]
            if np.max(pm) > 0:
                lo, hi = np.percentile(pm[pm > 0], [1, 99])
                img = ((np.clip(pm, lo, hi) - lo) / max(hi - lo, 1e-12) * 255).astype(np.uint8)
            else:
                img = np.zeros_like(pm, dtype=np.uint8)
            Image.fromarray(img).save(os.path.join(output_dir, f"{name}.png"))
            np.save(os.path.join(output_dir, f"{name}_raw.npy"), pm)
