"""Golden vectors for the PK-map (extended Tofts) fit, made by running the REFERENCE
``pk_fitting.py`` (build container only, CPU):

    python tests/golden/make_golden_pk.py [--ref /root/reference]

``pk_fitting.py`` imports cv2 at module level; cv2 is absent from this image.  The
path exercised here never calls it: ``ToftsModelFitter.preprocess_images`` (the only
cv2 user on the fit path: 5x5 morphological open/close of the tissue mask) is
replaced by a function returning ``images / 255`` and a GIVEN tissue mask, and
``output_dir=None`` skips the PNG writers.  So a module object named ``cv2`` with no
attributes is registered only to let the import statement succeed.

Cases (synthetic curves, seeded):
  * forward: ``extended_tofts_model_batch`` for 64 parameter triples at the default
    8 time points (pk_fitting.py:193-231)
  * fit: ``fit_volume_gpu`` (pk_fitting.py:233-420; runs on CPU here) over a 48x48
    volume with 1,371 tissue pixels = 2 batches of the reference's 1,024 (the
    second one ragged), 100 epochs of per-pixel Adam(lr 5e-3) + clamping.  Frames
    are passed on the 0-255 scale (preprocess_images divides by 255), so the curves
    the fit sees are O(0.1-1)
Output: tests/golden/pk_tofts.npz (inputs + reference outputs, no pickles).
"""
import argparse
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def load_reference(ref):
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))       # import-only stand-in (see docstring)
    spec = importlib.util.spec_from_file_location("ref_pk_fitting", os.path.join(ref, "pk_fitting.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def synthetic_volume(T, H, W, seed):
    """Subtraction frames on the 0-255 scale: smooth wash-in curves inside an
    elliptical tissue region, noise outside."""
    g = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    tissue = ((yy - H / 2) / (0.45 * H)) ** 2 + ((xx - W / 2) / (0.42 * W)) ** 2 < 1.0
    rate = 0.05 + 0.25 * g.random((H, W))
    amp = 0.2 + 0.6 * g.random((H, W))
    t = np.arange(T, dtype=np.float64)
    curves = amp[None] * (1.0 - np.exp(-rate[None] * t[:, None, None]))
    imgs = np.where(tissue[None], curves + 0.05, 0.01) + 0.01 * g.standard_normal((T, H, W))
    return (255.0 * np.clip(imgs, 0.0, 1.0)).astype(np.float32), tissue


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    torch.manual_seed(0)
    torch.set_num_threads(1)                      # one summation order
    pk = load_reference(args.ref)
    fitter = pk.ToftsModelFitter(device=torch.device("cpu"), aif_method="population")

    # forward model
    g = np.random.default_rng(5)
    kt = (0.001 + 0.5 * g.random(64)).astype(np.float32)
    ve = (0.01 + 0.45 * g.random(64)).astype(np.float32)
    vp = (0.2 * g.random(64)).astype(np.float32)
    fwd = fitter.extended_tofts_model_batch(fitter.time_points, torch.from_numpy(kt), torch.from_numpy(ve),
                                            torch.from_numpy(vp)).numpy()

    # full fit
    T, H, W = 8, 48, 48
    imgs, tissue = synthetic_volume(T, H, W, seed=11)

    def preprocess(images):
        return torch.tensor(images, dtype=torch.float32) / 255.0, torch.tensor(tissue, dtype=torch.bool)
    fitter.preprocess_images = preprocess
    maps = fitter.fit_volume_gpu(imgs, output_dir=None, debug_output_dir=None)
    out = os.path.join(HERE, "pk_tofts.npz")
    np.savez_compressed(out, fwd_ktrans=kt, fwd_ve=ve, fwd_vp=vp, fwd_out=fwd.astype(np.float32),
                        time_points=fitter.time_points.numpy(), images=imgs, tissue=tissue,
                        param_maps=maps.astype(np.float32))
    print("wrote", out, "valid pixels", int(tissue.sum()), "maps", maps.shape,
          "ktrans range", float(maps[0][tissue].min()), float(maps[0][tissue].max()))


if __name__ == "__main__":
    main()
