"""Tiny on-disk BreaDM-style tree for the DriveDataset tests (my_dataset.py layout)."""
import os

import numpy as np


def make_tree(root, n_patients=2, slices=3, size=(64, 80), pk=True, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    seqs = [f"VIBRANT+C{i}" for i in range(1, 9)]
    base = os.path.join(root, "seg", "training")
    for p in range(n_patients):
        pid = f"P{p:03d}"
        for s in seqs:
            d = os.path.join(base, "images", pid, s)
            os.makedirs(d, exist_ok=True)
            for k in range(slices):
                Image.fromarray(rng.integers(0, 256, size, dtype=np.uint8)).save(os.path.join(d, f"{k}.png"))
        d = os.path.join(base, "labels", pid, seqs[0])
        os.makedirs(d, exist_ok=True)
        for k in range(slices - (1 if p == 1 else 0)):              # patient 1 misses one label
            m = (rng.random(size) < 0.3).astype(np.uint8) * 255
            Image.fromarray(m).save(os.path.join(d, f"{k}.png"))
        if pk:
            d = os.path.join(base, "pk_maps", pid)
            os.makedirs(d, exist_ok=True)
            for name in ("ktrans", "ve") if p == 1 else ("ktrans", "ve", "vp"):   # patient 1: vp missing
                Image.fromarray(rng.integers(0, 256, size, dtype=np.uint8)).save(os.path.join(d, f"{name}.png"))
    # a patient without all sequences is skipped
    os.makedirs(os.path.join(base, "images", "P999", seqs[0]), exist_ok=True)
    os.makedirs(os.path.join(base, "labels", "P999"), exist_ok=True)
    return n_patients * slices - 1
