"""Loader for the trained-weight Dice fixture (``tests/golden/unet_trained.npz``, written by
``tests/golden/make_golden_trained.py`` from the reference's own training run)."""
import os

import numpy as np
import torch

from conftest import GOLDEN
from oracle.cases import dce_case

PATH = os.path.join(GOLDEN, "unet_trained.npz")


def load():
    z = np.load(PATH)
    base_c, b, t, hw, epochs, steps, eval_batches = (int(v) for v in z["config"])
    sd = {}
    for k in z.files:
        if k.startswith("bf16."):
            bits = z[k].astype(np.uint32) << 16
            sd[k[5:]] = torch.from_numpy(bits.view(np.float32).copy())
        elif k.startswith("state."):
            sd[k[6:]] = torch.from_numpy(z[k].copy())
    pred = np.unpackbits(z["pred_bits"])[: int(np.prod(z["pred_shape"]))].reshape(tuple(z["pred_shape"]))
    return {
        "state": sd, "base_c": base_c, "B": b, "T": t, "HW": hw, "epochs": epochs, "steps": steps,
        "dice": float(z["dice"]), "confmat": z["confmat"], "pred": pred,
        "margin": z["margin"].astype(np.float32).reshape(pred.shape),
        "eval": [dce_case(2000 + i, b, t, hw, hw) for i in range(eval_batches)],
        "train_batches": lambda ep: [dce_case(1000 + ep * steps + i, b, t, hw, hw) for i in range(steps)],
    }


def shaped(sd, template):
    """Reshape the flat fixture tensors to the template state_dict's shapes."""
    return {k: sd[k].reshape(v.shape).to(v.dtype) for k, v in template.items()}
