"""PK-map kernels (stf_tofts_forward / stf_tofts_fit) vs the reference's golden
outputs and the CPU oracle (oracle/pk.py).

Tolerances: model rel L2 <= 1e-6 (fp32 exp, fp64 accumulation vs torch's fp32 sum);
fit (hundreds of Adam steps) max abs <= 2e-5 and rel L2 <= 1e-5 per parameter map."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_tofts_forward_vs_reference():
    from stfunet.pk import ToftsModelFitter
    g = np.load(os.path.join(GOLDEN, "pk_tofts.npz"))
    f = ToftsModelFitter()
    kt, ve, vp = (torch.from_numpy(g[k]).cuda() for k in ("fwd_ktrans", "fwd_ve", "fwd_vp"))
    out = f.extended_tofts_model_batch(f.time_points, kt, ve, vp)
    ref = torch.from_numpy(g["fwd_out"])
    assert rel(out, ref) < 1e-6
    assert out[:, 0].abs().max().item() == 0        # t_0 = 0: no convolution points, stays 0


def test_tofts_fit_vs_reference():
    """The whole fit_volume_gpu loop (2 batches, the second ragged, 100 epochs) on the
    reference's own inputs; the tissue mask is the one the golden run used."""
    from stfunet.pk import ToftsModelFitter
    g = np.load(os.path.join(GOLDEN, "pk_tofts.npz"))
    f = ToftsModelFitter()
    imgs = torch.from_numpy(g["images"]).cuda() / 255.0
    mask = torch.from_numpy(g["tissue"]).cuda().reshape(-1)
    T = imgs.shape[0]
    curves = imgs.permute(1, 2, 0).reshape(-1, T)[mask]
    p = f.fit_curves(curves)
    ref = torch.from_numpy(g["param_maps"]).reshape(3, -1)[:, mask.cpu()]
    for k in range(3):
        assert (p[k].cpu() - ref[k]).abs().max().item() < 2e-5
        assert rel(p[k], ref[k]) < 1e-5


def test_tofts_fit_vs_oracle_many_batches():
    """5 batches of 512 (ragged last), 12 epochs, random curves incl. clamp-hitting ones."""
    from oracle import pk as o_pk
    from stfunet.pk import ToftsModelFitter
    g = torch.Generator().manual_seed(3)
    P, T = 2300, 8
    t = torch.arange(T, dtype=torch.float32)
    curves = (torch.rand(P, 1, generator=g) * (1 - torch.exp(-torch.rand(P, 1, generator=g) * t))
              + 0.02 * torch.randn(P, T, generator=g))
    ref = o_pk.fit(curves, t, batch=512, epochs=12)
    p = ToftsModelFitter().fit_curves(curves.cuda(), batch=512, epochs=12)
    for k in range(3):
        assert (p[k].cpu() - ref[k]).abs().max().item() < 2e-5
        assert rel(p[k], ref[k]) < 1e-5
