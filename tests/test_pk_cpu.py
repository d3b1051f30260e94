"""PK-map host logic (no GPU): the tissue-mask morphology restatement and the
constant tables (pk_fitting.py:157-203)."""
import numpy as np
import torch


def test_mask_morphology_open_close():
    from stfunet.pk import _morph
    m = np.zeros((20, 20), np.uint8)
    m[4:16, 4:16] = 1
    m[0, 19] = 1                     # isolated speck: removed by the 5x5 opening
    m[9, 9] = 0                      # pinhole: filled by the 5x5 closing
    o = _morph(_morph(m, 5, True), 5, False)
    assert o[0, 19] == 0 and o[4:16, 4:16].sum() == 143
    c = _morph(_morph(o, 5, False), 5, True)
    assert c[9, 9] == 1 and c[4:16, 4:16].all() and c.sum() == 144
    # border rule: erosion treats outside as foreground, so a full image survives
    full = np.ones((8, 8), np.uint8)
    assert _morph(full, 5, True).all()


def test_tables_match_oracle():
    from oracle import pk as o_pk
    from stfunet.pk import ToftsModelFitter
    f = ToftsModelFitter(device=torch.device("cpu"))
    tp, cpt, tau, cptau, nv, n = f._tables(f.time_points)
    r_tau, r_cptau, r_cpt, r_n = o_pk.conv_grid(f.time_points)
    assert torch.equal(tau, r_tau) and torch.equal(cptau, r_cptau) and torch.equal(cpt, r_cpt)
    assert nv.tolist() == r_n.tolist() and n == tau.numel() and nv[0] == 0
