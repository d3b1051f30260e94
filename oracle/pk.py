"""Extended-Tofts PK-map fit, fp32 CPU restatement (test infrastructure only).

Reference: ``pk_fitting.py`` ``ToftsModelFitter``:

* ``population_aif``              :28-46   Cp(t) = dose (a1 e^{-m1 t} + a2 e^{-m2 t}),
                                           Parker constants, dose 0.1
* ``extended_tofts_model_batch``  :193-231 C(t_i) = vp Cp(t_i) + Ktrans dt sum_{tau_j < t_i}
                                           Cp(tau_j) exp(-Ktrans (t_i - tau_j) / ve),
                                           tau = arange(0, t_last, 0.01); a time point with
                                           no tau_j < t_i (t_0 = 0) stays 0
* ``fit_volume_gpu``              :233-420 tissue pixels in row-major order, batches of
                                           1,024, 100 epochs; per batch MSE(C, curve) ->
                                           Adam(lr 5e-3) over the WHOLE parameter vectors
                                           (pixels outside the batch see a zero gradient
                                           but still take the Adam step), then clamps
                                           Ktrans [0, 1], ve [0.001, 0.5], vp [0, 0.2]

Differences from the reference code, none in value: gradients are the analytic
derivatives of C (the reference differentiates with autograd), and every pixel's
Adam state is advanced in one vectorised update per step.  Adam follows
``torch.optim.Adam`` (single-tensor path): m <- lerp(m, g, 1 - b1),
v <- b2 v + (1 - b2) g^2, p <- p - (lr / (1 - b1^s)) m / (sqrt(v) / sqrt(1 - b2^s) + eps),
bias corrections in double precision as torch computes them.

Pinned by ``tests/golden/pk_tofts.npz`` (``tests/golden/make_golden_pk.py`` ran the
reference's own ``extended_tofts_model_batch`` and ``fit_volume_gpu``).
"""
import math

import torch

A1, A2, M1, M2, DOSE = 3.99, 4.78, 0.144, 0.0111, 0.1
DT = 0.01
INIT = (0.05, 0.1, 0.01)                            # Ktrans, ve, vp initial guesses (:286-289)
BOUNDS = ((0.0, 1.0), (0.001, 0.5), (0.0, 0.2))     # constrain_params (:303-307)
LR, BETAS, EPS = 0.005, (0.9, 0.999), 1e-8
BATCH, EPOCHS = 1024, 100


def population_aif(t):
    return DOSE * (A1 * torch.exp(-M1 * t) + A2 * torch.exp(-M2 * t))


def conv_grid(time_points):
    """(tau, Cp(tau), Cp(t_i), n_i = #{tau_j < t_i}) as the reference builds them."""
    t = torch.as_tensor(time_points, dtype=torch.float32)
    tau = torch.arange(0, t[-1].item(), DT, dtype=torch.float32)
    n = torch.tensor([int((tau < ti).sum()) for ti in t], dtype=torch.int64)
    return tau, population_aif(tau), population_aif(t), n


def tofts(time_points, kt, ve, vp, want_grad=False):
    """C [P][T] (and dC/d(kt, ve, vp) [3][P][T] with want_grad)."""
    t = torch.as_tensor(time_points, dtype=torch.float32)
    tau, cp_tau, cp_t, n = conv_grid(t)
    P, T = kt.shape[0], t.shape[0]
    out = torch.zeros(P, T)
    grad = torch.zeros(3, P, T) if want_grad else None
    for i in range(T):
        if n[i] == 0:
            continue
        d = t[i] - tau[: n[i]]                                  # t_i - tau_j
        e = torch.exp(-kt.view(-1, 1) * d.view(1, -1) / ve.view(-1, 1))
        ae = cp_tau[: n[i]].view(1, -1) * e
        conv = ae.sum(1) * DT
        out[:, i] = vp * cp_t[i] + kt * conv
        if want_grad:
            s1 = (ae * d.view(1, -1)).sum(1) * DT               # dt sum Cp e (t_i - tau)
            grad[0, :, i] = conv - kt * s1 / ve
            grad[1, :, i] = kt * kt * s1 / (ve * ve)
            grad[2, :, i] = cp_t[i]
    return out, grad


def fit(curves, time_points, batch=BATCH, epochs=EPOCHS, lr=LR):
    """curves [P][T] (tissue pixels in row-major order) -> params [3][P] (Ktrans, ve, vp)."""
    curves = torch.as_tensor(curves, dtype=torch.float32)
    P, T = curves.shape
    p = torch.stack([torch.full((P,), v, dtype=torch.float32) for v in INIT])
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    b1, b2 = BETAS
    nb = (P + batch - 1) // batch
    step = 0
    for _ in range(epochs):
        for b in range(nb):
            lo, hi = b * batch, min(P, (b + 1) * batch)
            pred, dc = tofts(time_points, p[0, lo:hi], p[1, lo:hi], p[2, lo:hi], want_grad=True)
            gl = (2.0 / ((hi - lo) * T)) * (pred - curves[lo:hi])          # d mse / d C
            g = torch.zeros_like(p)
            g[:, lo:hi] = (dc * gl.unsqueeze(0)).sum(2)
            step += 1
            m = m + (1 - b1) * (g - m)
            v = v * b2 + (1 - b2) * g * g
            step_size = lr / (1 - b1 ** step)
            bc2 = math.sqrt(1 - b2 ** step)
            p = p + (-step_size) * m / (v.sqrt() / bc2 + EPS)
            for k, (a, z) in enumerate(BOUNDS):
                p[k].clamp_(a, z)
    return p


def fit_volume(images, tissue, time_points=None, **kw):
    """images [T][H][W] as passed to fit_volume_gpu (0-255 scale: divided by 255 first,
    :176), tissue [H][W] bool -> param maps [3][H][W] (zero outside the tissue)."""
    imgs = torch.as_tensor(images, dtype=torch.float32) / 255.0
    T, H, W = imgs.shape
    t = torch.arange(T, dtype=torch.float32) if time_points is None else time_points
    mask = torch.as_tensor(tissue, dtype=torch.bool).reshape(-1)
    curves = imgs.permute(1, 2, 0).reshape(-1, T)[mask]
    p = fit(curves, t, **kw)
    maps = torch.zeros(3, H * W)
    maps[:, mask] = p
    return maps.reshape(3, H, W)
