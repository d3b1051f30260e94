"""Canonical, platform-independent weights for parity tests (test infrastructure).

Every floating-point entry of a ``state_dict`` is drawn from a counter-based
splitmix64 stream keyed by (seed, key index in state_dict order, element
index), so a full-width model (27-31 M parameters) can be re-created bit for
bit on any host without committing weights.

Distribution mirrors PyTorch's default layer init, which the reference relies
on (``src/unet.py:12``, ``src/stf_lstm_unet.py:13,105,124``):

* conv / conv-transpose / linear weights and their biases: U(-b, b),
  b = 1/sqrt(fan_in), fan_in = shape[1] * prod(shape[2:]) (PyTorch's
  ``_calculate_fan_in_and_fan_out``; for ConvTranspose2d dim 1 is out_channels);
* BatchNorm: weight 1, bias 0, running_mean 0, running_var 1, num_batches_tracked 0;
* LSTM ``weight_ih/hh_l0`` and ``bias_ih/hh_l0``: U(-1/sqrt(H), 1/sqrt(H)).
"""
import numpy as np
import torch

_M1 = np.uint64(0x9E3779B97F4A7C15)
_M2 = np.uint64(0xBF58476D1CE4E5B9)
_M3 = np.uint64(0x94D049BB133111EB)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """Vectorised splitmix64 finaliser over uint64 counters."""
    with np.errstate(over="ignore"):
        z = x + _M1
        z = (z ^ (z >> np.uint64(30))) * _M2
        z = (z ^ (z >> np.uint64(27))) * _M3
        return z ^ (z >> np.uint64(31))


def uniform_stream(seed: int, stream: int, n: int) -> np.ndarray:
    """n float64 values in [-1, 1) from counter (seed, stream, i)."""
    base = np.uint64((seed * 0x100000001B3 + stream * 0x9E3779B1) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        ctr = np.arange(n, dtype=np.uint64) + (base << np.uint64(20))
    bits = splitmix64(ctr) >> np.uint64(11)          # 53 random bits
    return bits.astype(np.float64) * (2.0 / 9007199254740992.0) - 1.0


def _fan_in(shape):
    if len(shape) < 2:
        return shape[0]
    f = shape[1]
    for s in shape[2:]:
        f *= s
    return f


def canonical_state_dict(template, seed: int = 0):
    """Fill every tensor of ``template`` (a state_dict) canonically.

    Returns an ordered dict of CPU tensors with the template's dtypes/shapes.
    """
    keys = list(template.keys())
    out = {}
    for idx, key in enumerate(keys):
        t = template[key]
        prefix, _, leaf = key.rpartition(".")
        is_bn = (prefix + ".running_mean") in template
        if leaf == "num_batches_tracked":
            out[key] = torch.zeros_like(t)
            continue
        if is_bn:
            if leaf in ("weight", "running_var"):
                out[key] = torch.ones_like(t)
            else:
                out[key] = torch.zeros_like(t)
            continue
        if "_ih_l" in leaf or "_hh_l" in leaf:  # nn.LSTM
            hidden = template[prefix + ".weight_hh_l0"].shape[1]
            bound = 1.0 / np.sqrt(hidden)
        elif leaf == "bias":
            w = template.get(prefix + ".weight")
            bound = 1.0 / np.sqrt(_fan_in(tuple(w.shape))) if w is not None else 1.0
        else:
            bound = 1.0 / np.sqrt(_fan_in(tuple(t.shape)))
        vals = uniform_stream(seed, idx, t.numel()) * bound
        out[key] = torch.from_numpy(vals.astype(np.float32)).reshape(t.shape).to(t.dtype)
    return out
