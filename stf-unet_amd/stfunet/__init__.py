"""MI355X-native (gfx950) STF-Unet training hot path.

Drop-in replacements for the reference's ``src.UNet`` / ``src.STFLSTMUNet``
(same constructor signatures, ``input_format`` attribute, ``{"out": logits}``
output and ``state_dict`` keys) whose forward/backward run hand-written HIP
kernels through the C ABI in ``include/stfunet.h``.
"""
from . import _lib  # noqa: F401
from .stf_lstm_unet import STFLSTMUNet  # noqa: F401
from .unet import UNet  # noqa: F401

__all__ = ["STFLSTMUNet", "UNet"]
