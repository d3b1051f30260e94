"""bf16-storage emulation of the STF-LSTM-UNet oracle (test infrastructure).

Same functional graph as ``oracle.stf`` (src/stf_lstm_unet.py:139-256), rounding
to bf16 every tensor the gfx950 path stores in bf16 (conv inputs/weights/outputs,
BN(+residual)(+ReLU) outputs, LSTM inputs and hidden states; forward values and
their gradients), keeping fp32 for BN statistics, LSTM cell state and gates.
Used as the precision band for the model-level gradient parity test (see
``oracle.unet_bf16`` for the rationale).
"""
import torch
import torch.nn.functional as F

from .stf import RESNET34_LAYERS
from .unet import batch_norm
from .unet_bf16 import q


def _conv(x, w, b=None, **kw):
    return q(F.conv2d(x, q(w, False), b, **kw))


def _rcb(x, p, pre, tr):
    y = _conv(x, p[f"{pre}.conv_block.0.weight"], padding=1)
    y = q(F.relu(batch_norm(y, p, f"{pre}.conv_block.1", tr)))
    y = _conv(y, p[f"{pre}.conv_block.3.weight"], padding=1)
    return q(F.relu(batch_norm(y, p, f"{pre}.conv_block.4", tr) + x))


def _block(x, p, pre, stride, tr):
    y = _conv(x, p[f"{pre}.conv1.weight"], stride=stride, padding=1)
    y = q(F.relu(batch_norm(y, p, f"{pre}.bn1", tr)))
    y = _conv(y, p[f"{pre}.conv2.weight"], padding=1)
    y = batch_norm(y, p, f"{pre}.bn2", tr)
    if f"{pre}.downsample.0.weight" in p:
        sc = batch_norm(_conv(x, p[f"{pre}.downsample.0.weight"], stride=stride), p, f"{pre}.downsample.1", tr)
    else:
        sc = x
    return q(F.relu(y + sc))


def _lstm(seq, p, pre):
    w_ih, w_hh = q(p[f"{pre}.weight_ih_l0"], False), q(p[f"{pre}.weight_hh_l0"], False)
    bias = p[f"{pre}.bias_ih_l0"] + p[f"{pre}.bias_hh_l0"]
    n, t_len, _ = seq.shape
    h = seq.new_zeros(n, w_hh.shape[1])
    c = seq.new_zeros(n, w_hh.shape[1])
    for t in range(t_len):
        i, f, g, o = (seq[:, t] @ w_ih.t() + h @ w_hh.t() + bias).chunk(4, dim=1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
        h = q(torch.sigmoid(o) * torch.tanh(c))
    return h


def forward(p, x, training=True, use_pk_maps=False, pk_channels=3):
    b, total, ch, hgt, wid = x.shape
    pk = None
    steps = total
    if use_pk_maps:
        steps = total - pk_channels
        pk = q(x[:, steps:].reshape(b, pk_channels, ch, hgt, wid).squeeze(2))
        x = x[:, :steps]
    x = q(x)
    seqs = [[], [], [], []]
    for t in range(steps):
        xt = x[:, t] if pk is None else torch.cat([x[:, t], pk], 1)
        h = _conv(xt, p["conv1.weight"], stride=2, padding=3)
        h = q(F.relu(batch_norm(h, p, "bn1", training)))
        h = F.max_pool2d(h, 3, 2, 1)
        feats = []
        for li, (_, blocks, stride) in enumerate(RESNET34_LAYERS, start=1):
            for bi in range(blocks):
                h = _block(h, p, f"layer{li}.{bi}", stride if bi == 0 else 1, training)
            feats.append(h)
        if pk is not None:
            feats = [_conv(torch.cat([e, q(F.interpolate(pk, size=e.shape[2:], mode="bilinear",
                                                         align_corners=True))], 1),
                           p[f"pk_fusion{i}.weight"], p[f"pk_fusion{i}.bias"])
                     for i, e in enumerate(feats, start=1)]
        for s_, e in zip(seqs, feats):
            s_.append(e)
    fused = []
    for i, s_ in enumerate(seqs, start=1):
        st = torch.stack(s_, 1)
        bb, tt, cc, hh, ww = st.shape
        hT = _lstm(st.permute(0, 3, 4, 1, 2).reshape(bb * hh * ww, tt, cc), p, f"lstm{i}")
        fused.append(hT.reshape(bb, hh, ww, cc).permute(0, 3, 1, 2))
    e1, e2, e3, e4 = fused
    d = e4
    for name, skip in (("decoder4", e3), ("decoder3", e2), ("decoder2", e1)):
        up = q(F.conv_transpose2d(d, q(p[f"{name}.up.weight"], False), p[f"{name}.up.bias"], stride=2, padding=1,
                                  output_padding=1))
        if up.shape[2:] != skip.shape[2:]:          # the size fallback (src/stf_lstm_unet.py:56-57)
            up = q(F.interpolate(up, size=skip.shape[2:], mode="bilinear", align_corners=True))
        hcat = _conv(torch.cat([up, skip], 1), p[f"{name}.fusion.weight"], p[f"{name}.fusion.bias"])
        d = _rcb(hcat, p, f"{name}.res_conv", training)
    d = q(F.conv_transpose2d(d, q(p["upconv1.weight"], False), p["upconv1.bias"], stride=2, padding=1,
                             output_padding=1))
    d = _rcb(d, p, "final_res", training)
    return {"out": F.conv2d(d, p["final.weight"], p["final.bias"])}
