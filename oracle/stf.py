"""Functional fp32 CPU restatement of the reference STF-LSTM-UNet (test infrastructure).

Follows ``src/stf_lstm_unet.py``:

* ``ResidualConvBlock`` :7-35 -- bias-free conv3x3-BN-ReLU-conv3x3-BN, 1x1 conv+BN
  shortcut when Cin != Cout (:20-25), add, ReLU (:33-34)
* ``DecoderBlock`` :38-68 -- ConvT(k3, s2, p1, op1, bias) (:43), bilinear
  (align_corners=True) resize only on size mismatch (:56-57), cat [up, skip] (:60),
  1x1 fusion (bias) (:46,63), ResidualConvBlock (:49,66)
* ``STFLSTMUNet.__init__`` :89-137 and ``forward`` :139-256:
  PK split off the T axis (:146-160), per-t ResNet-34 encoder with its own
  BatchNorm batch statistics per t (:168-186), PK fusion (:188-200), per-pixel
  ``nn.LSTM(C, C)`` over T at four scales using only h_T (:214-242), decoder
  (:245-254). Output is at H/2 x W/2 (reference behaviour).

The encoder is ``torchvision.models.resnet34(weights=None)`` (:102-114); its
arithmetic is restated here as the standard BasicBlock ResNet-34 ([3, 4, 6, 3],
stride-2 first block with 1x1 conv + BN downsample in layer2-4, stem conv7x7 s2
+ BN + ReLU + maxpool3x3 s2 p1).  torchvision is unpinned and absent from the
build image, so this part is pinned to the standard architecture only.
"""
from collections import OrderedDict

import torch
import torch.nn.functional as F

from .unet import batch_norm

RESNET34_LAYERS = ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))


def _bn_shapes(prefix, c, out):
    for leaf in ("weight", "bias", "running_mean", "running_var"):
        out[f"{prefix}.{leaf}"] = (c,)
    out[f"{prefix}.num_batches_tracked"] = ()


def _resblock_shapes(prefix, cin, cout, out):
    out[f"{prefix}.conv_block.0.weight"] = (cout, cin, 3, 3)
    _bn_shapes(f"{prefix}.conv_block.1", cout, out)
    out[f"{prefix}.conv_block.3.weight"] = (cout, cout, 3, 3)
    _bn_shapes(f"{prefix}.conv_block.4", cout, out)
    if cin != cout:
        out[f"{prefix}.shortcut.0.weight"] = (cout, cin, 1, 1)
        _bn_shapes(f"{prefix}.shortcut.1", cout, out)


def param_shapes(in_channels=1, num_classes=2, use_pk_maps=False, pk_channels=3):
    s = OrderedDict()
    cin = in_channels + (pk_channels if use_pk_maps else 0)
    s["conv1.weight"] = (64, cin, 7, 7)
    _bn_shapes("bn1", 64, s)
    inplanes = 64
    for li, (planes, blocks, stride) in enumerate(RESNET34_LAYERS, start=1):
        for b in range(blocks):
            pre = f"layer{li}.{b}"
            st = stride if b == 0 else 1
            s[f"{pre}.conv1.weight"] = (planes, inplanes, 3, 3)
            _bn_shapes(f"{pre}.bn1", planes, s)
            s[f"{pre}.conv2.weight"] = (planes, planes, 3, 3)
            _bn_shapes(f"{pre}.bn2", planes, s)
            if b == 0 and (st != 1 or inplanes != planes):
                s[f"{pre}.downsample.0.weight"] = (planes, inplanes, 1, 1)
                _bn_shapes(f"{pre}.downsample.1", planes, s)
            inplanes = planes
    if use_pk_maps:
        for i, c in enumerate((64, 128, 256, 512), start=1):
            s[f"pk_fusion{i}.weight"] = (c, c + pk_channels, 1, 1)
            s[f"pk_fusion{i}.bias"] = (c,)
    for i, c in enumerate((64, 128, 256, 512), start=1):
        s[f"lstm{i}.weight_ih_l0"] = (4 * c, c)
        s[f"lstm{i}.weight_hh_l0"] = (4 * c, c)
        s[f"lstm{i}.bias_ih_l0"] = (4 * c,)
        s[f"lstm{i}.bias_hh_l0"] = (4 * c,)
    for name, cin_, skip, cout in (("decoder4", 512, 256, 256), ("decoder3", 256, 128, 128),
                                   ("decoder2", 128, 64, 64)):
        s[f"{name}.up.weight"] = (cin_, cout, 3, 3)
        s[f"{name}.up.bias"] = (cout,)
        s[f"{name}.fusion.weight"] = (cout, cout + skip, 1, 1)
        s[f"{name}.fusion.bias"] = (cout,)
        _resblock_shapes(f"{name}.res_conv", cout, cout, s)
    s["upconv1.weight"] = (64, 32, 3, 3)
    s["upconv1.bias"] = (32,)
    _resblock_shapes("final_res", 32, 32, s)
    s["final.weight"] = (num_classes, 32, 1, 1)
    s["final.bias"] = (num_classes,)
    return s


def template_state_dict(**kw):
    return OrderedDict(
        (k, torch.zeros(v, dtype=torch.int64) if k.endswith("num_batches_tracked")
         else torch.zeros(v, dtype=torch.float32))
        for k, v in param_shapes(**kw).items())


def residual_conv_block(x, p, pre, training):
    y = F.conv2d(x, p[f"{pre}.conv_block.0.weight"], padding=1)
    y = F.relu(batch_norm(y, p, f"{pre}.conv_block.1", training))
    y = F.conv2d(y, p[f"{pre}.conv_block.3.weight"], padding=1)
    y = batch_norm(y, p, f"{pre}.conv_block.4", training)
    if f"{pre}.shortcut.0.weight" in p:
        sc = batch_norm(F.conv2d(x, p[f"{pre}.shortcut.0.weight"]), p, f"{pre}.shortcut.1", training)
    else:
        sc = x
    return F.relu(y + sc)


def decoder_block(x, skip, p, pre, training):
    up = F.conv_transpose2d(x, p[f"{pre}.up.weight"], p[f"{pre}.up.bias"], stride=2,
                            padding=1, output_padding=1)
    if up.shape[2:] != skip.shape[2:]:
        up = F.interpolate(up, size=skip.shape[2:], mode="bilinear", align_corners=True)
    h = F.conv2d(torch.cat([up, skip], 1), p[f"{pre}.fusion.weight"], p[f"{pre}.fusion.bias"])
    return residual_conv_block(h, p, f"{pre}.res_conv", training)


def basic_block(x, p, pre, stride, training):
    y = F.conv2d(x, p[f"{pre}.conv1.weight"], stride=stride, padding=1)
    y = F.relu(batch_norm(y, p, f"{pre}.bn1", training))
    y = F.conv2d(y, p[f"{pre}.conv2.weight"], padding=1)
    y = batch_norm(y, p, f"{pre}.bn2", training)
    if f"{pre}.downsample.0.weight" in p:
        sc = F.conv2d(x, p[f"{pre}.downsample.0.weight"], stride=stride)
        sc = batch_norm(sc, p, f"{pre}.downsample.1", training)
    else:
        sc = x
    return F.relu(y + sc)


def encoder(x, p, training):
    """One time step through the ResNet-34 trunk -> (e1, e2, e3, e4)."""
    h = F.conv2d(x, p["conv1.weight"], stride=2, padding=3)
    h = F.relu(batch_norm(h, p, "bn1", training))
    h = F.max_pool2d(h, 3, 2, 1)
    feats = []
    for li, (_, blocks, stride) in enumerate(RESNET34_LAYERS, start=1):
        for b in range(blocks):
            h = basic_block(h, p, f"layer{li}.{b}", stride if b == 0 else 1, training)
        feats.append(h)
    return feats


def lstm_last_hidden(seq, p, pre):
    """nn.LSTM(C, C, batch_first) over seq [N, T, C]; returns h_T [N, C].

    Gate order i, f, g, o (torch); c' = f*c + i*g; h' = o*tanh(c').
    """
    w_ih, w_hh = p[f"{pre}.weight_ih_l0"], p[f"{pre}.weight_hh_l0"]
    bias = p[f"{pre}.bias_ih_l0"] + p[f"{pre}.bias_hh_l0"]
    n, t_len, c = seq.shape
    xproj = seq @ w_ih.t() + bias
    h = seq.new_zeros(n, w_hh.shape[1])
    cell = seq.new_zeros(n, w_hh.shape[1])
    for t in range(t_len):
        i, f, g, o = (xproj[:, t] + h @ w_hh.t()).chunk(4, dim=1)
        cell = torch.sigmoid(f) * cell + torch.sigmoid(i) * torch.tanh(g)
        h = torch.sigmoid(o) * torch.tanh(cell)
    return h


def forward(p, x, training=True, use_pk_maps=False, pk_channels=3):
    """x: [B, T (+pk), Cin, H, W] fp32 -> {"out": [B, classes, H/2, W/2]}."""
    b, total, ch, hgt, wid = x.shape
    pk = None
    steps = total
    if use_pk_maps:
        steps = total - pk_channels
        pk = x[:, steps:].reshape(b, pk_channels, ch, hgt, wid).squeeze(2)
        x = x[:, :steps]
    seqs = [[], [], [], []]
    for t in range(steps):
        xt = x[:, t]
        if pk is not None:
            xt = torch.cat([xt, pk], 1)
        feats = encoder(xt, p, training)
        if pk is not None:
            feats = [F.conv2d(torch.cat([e, F.interpolate(pk, size=e.shape[2:], mode="bilinear",
                                                           align_corners=True)], 1),
                              p[f"pk_fusion{i}.weight"], p[f"pk_fusion{i}.bias"])
                     for i, e in enumerate(feats, start=1)]
        for s, e in zip(seqs, feats):
            s.append(e)
    fused = []
    for i, s in enumerate(seqs, start=1):
        st = torch.stack(s, 1)                                   # [B, T, C, h, w]
        bb, tt, cc, hh, ww = st.shape
        hT = lstm_last_hidden(st.permute(0, 3, 4, 1, 2).reshape(bb * hh * ww, tt, cc), p, f"lstm{i}")
        fused.append(hT.reshape(bb, hh, ww, cc).permute(0, 3, 1, 2))
    e1, e2, e3, e4 = fused
    d = decoder_block(e4, e3, p, "decoder4", training)
    d = decoder_block(d, e2, p, "decoder3", training)
    d = decoder_block(d, e1, p, "decoder2", training)
    d = F.conv_transpose2d(d, p["upconv1.weight"], p["upconv1.bias"], stride=2, padding=1,
                           output_padding=1)
    d = residual_conv_block(d, p, "final_res", training)
    out = F.conv2d(d, p["final.weight"], p["final.bias"])
    if training:
        for k in p:
            if k.endswith("num_batches_tracked"):
                enc = k.startswith(("bn1.", "layer"))
                p[k] += steps if enc else 1
    return {"out": out}


def train_flops_per_sample(T=8, H=256, W=256, use_pk_maps=False, pk_channels=3):
    """Algorithmic FLOPs (2*MAC) of conv/convT/1x1/LSTM GEMMs per sample, x3 for
    training (SURVEY.md section 8(d) convention; ConvTranspose MACs counted per
    input pixel: h*w*Cin*Cout*k*k)."""
    cin = 1 + (pk_channels if use_pk_maps else 0)
    f = 0.0
    h, w = H // 2, W // 2
    f += T * 2 * h * w * 64 * 49 * cin                      # stem
    h, w = h // 2, w // 2
    inpl = 64
    scales = []
    for planes, blocks, stride in RESNET34_LAYERS:
        for b in range(blocks):
            st = stride if b == 0 else 1
            h2, w2 = h // st, w // st
            f += T * 2 * h2 * w2 * planes * 9 * inpl            # conv1
            f += T * 2 * h2 * w2 * planes * 9 * planes          # conv2
            if b == 0 and (st != 1 or inpl != planes):
                f += T * 2 * h2 * w2 * planes * inpl            # downsample 1x1
            h, w, inpl = h2, w2, planes
        scales.append((planes, h, w))
    for c, hh, ww in scales:
        if use_pk_maps:
            f += T * 2 * hh * ww * c * (c + pk_channels)
        f += T * 2 * hh * ww * 4 * c * (2 * c)                 # LSTM x- and h-projections
    for (cin_, hin, win), (cout, hh, ww) in zip(scales[:0:-1], scales[-2::-1]):
        f += 2 * hin * win * cin_ * cout * 9                    # ConvT k3 s2
        f += 2 * hh * ww * cout * (2 * cout)                    # 1x1 fusion
        f += 2 * 2 * hh * ww * cout * 9 * cout                  # ResidualConvBlock
    c, hh, ww = scales[0]
    f += 2 * hh * ww * 64 * 32 * 9                              # upconv1
    f += 2 * 2 * (2 * hh) * (2 * ww) * 32 * 9 * 32              # final_res
    f += 2 * (2 * hh) * (2 * ww) * 32 * 2                       # final 1x1
    return 3.0 * f
