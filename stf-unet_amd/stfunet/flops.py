"""Algorithmic training FLOPs per sample (2 x MAC of every conv / ConvT / 1x1 / LSTM GEMM,
x3 for forward + both backward GEMMs; SURVEY.md section 8(d) convention) -- the model
work ``bench.py`` divides by, computed from the architecture alone.

UNet: src/unet.py:5-57 (DoubleConv 3x3 x2 per level, ConvTranspose2d(2, 2) ups, OutConv).
STFLSTMUNet: src/stf_lstm_unet.py:71-256 (stem 7x7/s2, ResNet-34 BasicBlocks [3,4,6,3]
with 1x1 downsamples, per-level PK fusion 1x1, nn.LSTM(C, C) input + hidden projections,
DecoderBlocks = ConvT 3x3/s2 + 1x1 fusion + ResidualConvBlock, upconv1 + final block +
1x1 head); ConvTranspose MACs counted per input pixel (h*w*Cin*Cout*k*k).
"""

RESNET34_LAYERS = ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))


def unet_train_flops(in_channels=8, base_c=64, H=256, W=256):
    widths = [base_c * m for m in (1, 2, 4, 8, 16)]
    f, cin, h, w, sizes = 0.0, in_channels, H, W, []
    for i, c in enumerate(widths):
        if i:
            h, w = h // 2, w // 2
        f += 2 * h * w * c * 9 * (cin + c)                  # DoubleConv
        sizes.append((h, w))
        cin = c
    for lvl in range(4):
        hi, lo = widths[4 - lvl], widths[3 - lvl]
        hh, ww = sizes[3 - lvl]
        f += 2 * (hh // 2) * (ww // 2) * hi * lo * 4         # ConvT 2x2 / s2
        f += 2 * hh * ww * lo * 9 * (hi + lo)                # DoubleConv on the concat
    f += 2 * H * W * base_c * 2                              # OutConv 1x1
    return 3.0 * f


def stf_train_flops(T=8, H=256, W=256, use_pk_maps=False, pk_channels=3):
    f = 0.0
    h, w = H // 2, W // 2
    f += T * 2 * h * w * 64 * 49 * (1 + (pk_channels if use_pk_maps else 0))    # stem
    h, w, inpl, scales = h // 2, w // 2, 64, []
    for planes, blocks, stride in RESNET34_LAYERS:
        for b in range(blocks):
            st = stride if b == 0 else 1
            h, w = h // st, w // st
            f += T * 2 * h * w * planes * 9 * (inpl + planes)                    # conv1 + conv2
            if b == 0 and (st != 1 or inpl != planes):
                f += T * 2 * h * w * planes * inpl                               # downsample
            inpl = planes
        scales.append((planes, h, w))
    for c, hh, ww in scales:
        if use_pk_maps:
            f += T * 2 * hh * ww * c * (c + pk_channels)                         # PK fusion
        f += T * 2 * hh * ww * 4 * c * 2 * c                                     # LSTM gates
    for (cin, hin, win), (cout, hh, ww) in zip(scales[:0:-1], scales[-2::-1]):
        f += 2 * hin * win * cin * cout * 9                                      # ConvT 3x3 / s2
        f += 2 * hh * ww * cout * 2 * cout                                       # 1x1 fusion
        f += 2 * 2 * hh * ww * cout * 9 * cout                                   # ResidualConvBlock
    c, hh, ww = scales[0]
    f += 2 * hh * ww * 64 * 32 * 9                                               # upconv1
    f += 2 * 2 * (2 * hh) * (2 * ww) * 32 * 9 * 32                               # final block
    f += 2 * (2 * hh) * (2 * ww) * 32 * 2                                        # head
    return 3.0 * f
