"""Kernel-level parity of the gfx950 C-ABI against torch fp32 references.

Inputs are rounded to bf16 first, so the reference sees exactly the operands the
MFMA kernels see; remaining differences are fp32 accumulation order and the
bf16 rounding of stored outputs (tolerance: relative L2 <= 1e-2 for bf16
outputs, <= 2e-3 for fp32 outputs/statistics).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def bfr(t):
    return t.to(torch.bfloat16).float()


def feat_from(x, cs=None, off=0):
    """[N, C, H, W] float -> Feat holding bf16(x) (optionally inside a wider buffer)."""
    from stfunet.nhwc import Feat
    N, C, H, W = x.shape
    cs = cs or C
    buf = torch.zeros(N, H, W, cs, dtype=torch.bfloat16, device=DEV)
    buf[..., off:off + C] = x.permute(0, 2, 3, 1).to(torch.bfloat16)
    return Feat(buf.view(-1), N, H, W, C, cs, off)


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


@pytest.mark.parametrize("cin,cout,H,stride,R", [(64, 128, 16, 1, 3), (8, 64, 32, 1, 3), (8, 64, 20, 2, 7),
                                                  (8, 128, 18, 1, 3), (128, 64, 16, 1, 3),
                                                  (64, 128, 16, 2, 3), (64, 128, 16, 2, 1), (32, 32, 8, 1, 3),
                                                  (256, 512, 8, 1, 3)])
def test_conv_forward_stats_and_dgrad(cin, cout, H, stride, R):
    from stfunet import nhwc
    pad = R // 2
    x = bfr(torch.randn(2, cin, H, H + 2, device=DEV))
    w = bfr(torch.randn(cout, cin, R, R, device=DEV) / (cin * R * R) ** 0.5)
    b = torch.randn(cout, device=DEV)
    ref = F.conv2d(x, w, b, stride=stride, padding=pad)
    src = feat_from(x)
    Ho, Wo = ref.shape[2:]
    dst = nhwc.new_feat(2, Ho, Wo, cout, DEV)
    stats, tiles = nhwc.igemm(src, nhwc.pack_weight(w.contiguous(), 0, cin), cout, dst, R, R, stride, pad,
                              bias=b, want_stats=True)
    out = dst.dense()
    assert rel(out, ref) < 1e-2
    s = stats.view(tiles, 2, cout).sum(0)
    assert rel(s[0], out.sum((0, 2, 3))) < 2e-3
    assert rel(s[1], (out * out).sum((0, 2, 3))) < 2e-3
    # input gradient through the transposed gather
    if cin % 8 == 0 and cout % 8 == 0:
        dy = bfr(torch.randn_like(ref))
        xr = x.clone().requires_grad_(True)
        F.conv2d(xr, w, None, stride=stride, padding=pad).backward(dy)
        dsrc = feat_from(dy)
        dx = nhwc.new_feat(2, H, H + 2, cin, DEV)
        nhwc.igemm(dsrc, nhwc.pack_weight(w.contiguous(), 1), cin, dx, R, R, stride, pad, transposed=True)
        assert rel(dx.dense(), xr.grad) < 1e-2


@pytest.mark.parametrize("n,cin,cout,H,W,R,acc", [
    (2, 64, 128, 15, 17, 3, False),     # odd input sizes: the four parity classes differ in size
    (4, 128, 256, 32, 32, 3, True),     # several blocks per class, accumulate into dx
    (2, 64, 128, 13, 16, 1, False),     # 1x1 / stride 2: odd classes get no taps (dx = 0 there)
    (2, 256, 64, 8, 9, 1, True),        # 1x1 / stride 2, accumulate (odd classes keep dx)
    (3, 32, 64, 9, 11, 3, False),       # one 32-channel chunk, 256 x 64 tile (Nout <= 64)
])
def test_strided_dgrad_parity_classes(n, cin, cout, H, W, R, acc):
    """Stride-2 input gradient through the transposed gather with rows ordered by output
    parity class (each class walks only its own taps) vs torch."""
    from stfunet import nhwc
    pad = R // 2
    x = bfr(torch.randn(n, cin, H, W, device=DEV))
    w = bfr(torch.randn(cout, cin, R, R, device=DEV) / (cin * R * R) ** 0.5)
    xr = x.clone().requires_grad_(True)
    y = F.conv2d(xr, w, stride=2, padding=pad)
    dy = bfr(torch.randn_like(y))
    y.backward(dy)
    base = bfr(torch.randn(n, cin, H, W, device=DEV))
    dx = feat_from(base) if acc else nhwc.new_feat(n, H, W, cin, DEV)
    nhwc.conv_dgrad(feat_from(dy), w.contiguous(), dx, R, R, 2, pad, accumulate=acc)
    ref = xr.grad + base if acc else xr.grad
    assert rel(dx.dense(), ref) < 1e-2
    if R == 1 and not acc:                  # no tap reaches odd rows / columns
        assert dx.dense()[:, :, 1::2].abs().max().item() == 0
        assert dx.dense()[:, :, :, 1::2].abs().max().item() == 0
    if R == 1 and acc:                      # accumulating: the tap-less classes are not launched at all,
        b = feat_from(base).dense()         # so odd rows / columns keep dx bit for bit
        assert torch.equal(dx.dense()[:, :, 1::2], b[:, :, 1::2])
        assert torch.equal(dx.dense()[:, :, :, 1::2], b[:, :, :, 1::2])


@pytest.mark.parametrize("cin,cout,H,stride,R,pad", [(64, 128, 16, 1, 3, 1), (8, 64, 32, 1, 3, 1),
                                                     (64, 128, 16, 2, 3, 1), (64, 64, 16, 2, 1, 0),
                                                     (256, 256, 8, 1, 3, 1), (8, 64, 16, 2, 7, 3)])
def test_wgrad(cin, cout, H, stride, R, pad):
    from stfunet import nhwc
    x = bfr(torch.randn(2, cin, H, H, device=DEV))
    w = torch.randn(cout, cin, R, R, device=DEV).requires_grad_(True)
    y = F.conv2d(x, w, stride=stride, padding=pad)
    dy = bfr(torch.randn_like(y))
    y.backward(dy)
    out = torch.empty(cout * cin * R * R, device=DEV)
    nhwc.wgrad(feat_from(dy), feat_from(x), R, R, stride, pad, out)
    assert rel(out.view_as(w), w.grad) < 2e-3


@pytest.mark.parametrize("n,cin,cout,H,W,xcs,xoff,dycs", [
    (3, 64, 64, 37, 21, 64, 0, 64),        # ragged 16x4 pixel tiles at both edges
    (2, 128, 64, 32, 32, 192, 64, 64),     # x = slice of a concat buffer (dec1.0 shape)
    (2, 64, 128, 12, 9, 64, 0, 192),       # W < 16 -> 8x8 pixel tiles; dy slice of wider rows
    (1, 128, 128, 8, 8, 128, 0, 128),      # STF layer4-like 8x8
    (16, 64, 64, 64, 64, 64, 0, 64),       # many pixel tiles per split
])
def test_wgrad_fused_3x3(n, cin, cout, H, W, xcs, xoff, dycs):
    """Fused-tap 3x3/s1/p1 weight gradient (one block = all nine taps)."""
    from stfunet import nhwc
    x = bfr(torch.randn(n, cin, H, W, device=DEV))
    w = torch.randn(cout, cin, 3, 3, device=DEV).requires_grad_(True)
    y = F.conv2d(x, w, padding=1)
    dy = bfr(torch.randn_like(y))
    y.backward(dy)
    out = torch.empty(cout * cin * 9, device=DEV)
    nhwc.wgrad(feat_from(dy, cs=dycs), feat_from(x, cs=xcs, off=xoff), 3, 3, 1, 1, out)
    assert rel(out.view_as(w), w.grad) < 2e-3


@pytest.mark.parametrize("n,cin,cout,H,W,groups,acc,xcs,xoff", [
    (2, 64, 64, 37, 70, 1, False, 64, 0),        # ragged 16x32 halo tiles at both edges
    (4, 128, 128, 64, 64, 2, False, 192, 64),    # grouped statistics, source = concat slice
    (2, 32, 128, 20, 96, 1, True, 32, 0),        # one 32-channel chunk, accumulate into dst
    (1, 96, 64, 64, 80, 1, False, 96, 0),        # three chunks
    (4, 64, 128, 16, 16, 2, False, 64, 0),       # 16x16 tiles (16 <= W < 32), grouped statistics
    (2, 128, 64, 21, 24, 1, True, 128, 0),       # 16x16 tiles, ragged, accumulate
    (6, 256, 256, 16, 16, 3, True, 320, 64),     # two 16x16 images per 16x32 tile, accumulate, slice source
    (3, 64, 64, 16, 16, 3, False, 64, 0),        # one image per group: single-image 16x16 tiles
    (16, 512, 512, 8, 8, 4, False, 512, 0),      # four 8x8 images per 8x32 tile (STF layer4)
    (8, 256, 128, 8, 8, 2, True, 320, 64),       # 8x8 four-image tiles, accumulate, slice source
    (2, 128, 256, 37, 70, 1, False, 128, 0),     # wide kernel (128-channel slices): ragged tiles, two slices
    (4, 256, 128, 32, 64, 2, True, 320, 64),     # wide: grouped statistics, accumulate, slice source; wide dgrad
    (3, 64, 384, 40, 33, 3, False, 64, 0),       # wide: three slices, two chunks, one image per group
    (4, 1024, 512, 16, 16, 2, False, 1024, 0),   # UNet bottleneck (> 256 outputs at 16x16): two-image tiles, dgrad too
])
def test_conv3x3_halo(n, cin, cout, H, W, groups, acc, xcs, xoff):
    """3x3/s1/p1 conv through the halo kernel (auto for W >= 64): output, grouped
    BN partial statistics, accumulate, and the stride-1 dgrad over flipped taps."""
    from stfunet import nhwc
    # NaN-filled blocks back in the caching allocator: a statistics row the kernel does not
    # write (a grid that disagrees with stf_igemm_stat_tiles) shows up as NaN below
    torch.full((16 << 20,), float("nan"), device=DEV)
    x = bfr(torch.randn(n, cin, H, W, device=DEV))
    w = bfr(torch.randn(cout, cin, 3, 3, device=DEV) / (cin * 9) ** 0.5)
    b = torch.randn(cout, device=DEV)
    ref = F.conv2d(x, w, b, padding=1)
    dst = nhwc.new_feat(n, H, W, cout, DEV)
    base = None
    if acc:
        base = bfr(torch.randn_like(ref))
        dst.buf.view(n, H, W, cout).copy_(base.permute(0, 2, 3, 1).to(torch.bfloat16))
        ref = ref + base
    stats, tiles = nhwc.igemm(feat_from(x, cs=xcs, off=xoff), nhwc.pack_weight(w.contiguous(), 0, cin), cout, dst,
                              3, 3, 1, 1, bias=b, want_stats=True, groups=groups, accumulate=acc)
    out = dst.dense()
    assert rel(out, ref) < 1e-2
    st = stats.view(groups, tiles, 2, cout).sum(1)
    og = out.view(groups, n // groups, cout, H, W)
    for g in range(groups):
        assert rel(st[g, 0], og[g].sum((0, 2, 3))) < 2e-3
        assert rel(st[g, 1], (og[g] ** 2).sum((0, 2, 3))) < 2e-3
    dy = bfr(torch.randn(n, cout, H, W, device=DEV))
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, padding=1).backward(dy)
    dx = nhwc.new_feat(n, H, W, cin, DEV)
    nhwc.conv_dgrad(feat_from(dy), w.contiguous(), dx, 3, 3, 1, 1)
    assert rel(dx.dense(), xr.grad) < 1e-2


@pytest.mark.parametrize("n,cin,cout,H,W", [(2, 64, 64, 37, 70), (2, 128, 256, 37, 70), (3, 256, 128, 16, 16)])
def test_conv3x3_halo_bias_without_statistics(n, cin, cout, H, W):
    """The eval-mode forward (bias, no BatchNorm statistics) through the halo kernels: the 64-channel
    slices, the wide 128-channel slices (its no-statistics variant also runs the dgrads) and 16x16
    tiles."""
    from stfunet import nhwc
    x = bfr(torch.randn(n, cin, H, W, device=DEV))
    w = bfr(torch.randn(cout, cin, 3, 3, device=DEV) / (cin * 9) ** 0.5)
    b = torch.randn(cout, device=DEV)
    dst = nhwc.new_feat(n, H, W, cout, DEV)
    nhwc.igemm(feat_from(x), nhwc.pack_weight(w.contiguous(), 0, cin), cout, dst, 3, 3, 1, 1, bias=b,
               want_stats=False)
    assert rel(dst.dense(), F.conv2d(x, w, b, padding=1)) < 1e-2


@pytest.mark.parametrize("n,H,W,groups,dcs", [(6, 20, 36, 3, 64), (4, 64, 64, 2, 96), (2, 16, 16, 1, 64)])
def test_conv3x3_8channel_input(n, H, W, groups, dcs):
    """The 8-channel-input 3x3 kernel (conv3x3_c8_kernel: halo of 16-B pixel rows, one
    ds_read_b128 per tap fragment): output (into a wider destination), bias, grouped BN
    partial statistics against torch fp32 on bf16-rounded operands."""
    from stfunet import nhwc
    torch.full((16 << 20,), float("nan"), device=DEV)     # unwritten statistics rows would show as NaN
    x = bfr(torch.randn(n, 8, H, W, device=DEV))
    w = bfr(torch.randn(64, 8, 3, 3, device=DEV) / 72 ** 0.5)
    b = torch.randn(64, device=DEV)
    ref = F.conv2d(x, w, b, padding=1)
    wide = nhwc.new_feat(n, H, W, dcs, DEV)
    dst = wide.slice(0, 64)
    stats, tiles = nhwc.igemm(feat_from(x), nhwc.pack_weight(w.contiguous(), 0, 8), 64, dst, 3, 3, 1, 1, bias=b,
                              want_stats=True, groups=groups)
    out = dst.dense()
    assert rel(out, ref) < 1e-2
    st = stats.view(groups, tiles, 2, 64).sum(1)
    og = out.view(groups, n // groups, 64, H, W)
    for g in range(groups):
        assert rel(st[g, 0], og[g].sum((0, 2, 3))) < 2e-3
        assert rel(st[g, 1], (og[g] ** 2).sum((0, 2, 3))) < 2e-3


@pytest.mark.parametrize("n,cin,cout,H,W,R,groups,acc", [
    (16, 512, 512, 8, 8, 3, 8, False),           # STF layer4 shape (per-time-step groups), split 8
    (4, 2048, 1024, 8, 8, 1, 1, False),          # LSTM-backward-like 1x1, split 4
    (8, 256, 256, 8, 12, 3, 2, True),            # accumulate into dst, grouped
])
def test_conv_splitk(n, cin, cout, H, W, R, groups, acc):
    """Small-M plain gathers run split over K (fp32 partials + fold launch): output,
    accumulate, bias and grouped BN partial statistics vs torch fp32."""
    import ctypes
    from stfunet import _lib, nhwc
    pad = R // 2
    x = bfr(torch.randn(n, cin, H, W, device=DEV))
    w = bfr(torch.randn(cout, cin, R, R, device=DEV) / (cin * R * R) ** 0.5)
    b = torch.randn(cout, device=DEV)
    ref = F.conv2d(x, w, b, padding=pad)
    dst = nhwc.new_feat(n, H, W, cout, DEV)
    if acc:
        base = bfr(torch.randn_like(ref))
        dst.buf.view(n, H, W, cout).copy_(base.permute(0, 2, 3, 1).to(torch.bfloat16))
        ref = ref + base
    src = feat_from(x)
    a = _lib.IgemmArgs(nhwc._geom(src, H, W, R, R, 1, pad, False), src.ptr(), None, cout, dst.ptr(), cout)
    a.group_rows = n * H * W // groups
    assert _lib.load().stf_igemm_ws_bytes(ctypes.byref(a)) > 0, "shape expected to run split over K"
    stats, tiles = nhwc.igemm(src, nhwc.pack_weight(w.contiguous(), 0, cin), cout, dst, R, R, 1, pad, bias=b,
                              want_stats=True, groups=groups, accumulate=acc)
    out = dst.dense()
    assert rel(out, ref) < 1e-2
    st = stats.view(groups, tiles, 2, cout).sum(1)
    og = out.view(groups, n // groups, cout, H, W)
    for g in range(groups):
        assert rel(st[g, 0], og[g].sum((0, 2, 3))) < 2e-3
        assert rel(st[g, 1], (og[g] ** 2).sum((0, 2, 3))) < 2e-3


@pytest.mark.parametrize("n,cin,cout,H,W,groups,relu,acc", [
    (2, 64, 128, 40, 72, 1, True, False),     # halo 16x32 tiles, ragged edges
    (4, 128, 64, 24, 20, 2, True, False),     # halo 16x16 tiles, two BN groups
    (8, 256, 256, 16, 16, 2, True, False),    # two 16x16 images per halo tile (STF layer3)
    (2, 64, 64, 64, 64, 1, False, True),      # plain BN (no ReLU), accumulate
    (6, 256, 128, 8, 8, 2, True, False),      # linear kernel (6 images: no 4-image halo tiles): separate reduce
    (8, 256, 128, 8, 8, 2, True, False),      # 8x8 four-image halo tiles: separate reduce
    (2, 128, 64, 40, 72, 2, True, False),     # wide kernel (128-channel slice), ragged, one image per group
    (4, 256, 64, 48, 40, 2, True, False),     # wide kernel, two slices x two groups per workgroup run
    (2, 128, 128, 64, 64, 1, False, True),    # wide kernel, plain BN, accumulate
    (4, 512, 1024, 16, 16, 2, True, False),   # > 256 outputs at 16x16: two-image halo tiles (UNet bottleneck)
])
def test_dgrad_fused_bn_backward_reduce(n, cin, cout, H, W, groups, relu, acc):
    """conv_dgrad with ``bnr``: dz identical to the plain dgrad, and the fused partial
    sums (g, g*xhat) equal to a separate stf_bn_bwd_reduce pass over the stored dz."""
    from stfunet import nhwc
    from stfunet._lib import call, load, stream
    from stfunet.nhwc import BNState, _p
    w = bfr(torch.randn(cout, cin, 3, 3, device=DEV) / (cout * 9) ** 0.5)
    dy = feat_from(bfr(torch.randn(n, cout, H, W, device=DEV)))
    y = feat_from(bfr(torch.randn(n, cin, H, W, device=DEV) * 2 + 0.5))
    st = BNState(cin, DEV, n * H * W, groups)
    st.mean.copy_(torch.randn(groups, cin, device=DEV) * 0.3 + 0.5)
    st.invstd.copy_(torch.rand(groups, cin, device=DEV) + 0.5)
    st.scale.copy_(torch.randn(groups, cin, device=DEV))
    st.shift.copy_(torch.randn(groups, cin, device=DEV) * 0.5)
    base = bfr(torch.randn(n, cin, H, W, device=DEV))
    dx0 = feat_from(base) if acc else nhwc.new_feat(n, H, W, cin, DEV)
    nhwc.conv_dgrad(dy, w.contiguous(), dx0, 3, 3, 1, 1, accumulate=acc)
    dx = feat_from(base) if acc else nhwc.new_feat(n, H, W, cin, DEV)
    part, tiles = nhwc.conv_dgrad(dy, w.contiguous(), dx, 3, 3, 1, 1, accumulate=acc, bnr=(y, st, relu))
    assert torch.equal(dx.buf, dx0.buf)
    t2 = load().stf_bn_bwd_tiles(n, H, W, cin, groups, 0)
    ref = torch.empty(groups * t2 * 2 * cin, dtype=torch.float32, device=DEV)
    call("stf_bn_bwd_reduce", dx.ptr(), dx.cs, None, y.ptr(), y.cs, n, H, W, cin, groups, _p(st.scale),
         _p(st.shift), _p(st.mean), _p(st.invstd), int(relu), None, 0, None, _p(ref), stream())
    got = part.view(groups, tiles, 2, cin).double().sum(1)
    exp = ref.view(groups, t2, 2, cin).double().sum(1)
    assert rel(got, exp) < 1e-5
    # and against a direct float64 restatement
    g = dx.dense().double().view(groups, n // groups, cin, H, W)
    yy = y.dense().double().view(groups, n // groups, cin, H, W)
    sc, sh = st.scale.double()[:, None, :, None, None], st.shift.double()[:, None, :, None, None]
    if relu:
        g = g * ((yy * sc + sh) > 0)
    xh = (yy - st.mean.double()[:, None, :, None, None]) * st.invstd.double()[:, None, :, None, None]
    assert rel(got[:, 0], g.sum((1, 3, 4))) < 1e-5
    assert rel(got[:, 1], (g * xh).sum((1, 3, 4))) < 1e-5


def test_conv_into_concat_slice():
    from stfunet import nhwc
    x = bfr(torch.randn(2, 64, 8, 8, device=DEV))
    w = bfr(torch.randn(32, 64, 3, 3, device=DEV) / 24)
    ref = F.conv2d(x, w, padding=1)
    cat = nhwc.zeros_feat(2, 8, 8, 96, DEV)
    nhwc.igemm(feat_from(x, cs=72, off=8), nhwc.pack_weight(w.contiguous(), 0, 64), 32, cat.slice(64, 32),
               3, 3, 1, 1)
    full = cat.dense()
    assert rel(full[:, 64:], ref) < 1e-2
    assert full[:, :64].abs().max().item() == 0


@pytest.mark.parametrize("cin,cout,h", [(128, 64, 8), (1024, 512, 4), (64, 32, 16), (256, 128, 8)])
def test_convT2x2_fwd_dgrad_wgrad(cin, cout, h):
    from stfunet import nhwc
    x = bfr(torch.randn(2, cin, h, h, device=DEV))
    w = bfr(torch.randn(cin, cout, 2, 2, device=DEV) / cin ** 0.5).requires_grad_(True)
    b = torch.randn(cout, device=DEV)
    xr = x.clone().requires_grad_(True)
    ref = F.conv_transpose2d(xr, w, b, stride=2)
    dst = nhwc.zeros_feat(2, 2 * h, 2 * h, 2 * cout, DEV)
    nhwc.igemm(feat_from(x), nhwc.pack_weight(w.detach().contiguous(), 2), 4 * cout, dst.slice(0, cout), 1, 1,
               1, 0, bias=b, scatter2x2=True)
    assert rel(dst.dense()[:, :cout], ref) < 1e-2
    dy = bfr(torch.randn_like(ref))
    ref.backward(dy)
    dyf = feat_from(dy)
    dx = nhwc.new_feat(2, h, h, cin, DEV)
    nhwc.igemm(dyf, nhwc.pack_weight(w.detach().contiguous(), 3), cin, dx, 2, 2, 2, 0)
    assert rel(dx.dense(), xr.grad) < 1e-2
    dw = torch.empty(cin * cout * 4, device=DEV)
    nhwc.wgrad(feat_from(x), dyf, 2, 2, 2, 0, dw)
    assert rel(dw.view_as(w), w.grad) < 2e-3
    db = torch.empty(cout, device=DEV)
    nhwc.channel_sum(dyf, db)
    assert rel(db, dy.sum((0, 2, 3))) < 2e-3


def test_convT3x3_s2_gather():
    from stfunet import nhwc
    x = bfr(torch.randn(2, 64, 8, 8, device=DEV))
    w = bfr(torch.randn(64, 32, 3, 3, device=DEV) / 24)
    b = torch.randn(32, device=DEV)
    ref = F.conv_transpose2d(x, w, b, stride=2, padding=1, output_padding=1)
    dst = nhwc.new_feat(2, 16, 16, 32, DEV)
    nhwc.igemm(feat_from(x), nhwc.pack_weight(w.contiguous(), 4), 32, dst, 3, 3, 2, 1, transposed=True, bias=b)
    assert rel(dst.dense(), ref) < 1e-2


class _BN:
    def __init__(self, C):
        self.bn = torch.nn.BatchNorm2d(C).to(DEV)
        with torch.no_grad():
            self.bn.weight.uniform_(0.5, 1.5)
            self.bn.bias.uniform_(-0.5, 0.5)


@pytest.mark.parametrize("n,C,H,W,groups", [(4, 64, 20, 12, 2), (2, 128, 16, 16, 1), (6, 256, 6, 10, 3)])
def test_bn_act_pool_bitwise(n, C, H, W, groups):
    """The pooled BN apply (BN + ReLU + Down's 2x2 max pool in one pass): its full-size output equals
    the un-pooled apply bit for bit, and its pooled output is exactly the 2x2 max of that output
    (grouped statistics, a channel slice of a wider source and destination)."""
    from stfunet import nhwc
    y = feat_from(torch.randn(n, C, H, W, device=DEV) * 2 + 0.3, cs=C + 64, off=32)
    st = nhwc.BNState(C, DEV, n * H * W, groups)
    st.scale.copy_(torch.randn(groups, C, device=DEV))
    st.shift.copy_(torch.randn(groups, C, device=DEV) * 0.5)
    ref = nhwc.zeros_feat(n, H, W, C, DEV)
    nhwc.bn_act(y, st, ref)
    out = nhwc.zeros_feat(n, H, W, 2 * C, DEV).slice(C, C)
    pooled = nhwc.new_feat(n, H // 2, W // 2, C, DEV)
    nhwc.bn_act(y, st, out, pooled=pooled)
    assert torch.equal(out.dense(), ref.dense())
    assert torch.equal(pooled.dense(), F.max_pool2d(ref.dense(), 2))


@pytest.mark.parametrize("pool,C", [(False, 64), (True, 64), (True, 128), (True, 512)])
def test_bn_forward_backward(pool, C):
    from stfunet import nhwc
    H = 16
    y = bfr(torch.randn(2, C, H, H, device=DEV) * 2 + 0.5)
    m = _BN(C)
    ref_bn = torch.nn.BatchNorm2d(C).to(DEV)
    ref_bn.load_state_dict(m.bn.state_dict())
    yr = y.clone().requires_grad_(True)
    a_ref = F.relu(ref_bn(yr))
    yf = feat_from(y)
    s = y.sum((0, 2, 3))
    s2 = (y * y).sum((0, 2, 3))
    stats = torch.stack([s, s2]).contiguous().view(-1)
    st = nhwc.bn_finalize(stats, 1, m.bn, yf.M, training=True)
    out = nhwc.zeros_feat(2, H, H, 2 * C, DEV)
    pooled = nhwc.new_feat(2, H // 2, H // 2, C, DEV) if pool else None
    nhwc.bn_act(yf, st, out.slice(C, C), pooled=pooled)
    # (the finalize may run inside bn_act's launch: the running stats are final once the
    # BNState has been consumed -- or at nhwc.flush_batches_tracked())
    assert rel(m.bn.running_mean, ref_bn.running_mean) < 1e-5
    assert rel(m.bn.running_var, ref_bn.running_var) < 1e-5
    assert rel(out.dense()[:, C:], a_ref) < 1e-2
    if pool:
        # pool the bf16-rounded activations (straight-through) so ties break like the kernel
        a_q = a_ref + (bfr(a_ref) - a_ref).detach()
        p_ref = F.max_pool2d(a_q, 2)
        assert rel(pooled.dense(), p_ref) < 1e-2
        dp = bfr(torch.randn_like(p_ref))
        dz = bfr(torch.randn_like(a_ref))
        # route through the kernel's own bf16 activations (tie-breaking matches)
        (p_ref * dp).sum().add((a_ref * dz).sum()).backward()
        dzf = nhwc.zeros_feat(2, H, H, 2 * C, DEV).slice(C, C)
        dzf.buf.view(2, H, H, 2 * C)[..., C:] = dz.permute(0, 2, 3, 1).to(torch.bfloat16)
        dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        dy = nhwc.bn_backward(yf, st, m.bn, dg, db, dz=dzf, dpool=feat_from(dp))
    else:
        dz = bfr(torch.randn_like(a_ref))
        a_ref.backward(dz)
        dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        dy = nhwc.bn_backward(yf, st, m.bn, dg, db, dz=feat_from(dz))
    assert rel(dg, ref_bn.weight.grad) < 2e-2
    assert rel(db, ref_bn.bias.grad) < 2e-2
    assert rel(dy.dense(), yr.grad) < 2e-2


def test_head_and_loss():
    from stfunet import _lib, nhwc
    from stfunet._lib import call, stream
    from oracle import loss as o_loss
    N, C, H, W, K = 2, 64, 16, 16, 2
    y = bfr(torch.randn(N, C, H, W, device=DEV))
    m = _BN(C)
    wt = torch.randn(K, C, device=DEV) / 8
    bias = torch.randn(K, device=DEV)
    target = (torch.rand(N, H, W, device=DEV) > 0.7).long()
    yf = feat_from(y)
    stats = torch.stack([y.sum((0, 2, 3)), (y * y).sum((0, 2, 3))]).contiguous().view(-1)
    st = nhwc.bn_finalize(stats, 1, m.bn, yf.M, training=False)
    logits = torch.empty(N, K, H, W, device=DEV)
    p = lambda t: nhwc._p(t)  # noqa: E731
    call("stf_head_fwd", yf.ptr(), N, H, W, C, p(st.scale), p(st.shift), p(wt), p(bias), K, p(logits), stream())
    yr = y.clone().requires_grad_(True)
    wr = wt.clone().requires_grad_(True)
    br = bias.clone().requires_grad_(True)
    a = F.relu(yr * st.scale.view(1, -1, 1, 1) + st.shift.view(1, -1, 1, 1))
    ref = F.conv2d(a, wr.view(K, C, 1, 1), br)
    assert rel(logits, ref) < 1e-4
    # loss forward / backward vs the oracle criterion
    lg = logits.clone().requires_grad_(True)
    ref_loss = o_loss.criterion(lg, target)
    ref_loss.backward()
    terms = torch.empty(_lib.load().stf_loss_scratch_floats(N, K), device=DEV)
    loss = torch.empty(1, device=DEV)
    call("stf_loss_fwd", p(logits), p(target), N, H, W, K, p(terms), p(loss), stream())
    assert abs(loss.item() - ref_loss.item()) < 1e-5
    dl = torch.empty_like(logits)
    go = torch.ones(1, device=DEV)
    call("stf_loss_bwd", p(logits), p(target), N, H, W, K, p(terms), p(go), p(dl), stream())
    assert rel(dl, lg.grad) < 1e-4
    # head backward
    z = yr * st.scale.view(1, -1, 1, 1) + st.shift.view(1, -1, 1, 1)
    gref = torch.autograd.grad(ref, a, dl, retain_graph=True)[0] * (z > 0)
    ref.backward(dl)
    tiles = _lib.load().stf_head_tiles(N, H, W, C)
    g = nhwc.new_feat(N, H, W, C, DEV)
    bnp = torch.empty(tiles * 2 * C, device=DEV)
    hp = torch.empty((tiles + 1) * K * (C + 1), device=DEV)
    dw, dbias = torch.empty(K * C, device=DEV), torch.empty(K, device=DEV)
    call("stf_head_bwd", p(dl), yf.ptr(), N, H, W, C, p(st.scale), p(st.shift), p(st.mean), p(st.invstd),
         p(wt), K, g.ptr(), p(bnp), p(hp), p(dw), p(dbias), stream())
    assert rel(dw.view(K, C), wr.grad) < 1e-4
    assert rel(dbias, br.grad) < 1e-4
    assert rel(g.dense(), gref) < 1e-2


def test_loss_saturated_empty_set():
    from stfunet import _lib
    from stfunet._lib import call, stream
    from stfunet.nhwc import _p
    from oracle import loss as o_loss
    logits = torch.zeros(2, 2, 4, 4, device=DEV)
    logits[:, 0] = 200.0
    logits[:, 1] = -200.0
    target = torch.zeros(2, 4, 4, dtype=torch.long, device=DEV)
    terms = torch.empty(_lib.load().stf_loss_scratch_floats(2, 2), device=DEV)
    loss = torch.empty(1, device=DEV)
    call("stf_loss_fwd", _p(logits), _p(target), 2, 4, 4, 2, _p(terms), _p(loss), stream())
    ref = o_loss.criterion(logits, target).item()
    assert abs(loss.item() - ref) < 1e-6


def test_adamw_flat_matches_oracle():
    from stfunet._lib import call, stream
    from stfunet.nhwc import _p
    from oracle.optim import adamw_step
    n = 10007
    p0 = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    m = torch.randn(n, device=DEV) * 0.1
    v = torch.rand(n, device=DEV) * 0.1
    pr, mr, vr = p0.clone(), m.clone(), v.clone()
    adamw_step([pr], [g], [mr], [vr], 3, lr=1e-3)
    b1, b2 = 0.9, 0.999
    call("stf_adamw", _p(p0), _p(g), _p(m), _p(v), n, 1e-3, b1, b2, 1e-8, 1e-4, 1 - b1 ** 3, 1 - b2 ** 3, stream())
    assert rel(p0, pr) < 1e-6 and rel(m, mr) < 1e-6 and rel(v, vr) < 1e-6


PACK_JOBS = [((64, 8, 3, 3), 0, 8), ((128, 64, 3, 3), 0, 64), ((64, 128, 3, 3), 5, 0), ((64, 32, 3, 3), 1, 0),
             ((256, 128, 2, 2), 2, 0), ((256, 128, 2, 2), 3, 0), ((64, 32, 3, 3), 4, 0), ((96, 40, 1, 1), 0, 48)]
# ragged tiles (d0 not a multiple of 64 / 4, d1 not of 16 / 64), the stem's 49-column
# 1x1 view padded to 64, wide 1x1 / 3x3 layers
PACK_RAGGED = [((72, 20, 3, 3), 5, 0), ((72, 20, 3, 3), 1, 0), ((40, 72, 2, 2), 2, 0), ((40, 72, 2, 2), 3, 0),
               ((72, 24, 3, 3), 4, 0), ((64, 49, 1, 1), 0, 64), ((66, 130, 3, 3), 0, 136), ((512, 1024, 3, 3), 5, 0),
               ((1024, 512, 1, 1), 1, 0)]


@pytest.mark.parametrize("tiled,jobs", [("1", PACK_JOBS), ("0", PACK_JOBS), ("1", PACK_RAGGED),
                                        ("1", PACK_RAGGED + [((32, 16, 5, 5), 0, 16)])])
def test_pack_weights_batched_matches_single(monkeypatch, tiled, jobs):
    """stf_pack_weights(_tiled) (one launch, every layout) == stf_pack_weight per tensor, bit
    for bit (the last list has a 5x5 kernel: the whole list takes the element-wise kernel)."""
    from stfunet import nhwc
    monkeypatch.setenv("STF_PACK_TILED", tiled)
    cache = nhwc.PackCache()
    ws = [torch.randn(*shape, device=DEV) for shape, _, _ in jobs]
    nhwc.ACTIVE_PACKS = cache
    try:
        first = [cache.get(w, mode, cpad).clone() for w, (_, mode, cpad) in zip(ws, jobs)]   # on-demand + record
        for w in ws:
            w.mul_(-0.5)                                         # "optimizer step"
        cache.refresh()                                          # one batched launch
        batched = [cache.get(w, mode, cpad) for w, (_, mode, cpad) in zip(ws, jobs)]
    finally:
        nhwc.ACTIVE_PACKS = None
    assert len(cache.recorded) == len(jobs)
    for w, (_, mode, cpad), b, f in zip(ws, jobs, batched, first):
        single = nhwc.pack_weight(w, mode, cpad)
        assert torch.equal(b, single)
        assert not torch.equal(b, f)


@pytest.mark.parametrize("n,cin,cout,h", [(2, 256, 128, 16), (3, 128, 64, 12), (1, 64, 64, 40)])
def test_wgrad_convT2x2_fused(n, cin, cout, h):
    """Fused 4-tap ConvTranspose2d(2, 2) weight gradient (incl. ragged pixel tiles)."""
    from stfunet import nhwc
    x = bfr(torch.randn(n, cin, h, h, device=DEV))
    w = torch.randn(cin, cout, 2, 2, device=DEV).requires_grad_(True)
    y = F.conv_transpose2d(x, w, stride=2)
    dy = bfr(torch.randn_like(y))
    y.backward(dy)
    dw = torch.empty(cin * cout * 4, device=DEV)
    nhwc.wgrad(feat_from(x), feat_from(dy), 2, 2, 2, 0, dw)
    assert rel(dw.view_as(w), w.grad) < 2e-3


@pytest.mark.parametrize("n,H,W,dycs,dyoff", [
    (3, 37, 21, 64, 0),         # ragged 16x16 tiles at both edges, fewer tiles than workgroups
    (16, 64, 64, 64, 0),        # several tiles per workgroup
    (2, 12, 40, 192, 64),       # dy = slice of a wider concat buffer
    (8, 256, 256, 64, 0),       # UNet enc1.0 rows (256 x 256), many tiles per workgroup
])
def test_wgrad_fused_c8(n, H, W, dycs, dyoff):
    """Fused-tap weight gradient of the 8-channel-input 3x3 layer (wgrad3x3_c8_kernel: x halo and
    dy tile in LDS, K split over the waves) vs torch fp32 on the same bf16 operands."""
    from stfunet import nhwc, _lib
    import ctypes
    x = bfr(torch.randn(n, 8, H, W, device=DEV))
    w = torch.randn(64, 8, 3, 3, device=DEV).requires_grad_(True)
    y = F.conv2d(x, w, padding=1)
    dy = bfr(torch.randn_like(y))
    y.backward(dy)
    fx, fdy = feat_from(x), feat_from(dy, cs=dycs, off=dyoff)
    g = _lib.ConvGeom(n, H, W, 8, 8, H, W, 3, 3, 1, 1, 0)
    a = _lib.WgradArgs(g, fdy.ptr(), fdy.cs, 64, fx.ptr(), None, 0, 0)
    assert _lib.load().stf_wgrad_kernel_name(ctypes.byref(a)).startswith(b"wgrad3x3_c8_kernel")
    out = torch.empty(64 * 8 * 9, device=DEV)
    nhwc.wgrad(fdy, fx, 3, 3, 1, 1, out)
    assert rel(out.view_as(w), w.grad) < 2e-3
    out2 = torch.empty_like(out)
    nhwc.wgrad(fdy, fx, 3, 3, 1, 1, out2)
    assert torch.equal(out, out2)              # fixed-order fold: repeatable bit for bit
