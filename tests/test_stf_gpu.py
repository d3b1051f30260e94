"""STF-LSTM-UNet parity on the GPU.

bf16 storage makes the whole-model STF gradient chaotic at initialisation: the
bf16-storage emulation of the fp32 oracle (oracle/stf_bf16.py) already moves the
logits by ~14 % and the parameter gradients by ~80 % (median), because the
error grows block by block through the 16 ResNet-34 blocks (layer4 output ~10 %
off).  So parity is proven per component, where bf16 errors stay at the 1e-2
level and a wrong kernel shows as O(1), and the whole model is checked for
wiring (shapes, loss, running-stat bookkeeping) against the reference fixture:

  component (block, LSTM, pools, packs) vs torch fp32 on bf16-rounded operands:
      outputs rel L2 <= 2e-2, gradients rel L2 <= 4e-2; BasicBlock gradients
      (an isolated block already moves 3-5 % under bf16 storage) within
      2 * err(bf16-storage emulation of the block) + 0.01
  whole model vs golden (tests/golden/stf_t4.npz, stf_pk_t4.npz):
      |loss - loss_ref| <= 0.03, logits rel L2 <= 2 * (bf16-emulation error) + 0.05
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def bfr(t):
    return t.to(torch.bfloat16).float()


def feat_from(x, cs=None, off=0):
    from stfunet.nhwc import Feat
    N, C, H, W = x.shape
    cs = cs or C
    buf = torch.zeros(N, H, W, cs, dtype=torch.bfloat16, device=DEV)
    buf[..., off:off + C] = x.permute(0, 2, 3, 1).to(torch.bfloat16)
    return Feat(buf.view(-1), N, H, W, C, cs, off)


class _Grads:
    def __init__(self, module):
        self.g = {id(p): torch.zeros_like(p) for p in module.parameters()}

    def __call__(self, p):
        return self.g[id(p)]


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


def _bf16_params(module):
    with torch.no_grad():
        for p in module.parameters():
            if p.dim() > 1:
                p.copy_(bfr(p))
        for mod in module.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.3, 0.3)


@pytest.mark.parametrize("cin,cout,stride,groups", [(64, 64, 1, 1), (64, 128, 2, 2), (128, 128, 1, 3)])
def test_basic_block_grouped_bn(cin, cout, stride, groups):
    """ResNet BasicBlock with per-time-step BN groups vs torch run per group."""
    import copy
    from stfunet import nhwc
    from stfunet.stf_lstm_unet import ResBlockProgram, _resnet_layer
    blk = _resnet_layer(cin, cout, 1, stride)[0].to(DEV)
    _bf16_params(blk)
    ref = copy.deepcopy(blk)
    blk_ref0 = copy.deepcopy(blk)
    B, H = 2, 16
    x = bfr(torch.randn(groups * B, cin, H, H, device=DEV))
    R = bfr(torch.randn(groups * B, cout, H // stride, H // stride, device=DEV))
    prog = ResBlockProgram(blk.conv1, blk.bn1, blk.conv2, blk.bn2,
                           blk.downsample[0] if blk.downsample is not None else None,
                           blk.downsample[1] if blk.downsample is not None else None)
    src = feat_from(x)
    out = nhwc.new_feat(groups * B, H // stride, H // stride, cout, DEV)
    s = prog.forward(src, out, True, groups)
    nhwc.flush_batches_tracked()                     # what the model programs do after forward
    gv = _Grads(blk)
    dsrc = prog.backward(s, gv, dout=feat_from(R))
    nhwc.flush_bn_grads()                            # grouped dgamma/dbeta, as the programs do
    # torch reference: one BN batch per group, running stats advanced per group in order
    xr = x.clone().requires_grad_(True)
    outs = []
    for g in range(groups):
        xg = xr[g * B:(g + 1) * B]
        y = F.relu(ref.bn1(ref.conv1(xg)))
        y = ref.bn2(ref.conv2(y))
        sc = ref.downsample(xg) if ref.downsample is not None else xg
        outs.append(F.relu(y + sc))
    o = torch.cat(outs)
    (o * R).sum().backward()
    # bf16-storage emulation of the same block: the gradient band (isolated blocks
    # already move 3-5 % under bf16 storage, measured)
    from oracle.unet_bf16 import q
    emu = copy.deepcopy(blk_ref0)
    xe = x.clone().requires_grad_(True)
    outs = []
    for g in range(groups):
        xg = xe[g * B:(g + 1) * B]
        y = q(F.relu(emu.bn1(q(F.conv2d(xg, emu.conv1.weight, stride=stride, padding=1)))))
        y = emu.bn2(q(F.conv2d(y, emu.conv2.weight, padding=1)))
        sc = emu.downsample[1](q(F.conv2d(xg, emu.downsample[0].weight, stride=stride))) \
            if emu.downsample is not None else xg
        outs.append(q(F.relu(y + sc)))
    (torch.cat(outs) * R).sum().backward()
    assert rel(out.dense(), o.detach()) < 2e-2
    assert rel(dsrc.dense(), xr.grad) <= 2 * rel(xe.grad, xr.grad) + 0.01
    for (name, p), (_, pr), (_, pe) in zip(blk.named_parameters(), ref.named_parameters(),
                                           emu.named_parameters()):
        assert rel(gv(p), pr.grad) <= 2 * rel(pe.grad, pr.grad) + 0.01, name
    for (name, b), (_, br) in zip(blk.named_buffers(), ref.named_buffers()):
        if "running" in name:
            assert rel(b, br) < 1e-2, name
        else:
            assert int(b) == int(br) == groups, name


@pytest.mark.parametrize("C,T", [(64, 3), (128, 2), (16, 3), (32, 2)])
def test_lstm_component(C, T):
    """Per-pixel nn.LSTM over T (only h_T used) vs torch nn.LSTM.  C = 16: a hidden size
    that fills only part of a GEMM tile's hidden channels (the staged epilogue's chunk
    bounds); stf_lstm_pack rejects sizes outside {16, 32, ..., 512}."""
    from stfunet import nhwc
    from stfunet.stf_lstm_unet import LSTMProgram
    lstm = torch.nn.LSTM(C, C, batch_first=True).to(DEV)
    with torch.no_grad():
        for p in lstm.parameters():
            p.copy_(bfr(p))
    B, H = 2, 4
    npix = B * H * H
    xs = bfr(torch.randn(T, npix, C, device=DEV))              # x_t per pixel, t-major
    lbuf = nhwc.zeros_feat(T * B, H, H, 2 * C, DEV)
    lbuf.buf.view(T, npix, 2 * C)[:, :, :C] = xs.to(torch.bfloat16)
    hT = nhwc.new_feat(B, H, H, C, DEV)
    prog = LSTMProgram(lstm)
    st = prog.forward(lbuf, T, B, hT)
    xr = xs.permute(1, 0, 2).contiguous().requires_grad_(True)   # [npix, T, C]
    out, _ = lstm(xr)
    h_ref = out[:, -1]
    assert rel(hT.buf.view(npix, C).float(), h_ref.detach()) < 2e-2
    dh = bfr(torch.randn(npix, C, device=DEV))
    h_ref.backward(dh)
    gv = _Grads(lstm)
    dhf = nhwc.new_feat(B, H, H, C, DEV)
    dhf.buf.view(npix, C).copy_(dh.to(torch.bfloat16))
    dx = prog.backward(st, dhf, gv)
    dx_t = dx.buf.view(T, npix, 2 * C)[:, :, :C].float()
    assert rel(dx_t, xr.grad.permute(1, 0, 2)) < 4e-2
    for name, p in lstm.named_parameters():
        assert rel(gv(p), p.grad) < 4e-2, name


def test_lstm_rejects_unsupported_hidden_size():
    from stfunet.stf_lstm_unet import LSTMProgram
    from stfunet import nhwc
    from stfunet._lib import HipError
    C = 48
    lstm = torch.nn.LSTM(C, C, batch_first=True).to(DEV)
    lbuf = nhwc.zeros_feat(2 * 2, 4, 4, 2 * C, DEV)
    with pytest.raises(HipError):
        LSTMProgram(lstm).forward(lbuf, 2, 2, nhwc.new_feat(2, 4, 4, C, DEV))


def test_maxpool3_fwd_bwd():
    """MaxPool2d(3,2,1) incl. ties (bf16 values repeat): the recorded first maximum
    must route the gradient exactly like torch."""
    from stfunet import nhwc
    from stfunet._lib import call, stream
    from stfunet.nhwc import _p
    x = bfr(torch.randn(2, 64, 15, 16, device=DEV))
    x[:, :8] = torch.round(x[:, :8])                       # many ties in the first channels
    xr = x.clone().requires_grad_(True)
    ref = F.max_pool2d(xr, 3, 2, 1)
    xf = feat_from(x)
    out = nhwc.new_feat(2, ref.shape[2], ref.shape[3], 64, DEV)
    arg = torch.empty(2 * ref.shape[2] * ref.shape[3] * 64, dtype=torch.uint8, device=DEV)
    call("stf_maxpool3s2_fwd", xf.ptr(), 2, 15, 16, 64, out.ptr(), _p(arg), stream())
    assert torch.equal(out.dense(), ref.detach())
    d = bfr(torch.randn_like(ref))
    ref.backward(d)
    dx = nhwc.new_feat(2, 15, 16, 64, DEV)
    call("stf_maxpool3s2_bwd", _p(arg), feat_from(d).ptr(), 2, 15, 16, 64, dx.ptr(), stream())
    assert rel(dx.dense(), xr.grad) < 1e-2


def test_pack_sequence_and_pk_resize():
    from stfunet import nhwc
    from stfunet._lib import call, stream
    from stfunet.nhwc import _p
    B, T, P, H, W = 2, 3, 3, 32, 32
    x = torch.randn(B, T + P, 1, H, W, device=DEV)
    out = nhwc.new_feat(T * B, H, W, 8, DEV)
    call("stf_pack_sequence", _p(x), B, T + P, 1, H, W, T, P, 8, out.ptr(), stream())
    got = out.dense().view(T, B, 8, H, W)
    for t in range(T):
        assert rel(got[t, :, 0], x[:, t, 0]) < 4e-3
        assert rel(got[t, :, 1:4], x[:, T:, 0]) < 4e-3
    assert got[:, :, 4:].abs().max().item() == 0
    dst = nhwc.zeros_feat(T * B, 8, 8, 72, DEV)
    call("stf_pk_resize", _p(x), B, T + P, T, P, H, W, 8, 8, dst.ptr(), 72, 64, stream())
    ref = F.interpolate(x[:, T:, 0], size=(8, 8), mode="bilinear", align_corners=True)
    d = dst.dense().view(T, B, 72, 8, 8)
    for t in range(T):
        assert rel(d[t, :, 64:67], ref) < 4e-3


@pytest.mark.parametrize("P", [0, 3])
def test_stem_im2col_gemm(P):
    """Stem conv 7x7/s2/p3 (src/stf_lstm_unet.py:108,177) as im2col + 1x1 GEMM:
    columns bit-exact vs F.unfold of the bf16-rounded input; conv output and
    weight gradient vs torch fp32 on bf16-rounded operands (rel L2 <= 1e-2)."""
    from stfunet import nhwc
    from stfunet._lib import call, stream
    from stfunet.nhwc import _p
    B, T, H, W = 2, 3, 40, 48
    cin = 1 + P
    kreal = cin * 49
    kpad = 64 if kreal <= 64 else (kreal + 31) // 32 * 32
    x = torch.randn(B, T + P, 1, H, W, device=DEV)
    ho, wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    cols = nhwc.new_feat(T * B, ho, wo, kpad, DEV)
    call("stf_stem_im2col", _p(x), B, T + P, 1, H, W, T, P, 7, 2, 3, kpad, cols.ptr(), stream())
    frames = torch.cat([torch.cat([x[:, t], x[:, T:, 0]], 1) for t in range(T)], 0)     # [T*B, cin, H, W]
    ref = F.unfold(bfr(frames), 7, padding=3, stride=2)                                  # [T*B, cin*49, ho*wo]
    got = cols.dense().flatten(2)
    assert torch.equal(got[:, :kreal].float(), ref)
    assert got[:, kreal:].abs().max().item() == 0
    w = torch.randn(64, cin, 7, 7, device=DEV) * 0.05
    y = nhwc.new_feat(T * B, ho, wo, 64, DEV)
    nhwc.igemm(cols, nhwc.pack_weight(w.view(64, -1, 1, 1), 0, kpad), 64, y, 1, 1, 1, 0)
    yr = F.conv2d(bfr(frames), bfr(w), stride=2, padding=3)
    assert rel(y.dense(), yr) < 1e-2
    dy = bfr(torch.randn_like(yr))
    dw = torch.empty(64 * kpad, device=DEV)
    nhwc.wgrad(feat_from(dy), cols, 1, 1, 1, 0, dw)
    wr = bfr(w).requires_grad_(True)
    F.conv2d(bfr(frames), wr, stride=2, padding=3).backward(dy)
    assert rel(dw.view(64, kpad)[:, :kreal].view(64, cin, 7, 7), wr.grad) < 1e-2


@pytest.mark.parametrize("P", [3, 1])
def test_stem_pk_gather_path(P):
    """The PK-map stem (src/stf_lstm_unet.py:105,172-177 with use_pk_maps: Cin = 1 + P):
    stf_pack_sequence packs frame t and the P maps into 8 zero-padded channels, the 7x7/s2/p3
    conv runs as an 8-channel tap-gather igemm, and its weight gradient as a 7x7/s2/p3 wgrad
    on Cs = 8 (STFProgram's stem_gather path, the one cfg5 trains through).  Packed input
    bit-exact; conv output and the real 1 + P weight-gradient columns vs F.conv2d autograd on
    bf16-rounded operands (rel L2 <= 1e-2); the padded columns' gradient is exactly 0."""
    from stfunet import nhwc
    from stfunet._lib import call, stream
    from stfunet.nhwc import _p
    B, T, H, W = 2, 3, 40, 48
    cin = 1 + P
    torch.manual_seed(P)
    x = torch.randn(B, T + P, 1, H, W, device=DEV)
    xin = nhwc.new_feat(T * B, H, W, 8, DEV)
    call("stf_pack_sequence", _p(x), B, T + P, 1, H, W, T, P, 8, xin.ptr(), stream())
    frames = torch.cat([torch.cat([x[:, t], x[:, T:, 0]], 1) for t in range(T)], 0)     # [T*B, cin, H, W]
    got = xin.dense()
    assert torch.equal(got[:, :cin].float(), bfr(frames))
    assert got[:, cin:].abs().max().item() == 0
    w = torch.randn(64, cin, 7, 7, device=DEV) * 0.05
    ho, wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y = nhwc.new_feat(T * B, ho, wo, 64, DEV)
    nhwc.igemm(xin, nhwc.pack_weight(w, 0, 8), 64, y, 7, 7, 2, 3)
    yr = F.conv2d(bfr(frames), bfr(w), stride=2, padding=3)
    assert rel(y.dense(), yr) < 1e-2
    dy = bfr(torch.randn_like(yr))
    tmp = torch.empty(64 * 8 * 49, device=DEV)
    nhwc.wgrad(feat_from(dy), xin, 7, 7, 2, 3, tmp, defer=False)
    wr = bfr(w).requires_grad_(True)
    F.conv2d(bfr(frames), wr, stride=2, padding=3).backward(dy)
    dw = tmp.view(64, 8, 7, 7)
    assert rel(dw[:, :cin], wr.grad) < 1e-2
    assert dw[:, cin:].abs().max().item() == 0


@pytest.mark.parametrize("pk", [False, True])
def test_stf_model_vs_golden(pk):
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet
    from stfunet.loss import criterion
    g = np.load(os.path.join(GOLDEN, "stf_pk_t4.npz" if pk else "stf_t4.npz"))
    m = STFLSTMUNet(use_pk_maps=pk, time_steps=4)
    m.load_state_dict(canonical_state_dict(m.state_dict(), seed=0))
    m = m.to(DEV).train()
    x, t = torch.from_numpy(g["x"]), torch.from_numpy(g["target"])
    out = m(x.to(DEV))["out"]
    assert out.shape == g["logits"].shape                   # H/2 x W/2, like the reference
    loss = criterion({"out": out}, t.to(DEV))
    loss.backward()
    assert abs(loss.item() - float(g["loss"])) < 0.03
    emu = 0.14 if not pk else 0.19                          # measured bf16-emulation logits error
    assert rel(out.detach(), torch.from_numpy(g["logits"])) < 2 * emu + 0.05
    T = 4
    for k, v in m.state_dict().items():
        if k.endswith("num_batches_tracked"):
            enc = k.startswith(("bn1.", "layer"))
            assert int(v) == (T if enc else 1), k
    for k, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), k


def test_stf_eval_mode_vs_oracle():
    """Whole-model STF forward in eval mode (running statistics) vs the fp32 oracle.
    Training-mode BatchNorm amplifies 16-bit rounding ~30x in this net (pre-BN conv
    outputs carry a large per-channel offset relative to their spread, see DESIGN.md
    "Parity"); with fixed statistics the bf16 emulation stays at ~1e-3, so every forward
    kernel of the model (stem, ResNet blocks, LSTMs, decoder, head) is checked tightly
    here: logits within 2x the emulation's error + 2e-3."""
    import oracle.unet_bf16 as o_q
    from oracle import stf as o_stf, stf_bf16 as o_emu
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet
    g = np.load(os.path.join(GOLDEN, "stf_t4.npz"))
    m = STFLSTMUNet(time_steps=4)
    sd = canonical_state_dict(m.state_dict(), seed=0)
    gen = torch.Generator().manual_seed(3)
    for k, v in sd.items():
        if "running_mean" in k:
            sd[k] = torch.rand(v.shape, generator=gen) * 0.2 - 0.1
        if "running_var" in k:
            sd[k] = torch.rand(v.shape, generator=gen) * 0.5 + 0.75
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        out = m(x.to(DEV))["out"]
        ref = o_stf.forward(sd, x, False)["out"]
        with o_q.storage(torch.bfloat16):
            emu = o_emu.forward(sd, x, False)["out"]
    e_emu = rel(emu, ref)
    assert rel(out, ref) <= 2 * e_emu + 2e-3, (rel(out, ref), e_emu)
    for k, v in m.state_dict().items():                     # eval never moves the statistics
        assert torch.equal(v.cpu(), sd[k]), k


@pytest.mark.parametrize("T,B,H", [(5, 3, 6), (1, 2, 8), (8, 16, 8)])
def test_lstm_whole_sequence_equals_per_step(monkeypatch, T, B, H):
    """stf_lstm_seq_fwd / _bwd (C = 64: all T steps in one launch, 64 pixels per
    workgroup, ragged last workgroup when B*H*H % 64 != 0) produce bit for bit the
    per-step launches' h_T, cell states, [x | h] rows, input and weight gradients."""
    from stfunet import nhwc
    from stfunet.stf_lstm_unet import LSTMProgram
    C = 64
    lstm = torch.nn.LSTM(C, C, batch_first=True).to(DEV)
    lbuf = nhwc.zeros_feat(T * B, H, H, 2 * C, DEV)
    lbuf.buf.view(-1, 2 * C)[:, :C].normal_()
    dhT = nhwc.new_feat(B, H, H, 3 * C, DEV).slice(C, C)       # strided h_T gradient (decoder slice)
    dhT.buf.normal_()
    prog = LSTMProgram(lstm)
    out = {}
    monkeypatch.setenv("STF_LSTM_HOIST", "0")            # per-step [dx | dh] like the sequence kernel
    for mode in ("0", "1"):
        monkeypatch.setenv("STF_LSTM_SEQ", mode)
        hT = nhwc.new_feat(B, H, H, 2 * C, DEV).slice(0, C)
        st = prog.forward(lbuf, T, B, hT)
        assert st.fused == (mode == "1")
        gv = _Grads(lstm)
        dx = prog.backward(st, dhT, gv)
        out[mode] = [hT.dense(), st.c, lbuf.buf.clone(), dx.dense()] + [gv(p).clone() for p in lstm.parameters()]
    for a, b in zip(out["0"], out["1"]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("C,T,B,H", [(128, 5, 3, 6), (256, 3, 2, 8), (512, 4, 16, 8), (128, 8, 16, 32)])
def test_lstm_coop_forward_equals_per_step(monkeypatch, C, T, B, H):
    """stf_lstm_coop_fwd (C = 128 / 256 / 512: one persistent launch, the C/32 workgroups of a
    64-pixel block exchanging h_t in-launch; ragged last block when B*H*H % 64 != 0; (512, 4,
    16, 8) and (128, 8, 16, 32) are lstm4 / lstm2 of cfg3) gives bit for bit the per-step
    launches' h_T, cell states and [x | h] rows, and no hand-off timed out.  The cooperative
    backward (stf_lstm_coop_bwd: the forward's gates, dgates and [dx | dh] exchanged in-launch)
    gives the per-step backward's input and weight gradients: bit for bit where the per-step
    dgates x W GEMM runs unsplit (lstm2 at cfg3), else within rel 2e-3 (small pixel counts split
    that GEMM over K: a different fp32 summation order before the 16-bit rounding).  Mode "g":
    cooperative forward, per-step backward from the forward's stored gates (cell backward +
    [dx | dh] GEMM, no gate recompute): bit for bit the per-step path everywhere."""
    from stfunet import nhwc
    from stfunet.stf_lstm_unet import LSTMProgram
    lstm = torch.nn.LSTM(C, C, batch_first=True).to(DEV)
    lbuf = nhwc.zeros_feat(T * B, H, H, 2 * C, DEV)
    lbuf.buf.view(-1, 2 * C)[:, :C].normal_()
    dhT = nhwc.new_feat(B, H, H, 3 * C, DEV).slice(C, C)
    dhT.buf.normal_()
    prog = LSTMProgram(lstm)
    out = {}
    monkeypatch.setenv("STF_LSTM_HOIST", "0")            # per-step [dx | dh] like the cooperative backward
    for mode in ("0", "1", "g"):
        monkeypatch.setenv("STF_LSTM_COOP", "0" if mode == "0" else "1")
        monkeypatch.setenv("STF_LSTM_COOP_BWD", "1" if mode == "1" else "0")
        lb = nhwc.zeros_feat(T * B, H, H, 2 * C, DEV)
        lb.buf.copy_(lbuf.buf)
        hT = nhwc.new_feat(B, H, H, 2 * C, DEV).slice(0, C)
        st = prog.forward(lb, T, B, hT)
        if mode != "0":
            assert (st.coop == (mode == "1")) and st.gates is not None and prog.coop_error() == 0
        gv = _Grads(lstm)
        dx = prog.backward(st, dhT, gv)
        if mode == "1":
            assert prog.coop_error() == 0
        out[mode] = [hT.dense(), st.c, lb.buf.clone(), dx.dense()] + [gv(p).clone() for p in lstm.parameters()]
    for i, (a, b) in enumerate(zip(out["0"], out["g"])):
        assert torch.equal(a, b), i
    for i, (a, b) in enumerate(zip(out["0"], out["1"])):
        if i < 3:                                   # forward: always bitwise
            dd = (a.float() - b.float()).abs()
            assert torch.equal(a, b), (i, int((dd > 0).sum()), dd.max().item(), a.shape,
                                       torch.nonzero(dd.reshape(-1) > 0)[:8].flatten().tolist())
        else:
            e = ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()
            unsplit = (C, B * H * H) == (128, 16 * 32 * 32)      # lstm2 at cfg3: per-step GEMM not split
            assert torch.equal(a, b) or (not unsplit and e < 2e-3), (i, e)


def test_stf_model_with_cooperative_lstms_matches_per_step(monkeypatch):
    """The whole STF training step with every LSTM on the cooperative kernels (forward and
    backward, STF_LSTM_COOP=1, STF_LSTM_COOP_BWD=1) against the same step on the per-step
    launches: logits and loss bit for bit (the forward is); the decoder's gradients bit for bit
    (its backward runs before any LSTM's); the LSTMs' within rel 1e-2 (the per-step dgates x W
    GEMMs split over K at these small sizes); the encoder's -- downstream of the LSTMs' d x_t,
    through 36 train-mode BatchNorms at initialisation, which amplify any perturbation (DESIGN.md
    section 4: the fp32 oracle's gradients move 2.3 % for a 1e-6 input change) -- within rel 5e-2,
    median over them 1e-2."""
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet
    from stfunet.loss import criterion
    g = np.load(os.path.join(GOLDEN, "stf_t4.npz"))
    x, t = torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["target"]).to(DEV)
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("STF_LSTM_COOP", mode)
        monkeypatch.setenv("STF_LSTM_COOP_BWD", mode)
        m = STFLSTMUNet(time_steps=4)
        m.load_state_dict(canonical_state_dict(m.state_dict(), seed=0))
        m = m.to(DEV).train()
        out = m(x)["out"]
        loss = criterion({"out": out}, t)
        loss.backward()
        res[mode] = (out.detach(), loss.item(), {k: p.grad.detach().clone() for k, p in m.named_parameters()})
    assert torch.equal(res["0"][0], res["1"][0]) and res["0"][1] == res["1"][1]
    enc = []
    for k, g0 in res["0"][2].items():
        e = rel(res["1"][2][k], g0)
        if k.startswith(("decoder", "upconv1", "final")):
            assert torch.equal(res["1"][2][k], g0), k
        elif k.startswith("lstm"):
            assert e < 1e-2, (k, e)
        else:
            assert e < 5e-2, (k, e)
            enc.append(e)
    assert float(np.median(enc)) < 1e-2, np.median(enc)


def test_stf_eval_mode_backward_vs_oracle():
    """Whole-model STF backward in eval mode (BatchNorm with running statistics) vs autograd
    of the fp32 oracle: with constant statistics the bf16 error stays small, so the
    gradients are compared directly (within 2x the bf16 emulation's error + 0.02)."""
    import oracle.unet_bf16 as o_q
    from oracle import loss as o_loss, stf as o_stf, stf_bf16 as o_emu
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet
    from stfunet.loss import criterion
    g = np.load(os.path.join(GOLDEN, "stf_t4.npz"))
    m = STFLSTMUNet(time_steps=4)
    sd = canonical_state_dict(m.state_dict(), seed=0)
    gen = torch.Generator().manual_seed(3)
    for k, v in sd.items():
        if "running_mean" in k:
            sd[k] = torch.rand(v.shape, generator=gen) * 0.2 - 0.1
        if "running_var" in k:
            sd[k] = torch.rand(v.shape, generator=gen) * 0.5 + 0.75
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    x, t = torch.from_numpy(g["x"]), torch.from_numpy(g["target"])
    p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    o_loss.criterion(o_stf.forward(p, x, False)["out"], t).backward()
    pe = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    with o_q.storage(torch.bfloat16):
        o_loss.criterion(o_emu.forward(pe, x, False)["out"], t).backward()
    criterion({"out": m(x.to(DEV))["out"]}, t.to(DEV)).backward()
    bad = []
    for k, prm in m.named_parameters():
        e_hip, e_emu = rel(prm.grad, p[k].grad), rel(pe[k].grad, p[k].grad)
        if e_hip > 2 * e_emu + 0.02:
            bad.append((k, e_hip, e_emu))
    assert not bad, bad


@pytest.mark.parametrize("train", [False, True])
def test_stf_input_gradient_vs_oracle(train):
    """x.requires_grad: the input sequence's gradient (reference autograd returns it,
    src/stf_lstm_unet.py:139-256) -- the eager forward, then the stem's stf_stem_dgrad7 after the
    backward -- vs autograd of the fp32 oracle in eval and in training mode (within 2x the bf16
    emulation's error + 0.02, as the parameter gradients above); the parameter gradients and, in
    training mode, the BatchNorm running statistics and num_batches_tracked are those of the plain
    call (the eager forward advances them exactly once); N such backwards leave the weight-pack
    cache at a constant size (no per-call temporaries cached)."""
    import oracle.unet_bf16 as o_q
    from oracle import loss as o_loss, stf as o_stf, stf_bf16 as o_emu
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet
    from stfunet.loss import criterion
    g = np.load(os.path.join(GOLDEN, "stf_t4.npz"))
    m = STFLSTMUNet(time_steps=4)
    sd = canonical_state_dict(m.state_dict(), seed=0)
    m.load_state_dict(sd)
    m = m.to(DEV).train(train)
    x, t = torch.from_numpy(g["x"]), torch.from_numpy(g["target"])
    p = {k: v.clone() for k, v in sd.items()}
    xo = x.clone().requires_grad_(True)
    o_loss.criterion(o_stf.forward(p, xo, train)["out"], t).backward()
    xe = x.clone().requires_grad_(True)
    with o_q.storage(torch.bfloat16):
        o_loss.criterion(o_emu.forward(p, xe, train)["out"], t).backward()
    xh = x.to(DEV).requires_grad_(True)
    criterion({"out": m(xh)["out"]}, t.to(DEV)).backward()
    assert xh.grad is not None and xh.grad.shape == x.shape and torch.isfinite(xh.grad).all()
    e_hip, e_emu = rel(xh.grad, xo.grad), rel(xe.grad, xo.grad)
    assert e_hip < 2 * e_emu + 0.02, (e_hip, e_emu)
    grads = {k: v.grad.clone() for k, v in m.named_parameters()}
    bufs = {k: v.clone() for k, v in m.state_dict().items() if "running" in k or "num_batches" in k}
    m.load_state_dict(sd)
    m.zero_grad(set_to_none=True)
    criterion({"out": m(x.to(DEV))["out"]}, t.to(DEV)).backward()      # the planned path, no input grad
    for k, v in m.named_parameters():
        assert torch.equal(v.grad, grads[k]), k
    for k, v in m.state_dict().items():
        if k in bufs:
            assert torch.equal(v, bufs[k]), k
    n_packs = None
    for _ in range(3):
        m.zero_grad(set_to_none=True)
        xh = x.to(DEV).requires_grad_(True)
        criterion({"out": m(xh)["out"]}, t.to(DEV)).backward()
        n = len(m.program.packs.bufs)
        assert n_packs is None or n == n_packs, (n, n_packs)
        n_packs = n


@pytest.mark.parametrize("train", [False, True])
def test_stf_input_gradient_pk_vs_oracle(train):
    """The same with PK maps on the T axis (x [B, T + 3, 1, H, W]): the frames' gradient from the
    stem, the PK maps' from the stem (every frame reads them) plus the four fusion branches through
    the bilinear resize's backward, summed over the frames -- vs autograd of the fp32 oracle, eval
    and training mode; the fusion branches' zero-padded dgrad weights are per-call temporaries that
    must not accumulate in the weight-pack cache."""
    import oracle.unet_bf16 as o_q
    from oracle import loss as o_loss, stf as o_stf, stf_bf16 as o_emu
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet
    from stfunet.loss import criterion
    m = STFLSTMUNet(time_steps=3, use_pk_maps=True)
    sd = canonical_state_dict(m.state_dict(), seed=1)
    m.load_state_dict(sd)
    m = m.to(DEV).train(train)
    gen = torch.Generator().manual_seed(5)
    x = torch.rand(2, 6, 1, 96, 64, generator=gen)
    t = torch.randint(0, 2, (2, 48, 32), generator=gen)
    p = {k: v.clone() for k, v in sd.items()}
    xo = x.clone().requires_grad_(True)
    o_loss.criterion(o_stf.forward(p, xo, train, use_pk_maps=True)["out"], t).backward()
    xe = x.clone().requires_grad_(True)
    with o_q.storage(torch.bfloat16):
        o_loss.criterion(o_emu.forward(p, xe, train, use_pk_maps=True)["out"], t).backward()
    xh = x.to(DEV).requires_grad_(True)
    criterion({"out": m(xh)["out"]}, t.to(DEV)).backward()
    assert xh.grad is not None and xh.grad.shape == x.shape and torch.isfinite(xh.grad).all()
    for sl in (slice(0, 3), slice(3, 6)):                  # frames, PK maps
        e_hip, e_emu = rel(xh.grad[:, sl], xo.grad[:, sl]), rel(xe.grad[:, sl], xo.grad[:, sl])
        assert e_hip < 2 * e_emu + 0.02, (sl, e_hip, e_emu)
    n_packs = None
    for _ in range(3):
        m.zero_grad(set_to_none=True)
        xh = x.to(DEV).requires_grad_(True)
        criterion({"out": m(xh)["out"]}, t.to(DEV)).backward()
        n = len(m.program.packs.bufs)
        assert n_packs is None or n == n_packs, (n, n_packs)
        n_packs = n


@pytest.mark.parametrize("B,T,Cf,H,W", [(2, 3, 1, 45, 38), (1, 2, 3, 64, 33), (1, 1, 6, 32, 32)])
def test_stem_dgrad7_vs_torch(B, T, Cf, H, W):
    """stf_stem_dgrad7 (the stem conv's input gradient, parity-class workgroups, fp32 weights)
    vs torch's conv2d input gradient in fp32 on the same 16-bit dy (odd sizes: ragged tiles and
    partial tap sets at the borders; 6 channels: two channel passes)."""
    from stfunet import _lib
    from stfunet._lib import call, stream
    from stfunet.nhwc import _p
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    w = torch.randn(64, Cf, 7, 7, device=DEV) / (Cf * 49) ** 0.5
    dy = torch.randn(T * B, 64, Ho, Wo, device=DEV).to(_lib.storage_dtype())
    dyf = dy.float()
    ref = torch.nn.grad.conv2d_input((T * B, Cf, H, W), w, dyf, stride=2, padding=3)     # [t*B + b]
    ref = ref.view(T, B, Cf, H, W).transpose(0, 1)
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    dx = torch.full((B, T, Cf, H, W), float("nan"), device=DEV)
    call("stf_stem_dgrad7", _p(dyn), _p(w), B, T, Cf, H, W, T, _p(dx), stream())
    torch.cuda.synchronize()
    assert rel(dx, ref) < 1e-5


def test_stem_bn_act_maxpool_fused_equals_two_passes():
    """stf_bn_act_maxpool3s2 (the stem's BN + ReLU inside its MaxPool(3,2,1)) gives the pooled
    output and the window argmax of stf_bn_act followed by stf_maxpool3s2_fwd bit for bit
    (odd sizes: partial windows at the border; 3 statistics groups; ties from the ReLU zeros)."""
    from stfunet import nhwc
    from stfunet._lib import call, stream
    from stfunet.nhwc import BNState, _p
    N, H, W, C, G = 6, 21, 18, 64, 3
    y = nhwc.new_feat(N, H, W, C, DEV)
    y.buf.normal_()
    st = BNState(C, DEV, N * H * W, G)
    st.scale.uniform_(0.5, 1.5)
    st.shift.uniform_(-0.5, 0.5)
    a = nhwc.new_feat(N, H, W, C, DEV)
    nhwc.bn_act(y, st, a)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    p_ref = torch.empty(N * Ho * Wo * C, dtype=torch.bfloat16, device=DEV)
    arg_ref = torch.empty(N * Ho * Wo * C, dtype=torch.uint8, device=DEV)
    call("stf_maxpool3s2_fwd", a.ptr(), N, H, W, C, _p(p_ref), _p(arg_ref), stream())
    p = torch.empty_like(p_ref)
    arg = torch.empty_like(arg_ref)
    call("stf_bn_act_maxpool3s2", y.ptr(), N, H, W, C, G, _p(st.scale), _p(st.shift), _p(p), _p(arg), stream())
    torch.cuda.synchronize()
    assert torch.equal(p.view(torch.int16), p_ref.view(torch.int16))
    assert torch.equal(arg, arg_ref)


def test_stem_bn_backward_through_maxpool():
    """nhwc.bn_backward_maxpool3 (the pooled gradient routed by the argmax inside the BN
    backward's reduce and apply: stf_bn_bwd_*_pool3) against stf_maxpool3s2_bwd + the
    mask-recomputing nhwc.bn_backward it replaces: dy within bf16 rounding (the partial sums
    are added in another order), dgamma / dbeta within 1e-4 relative."""
    from stfunet import nhwc
    from stfunet._lib import call, stream
    from stfunet.nhwc import BNState, _p
    N, H, W, C, G = 8, 34, 29, 64, 4
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y = nhwc.new_feat(N, H, W, C, DEV)
    y.buf.normal_()
    st = BNState(C, DEV, N * H * W, G)
    st.scale.uniform_(0.5, 1.5)
    st.shift.uniform_(-0.5, 0.5)
    st.mean.normal_(0, 0.1)
    st.invstd.uniform_(0.8, 1.2)
    p0 = nhwc.new_feat(N, Ho, Wo, C, DEV)
    arg = torch.empty(N * Ho * Wo * C, dtype=torch.uint8, device=DEV)
    call("stf_bn_act_maxpool3s2", y.ptr(), N, H, W, C, G, _p(st.scale), _p(st.shift), p0.ptr(), _p(arg), stream())
    dpool = nhwc.new_feat(N, Ho, Wo, C, DEV)
    dpool.buf.normal_()
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    res = {}
    for mode in ("old", "new"):
        dg = torch.zeros(C, device=DEV)
        db = torch.zeros(C, device=DEV)
        if mode == "old":
            da = nhwc.new_feat(N, H, W, C, DEV)
            call("stf_maxpool3s2_bwd", _p(arg), dpool.ptr(), N, H, W, C, da.ptr(), stream())
            dy = nhwc.bn_backward(y, st, bn, dg, db, dz=da)
        else:
            dy = nhwc.bn_backward_maxpool3(y, st, bn, dg, db, arg, dpool)
        nhwc.flush_bn_grads()
        res[mode] = (dy.dense(), dg.clone(), db.clone())
    torch.cuda.synchronize()
    assert rel(res["new"][0], res["old"][0]) < 5e-3
    assert rel(res["new"][1], res["old"][1]) < 1e-4 and rel(res["new"][2], res["old"][2]) < 1e-4


def test_lstm_coop_timeout_raises(monkeypatch):
    """A cooperative LSTM launch whose in-launch hand-off times out must not pass silently
    (VERDICT r03 weak #6): the kernel sets its error word and drains, the launch ORs it into the
    program's sticky device flag, and the next step boundary (forward) -- or the epoch's end,
    block=True -- raises RuntimeError.  Forced with spin_limit 0xFFFFFFFF (every hand-off reports
    a timeout at once); a normal step with the default limit never raises."""
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet
    from stfunet.loss import criterion
    monkeypatch.setenv("STF_LSTM_COOP", "512")
    g = np.load(os.path.join(GOLDEN, "stf_t4.npz"))
    x, t = torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["target"]).to(DEV)
    m = STFLSTMUNet(time_steps=4)
    m.load_state_dict(canonical_state_dict(m.state_dict(), seed=0))
    m = m.to(DEV).train()
    for _ in range(2):
        criterion(m(x), t).backward()
    m.program.check_device_errors(block=True)                  # default limit: no timeout
    lp = m.program.lstm_progs[3]
    lp.spin_limit = 0xFFFFFFFF
    out = m(x)
    assert lp.coop_error() != 0                                 # the launch saw its hand-offs fail
    criterion(out, t).backward()
    lp.spin_limit = 0
    with pytest.raises(RuntimeError, match="cooperative LSTM"):
        m.program.check_device_errors(block=True)
    m.program.check_device_errors(block=True)                  # flag cleared after the raise
    lp.spin_limit = 0xFFFFFFFF
    m(x)
    lp.spin_limit = 0
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="cooperative LSTM"):
        for _ in range(2):                                      # the copy issued at the boundary
            m(x)                                                # lands; a later boundary raises
            torch.cuda.synchronize()


@pytest.mark.parametrize("H,W,h,w", [(14, 18, 13, 17), (6, 8, 5, 7), (7, 9, 13, 17), (1, 4, 3, 1)])
def test_bilinear_align_corners_kernels(H, W, h, w):
    """stf_bilinear_ac_fwd / _bwd (the DecoderBlock size fallback, src/stf_lstm_unet.py:56-57)
    against F.interpolate(mode="bilinear", align_corners=True) and its autograd on the bf16 values
    in fp32: down- and up-sizing, ragged sizes, a size-1 side; strided NHWC slices as in the
    decoder (the output is the concat buffer's first channels).  bf16 outputs: rel-L2 <= 1e-2,
    and the 16-bit rounding of each output is the only difference (max abs <= 1 bf16 ulp-ish)."""
    from stfunet import _lib, nhwc
    N, C = 3, 64
    x = nhwc.new_feat(N, H, W, C + 8, DEV).slice(8, C)
    x.buf.normal_()
    y = nhwc.new_feat(N, h, w, 2 * C, DEV).slice(0, C)
    _lib.call("stf_bilinear_ac_fwd", x.ptr(), N, H, W, C, x.cs, y.ptr(), h, w, y.cs, _lib.stream())
    xr = x.dense().contiguous().requires_grad_(True)                  # dense(): [N, C, H, W] fp32
    ref = F.interpolate(xr, size=(h, w), mode="bilinear", align_corners=True)
    got = y.dense()
    assert rel(got, ref) <= 1e-2, rel(got, ref)
    assert (got - ref.to(torch.bfloat16).float()).abs().max().item() <= 2e-2 * ref.abs().max().item()
    dy = nhwc.new_feat(N, h, w, C + 16, DEV).slice(16, C)
    dy.buf.normal_()
    dx = nhwc.new_feat(N, H, W, C, DEV)
    _lib.call("stf_bilinear_ac_bwd", dy.ptr(), N, h, w, C, dy.cs, dx.ptr(), H, W, dx.cs, _lib.stream())
    ref.backward(dy.dense())
    gdx = dx.dense()
    assert rel(gdx, xr.grad) <= 1e-2, rel(gdx, xr.grad)


def test_stf_size_fallback_vs_oracle():
    """H, W not divisible by 32 (72 x 104: layer4 is 3 x 4, so decoder4 and decoder3 resize their
    transposed-conv outputs 6x8 -> 5x7 and 10x14 -> 9x13 to the skips; src/stf_lstm_unet.py:56-57):
    whole-model logits in eval mode (fixed running statistics) within 2x the bf16 emulation's error
    + 2e-3 of the fp32 restatement, and every parameter gradient of an eval-mode backward within 2x
    the emulation's error + 0.02 (as test_stf_fullsize_eval_backward_vs_fp32)."""
    import oracle.unet_bf16 as o_q
    from oracle import loss as o_loss, stf as o_stf, stf_bf16 as o_emu
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet
    from stfunet.loss import criterion
    from stfunet.synthetic import dce_batch
    m = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=3)
    sd = canonical_state_dict(m.state_dict(), seed=0)
    gen = torch.Generator().manual_seed(5)
    for k, v in sd.items():
        if "running_mean" in k:
            sd[k] = torch.rand(v.shape, generator=gen) * 0.2 - 0.1
        if "running_var" in k:
            sd[k] = torch.rand(v.shape, generator=gen) * 0.5 + 0.75
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    sd = {k: v.to(DEV) for k, v in sd.items()}
    x, t = dce_batch(2, 3, 72, 104, seed=12, device=DEV, mask_hw=(36, 52))
    p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    ref = o_stf.forward(p, x, False)["out"]
    ref_loss = o_loss.criterion(ref, t)
    ref_loss.backward()
    pe = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    with o_q.storage(torch.bfloat16):
        emu = o_emu.forward(pe, x, False)["out"]
        o_loss.criterion(emu, t).backward()
    out = m(x)["out"]
    assert out.shape == ref.shape == (2, 2, 36, 52)
    e_hip, e_emu = rel(out, ref), rel(emu, ref)
    assert e_hip <= 2 * e_emu + 2e-3, (e_hip, e_emu)
    loss = criterion({"out": out}, t)
    loss.backward()
    assert abs(loss.item() - ref_loss.item()) < 1e-2, (loss.item(), ref_loss.item())
    bad = []
    for k, prm in m.named_parameters():
        eh, ee = rel(prm.grad, p[k].grad), rel(pe[k].grad, p[k].grad)
        if eh > 2 * ee + 0.02:
            bad.append((k, eh, ee))
    print(f"\nSTF 72x104 (size fallback): logits rel {e_hip:.3e} (emu {e_emu:.3e}), loss {loss.item():.6f} vs "
          f"{ref_loss.item():.6f}")
    assert not bad, bad


def test_stf_size_fallback_train_vs_reference():
    """Training mode at 72 x 104 (train-mode BatchNorm at the odd sizes 18x26 / 9x13 / 5x7 / 3x4, the
    bilinear size fallback in decoder4 / decoder3) on the input of the REFERENCE's own run
    (tests/golden/stf_t3_72x104.npz, make_golden.py gen_stf_size_fallback):
      the fp32 restatement, run here on the GPU, reproduces the fixture (logits rel 1e-4, loss 1e-5,
          every gradient's abs-sum checksum 2e-3: the CPU test's pins, re-checked on this device);
      the HIP path against it with the full-size train-mode rule (test_stf_fullsize_train_vs_fp32):
          logits <= 1.3 x the bf16 emulation's error + 0.01, loss within 0.03, every parameter gradient
          within 2 x the emulation's error + 0.03.  (The reference's own bf16-autocast step is not run
          here: MIOpen's bf16 batch norm crashes the process at these odd sizes.)"""
    import oracle.unet_bf16 as o_q
    from oracle import loss as o_loss, stf as o_stf, stf_bf16 as o_emu
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet
    from stfunet.loss import criterion
    g = np.load(os.path.join(GOLDEN, "stf_t3_72x104.npz"))
    m = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=3)
    sd = canonical_state_dict(m.state_dict(), seed=0)
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    sd = {k: v.to(DEV) for k, v in sd.items()}
    x, t = torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["target"]).to(DEV)

    def params():
        return {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    p, pe = params(), params()
    ref = o_stf.forward(p, x, True)["out"]
    ref_loss = o_loss.criterion(ref, t)
    ref_loss.backward()
    # the restatement on this device against the reference's own run
    assert rel(ref, torch.from_numpy(g["logits"])) < 1e-4
    assert abs(ref_loss.item() - float(g["loss"])) < 1e-5
    for k in g.files:
        if k.startswith("gradck."):
            ck = float(g[k][1])
            got = p[k[7:]].grad.double().abs().sum().item()
            assert abs(got - ck) <= 2e-3 * abs(ck) + 1e-6 * p[k[7:]].numel(), k
    with o_q.storage(torch.bfloat16):
        emu = o_emu.forward(pe, x, True)["out"]
        o_loss.criterion(emu, t).backward()
    out = m(x)["out"]
    loss = criterion({"out": out}, t)
    loss.backward()
    assert out.shape == ref.shape == (1, 2, 36, 52)
    e_hip, e_emu = rel(out, ref), rel(emu, ref)
    bad, errs = [], []
    for k, prm in m.named_parameters():
        eh, ee = rel(prm.grad, p[k].grad), rel(pe[k].grad, p[k].grad)
        errs.append(eh)
        if eh > 2 * ee + 0.03:
            bad.append((k, eh, ee))
    errs.sort()
    print(f"\nSTF 72x104 train: logits rel {e_hip:.3e} (emu {e_emu:.3e}), loss {loss.item():.6f} vs "
          f"{ref_loss.item():.6f}; gradient rel median {errs[len(errs) // 2]:.3e}")
    assert e_hip <= 1.3 * e_emu + 0.01, (e_hip, e_emu)
    assert abs(loss.item() - ref_loss.item()) < 0.03
    assert not bad, bad


@pytest.mark.parametrize("C,T,B,H", [(64, 5, 3, 6), (128, 8, 16, 32), (256, 8, 16, 16), (512, 8, 16, 8)])
@pytest.mark.parametrize("gates", [False, True])
def test_lstm_hoisted_input_projection(monkeypatch, C, T, B, H, gates):
    """BPTT with the input projection hoisted out of the recurrence (STF_LSTM_HOIST, the default:
    per step only dh_{t-1} = dgates_t W_hh, then d x for all T steps as ONE GEMM)
    against the per-step [dx | dh] GEMM: dgates, the weight / bias gradients and d x within rel
    2e-3 (bitwise where both GEMMs run unsplit: only the split-K choice of the narrower per-step
    GEMM can change a summation order).  cfg3's lstm2 / lstm3 / lstm4 shapes, both cell-backward
    sources (gate recompute; the cooperative forward's stored gates)."""
    from stfunet import nhwc
    from stfunet.stf_lstm_unet import LSTMProgram
    monkeypatch.setenv("STF_LSTM_SEQ", "0")
    monkeypatch.setenv("STF_LSTM_COOP", "1" if gates else "0")
    monkeypatch.setenv("STF_LSTM_COOP_BWD", "0")
    if gates and C == 64:
        pytest.skip("no cooperative forward at C = 64")
    lstm = torch.nn.LSTM(C, C, batch_first=True).to(DEV)
    lbuf = nhwc.zeros_feat(T * B, H, H, 2 * C, DEV)
    lbuf.buf.view(-1, 2 * C)[:, :C].normal_()
    dhT = nhwc.new_feat(B, H, H, 3 * C, DEV).slice(C, C)
    dhT.buf.normal_()
    prog = LSTMProgram(lstm)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("STF_LSTM_HOIST", mode)
        lb = nhwc.zeros_feat(T * B, H, H, 2 * C, DEV)
        lb.buf.copy_(lbuf.buf)
        hT = nhwc.new_feat(B, H, H, 2 * C, DEV).slice(0, C)
        st = prog.forward(lb, T, B, hT)
        assert (st.gates is not None) == gates
        gv = _Grads(lstm)
        dx = prog.backward(st, dhT, gv)
        out[mode] = [hT.dense(), dx.dense()] + [gv(p).clone() for p in lstm.parameters()]
    assert torch.equal(out["0"][0], out["1"][0])             # the forward is untouched
    for i, (a, b) in enumerate(zip(out["0"][1:], out["1"][1:])):
        e = ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()
        assert e <= 2e-3, (i, e)


def test_stf_training_steps_repeatable(monkeypatch):
    """Eight eager training steps, twice from the same weights, with no host sync inside the loop:
    the losses and the final parameters are identical bit for bit.  The LSTM backwards run on side
    streams beside the encoder's backward; encoder layer li's first block accumulates into the d x_t
    of lstm li-1 (side stream li-1), so a missing stream wait shows up here as a nondeterministic
    loss (a two-rank run of this loop diverged once every ~16 steps, once to NaN, before the wait
    was placed)."""
    from stfunet import STFLSTMUNet, engine
    from stfunet.optim import AdamW
    from stfunet.synthetic import dce_batch
    monkeypatch.setenv("STF_PLAN", "0")
    bs = [dce_batch(2, 4, 128, 128, seed=900 + r, device="cuda", mask_hw=(64, 64)) for r in range(2)]

    def run():
        torch.manual_seed(0)
        m = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=4).cuda().train()
        opt = AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
        losses = []
        for i in range(8):
            x, t = bs[i % 2]
            loss = engine.criterion(m(x), t)
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.detach().clone())
        torch.cuda.synchronize()
        return torch.stack(losses), m.program.flat.data.detach().clone()

    la, pa = run()
    lb, pb = run()
    assert torch.isfinite(la).all()
    assert torch.equal(la, lb), (la, lb)
    assert torch.equal(pa, pb)


@pytest.mark.parametrize("B, T, H, W", [(2, 3, 64, 80), (1, 2, 37, 50)])
def test_stem_conv7_direct_equals_im2col_gemm(B, T, H, W):
    """The direct 7x7/s2 stem kernel (stf_stem_conv7) against the im2col + 1x1 GEMM path it replaces
    (src/stf_lstm_unet.py:108,177): the bf16 output bit for bit (same k order and MFMA sequence), the
    per-time-step BatchNorm sums of its statistics rows to fp32 rounding; odd sizes hit partial tiles
    and the zero padding."""
    from stfunet import _lib, nhwc
    from stfunet._lib import call
    torch.manual_seed(5)
    x = torch.randn(B, T + 1, 1, H, W, device="cuda")          # one extra frame the stem must skip
    w1 = torch.randn(64, 1, 7, 7, device="cuda") * 0.1
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    wp = nhwc.pack_weight(w1.view(64, -1, 1, 1), 0, 64)
    xin = nhwc.new_feat(T * B, Ho, Wo, 64, "cuda")
    call("stf_stem_im2col", x.data_ptr(), B, T + 1, 1, H, W, T, 0, 7, 2, 3, 64, xin.ptr(), _lib.stream())
    y_ref = nhwc.new_feat(T * B, Ho, Wo, 64, "cuda")
    st_ref, tiles_ref = nhwc.igemm(xin, wp, 64, y_ref, 1, 1, 1, 0, want_stats=True, groups=T)
    y = nhwc.new_feat(T * B, Ho, Wo, 64, "cuda")
    tiles = _lib.load().stf_stem_conv7_grid(B, T, H, W)
    st = torch.empty(T * tiles * 2 * 64, dtype=torch.float32, device="cuda")
    call("stf_stem_conv7", x.data_ptr(), B, T + 1, H, W, T, wp.data_ptr(), y.ptr(), st.data_ptr(), _lib.stream())
    torch.cuda.synchronize()
    assert torch.equal(y.buf, y_ref.buf)
    s_new = st.view(T, tiles, 2, 64).double().sum(1)
    s_ref = st_ref.view(T, tiles_ref, 2, 64).double().sum(1)
    assert torch.allclose(s_new, s_ref, rtol=1e-5, atol=1e-3)
    # the weight gradient from the frames (stf_stem_wgrad7 + reduce) against the GEMM wgrad over the
    # im2col columns, with a random output gradient
    dy = nhwc.new_feat(T * B, Ho, Wo, 64, "cuda")
    dy.buf.copy_(torch.randn(dy.buf.numel(), device="cuda").to(dy.buf.dtype))
    ref = torch.empty(64 * 64, dtype=torch.float32, device="cuda")
    nhwc.wgrad(dy, xin, 1, 1, 1, 0, ref, defer=False)
    ws = torch.empty(tiles * 64 * 64, dtype=torch.float32, device="cuda")
    call("stf_stem_wgrad7", x.data_ptr(), B, T + 1, H, W, T, dy.ptr(), ws.data_ptr(), _lib.stream())
    got = torch.empty(64 * 64, dtype=torch.float32, device="cuda")
    call("stf_wgrad_reduce", ws.data_ptr(), tiles, 64, 1, 1, 64, got.data_ptr(), _lib.stream())
    torch.cuda.synchronize()
    ref, got = ref.view(64, 64), got.view(64, 64)
    assert torch.count_nonzero(got[:, 49:]) == 0
    err = (got - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item() + 1e-3, err
