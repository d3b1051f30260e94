"""Drop-in ``STFLSTMUNet`` (reference ``src/stf_lstm_unet.py:89-256``) on gfx950 kernels.

Surface kept: ``STFLSTMUNet(in_channels=1, num_classes=2, time_steps=8,
use_pk_maps=False, pk_channels=3)``, ``forward(x, pk_maps=None) -> {"out": logits}``
with x [B, T(+P), C, H, W] and logits at H/2 x W/2 (the reference's output size,
SURVEY.md section 0), the module tree and therefore all ``state_dict`` keys:
``conv1``/``bn1``/``layer1..4`` (torchvision ResNet-34 names, BasicBlock
``conv1,bn1,conv2,bn2,downsample``), ``pk_fusion1..4``, ``lstm1..4`` (nn.LSTM
parameters), ``decoder4..2`` (``up``, ``fusion``, ``res_conv.conv_block``),
``upconv1``, ``final_res``, ``final``.

Schedule (all NHWC bf16, fp32 statistics; ``STFProgram``):
  * the T time steps are one batch of T*B images, t-major; every BatchNorm of the
    encoder keeps per-time-step statistics (groups = T) and advances its running
    stats T times, as the reference's per-t loop does (:168-186);
  * stem conv7x7/s2 (+BN+ReLU) -> MaxPool(3,2,1) -> ResNet-34 BasicBlocks with the
    residual add + ReLU fused into the second BN's apply pass;
  * each layer's output is written straight into the [x_t | h_{t-1}] buffer of
    its LSTM; every LSTM step is ONE implicit GEMM (K = 2C, N = 4C gate-interleaved)
    whose epilogue is the cell update, writing h_t into the next step's buffer
    and h_T into the decoder's concat buffer (skip "cat" without a copy);
  * decoder: ConvTranspose2d(3,2,1,1) as a transposed gather into the concat
    buffer, 1x1 fusion conv, ResidualConvBlock; final 1x1 fused into the head.
  * backward mirrors it (BPTT = per-step cell kernel + one GEMM; LSTM weight
    gradients = one GEMM over all T steps).
"""
import os

import torch
import torch.nn as nn

from . import _lib, nhwc
from ._lib import LstmEpi, call, stream
from .flat import FlatParams
from .nhwc import BNState, Feat, _p, new_feat, rows, zeros_feat
from .plan import StepRuntime


# ------------------------------------------------------------------ module tree
class BasicBlock(nn.Module):
    """torchvision ResNet BasicBlock parameter container (names are the contract)."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride


def _resnet_layer(inplanes, planes, blocks, stride):
    ds = None
    if stride != 1 or inplanes != planes:
        ds = nn.Sequential(nn.Conv2d(inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
    layers = [BasicBlock(inplanes, planes, stride, ds)]
    layers += [BasicBlock(planes, planes) for _ in range(1, blocks)]
    return nn.Sequential(*layers)


class ResidualConvBlock(nn.Module):
    """src/stf_lstm_unet.py:7-35 (conv_block 0/1/3/4, optional 1x1 shortcut)."""
    input_format = "time_sequence"

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv_block = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, 3, padding=1, bias=False), nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True), nn.Conv2d(out_channels, out_channels, 3, padding=1, bias=False),
            nn.BatchNorm2d(out_channels))
        self.shortcut = nn.Sequential()
        if in_channels != out_channels:
            self.shortcut = nn.Sequential(nn.Conv2d(in_channels, out_channels, 1, bias=False),
                                          nn.BatchNorm2d(out_channels))
        self.relu = nn.ReLU(inplace=True)


class DecoderBlock(nn.Module):
    """src/stf_lstm_unet.py:38-68."""

    def __init__(self, in_channels, skip_channels, out_channels):
        super().__init__()
        self.up = nn.ConvTranspose2d(in_channels, out_channels, kernel_size=3, stride=2, padding=1,
                                     output_padding=1)
        self.fusion = nn.Conv2d(out_channels + skip_channels, out_channels, kernel_size=1)
        self.res_conv = ResidualConvBlock(out_channels, out_channels)


class _S:
    pass


# ------------------------------------------------------------------ block programs
class ResBlockProgram:
    """BasicBlock / ResidualConvBlock: out = relu(bn2(conv2(relu(bn1(conv1 x)))) + sc(x))."""

    def __init__(self, conv1, bn1, conv2, bn2, sc_conv=None, sc_bn=None):
        self.conv1, self.bn1, self.conv2, self.bn2 = conv1, bn1, conv2, bn2
        self.sc_conv, self.sc_bn = sc_conv, sc_bn
        self.stride = conv1.stride[0]
        self.cout = conv1.out_channels

    def forward(self, src: Feat, out: Feat, training, groups):
        dev, C, st = src.buf.device, self.cout, self.stride
        Ho, Wo = (src.H - 1) // st + 1, (src.W - 1) // st + 1
        s = _S()
        s.src, s.out = src, out
        y1 = new_feat(src.N, Ho, Wo, C, dev)
        stats, tiles = nhwc.igemm(src, nhwc.pack_weight(self.conv1.weight, 0, src.C), C, y1, 3, 3, st, 1,
                                  want_stats=training, groups=groups)
        s.bn1 = nhwc.bn_finalize(stats, tiles, self.bn1, y1.M, training, groups)
        a1 = new_feat(src.N, Ho, Wo, C, dev)
        nhwc.bn_act(y1, s.bn1, a1)
        y2 = new_feat(src.N, Ho, Wo, C, dev)
        stats, tiles = nhwc.igemm(a1, nhwc.pack_weight(self.conv2.weight, 0, C), C, y2, 3, 3, 1, 1,
                                  want_stats=training, groups=groups)
        s.bn2 = nhwc.bn_finalize(stats, tiles, self.bn2, y2.M, training, groups)
        s.yd = s.bnd = None
        if self.sc_conv is not None:
            yd = new_feat(src.N, Ho, Wo, C, dev)
            stats, tiles = nhwc.igemm(src, nhwc.pack_weight(self.sc_conv.weight, 0, src.C), C, yd, 1, 1, st, 0,
                                      want_stats=training, groups=groups)
            s.bnd = nhwc.bn_finalize(stats, tiles, self.sc_bn, yd.M, training, groups)
            s.yd = yd
            nhwc.bn_act(y2, s.bn2, out, res=yd, res_st=s.bnd)
        else:
            nhwc.bn_act(y2, s.bn2, out, res=src)
        s.y1, s.a1, s.y2 = y1, a1, y2
        return s

    def backward(self, s, gv, dout: Feat = None, g: Feat = None, dsrc: Feat = None, need_dsrc=True):
        """``dout``: grad w.r.t. the block output (masked here by out > 0), or
        ``g``: already-masked grad (the head fused the final ReLU).  ``dsrc``:
        destination that the input gradient is accumulated into (None: new)."""
        src = s.src
        if g is None:
            dy2, g = nhwc.bn_backward(s.y2, s.bn2, self.bn2, gv(self.bn2.weight), gv(self.bn2.bias), dz=dout,
                                      mask=s.out, keep_g=True)
        else:
            dy2 = nhwc.bn_backward(s.y2, s.bn2, self.bn2, gv(self.bn2.weight), gv(self.bn2.bias), dz=g,
                                   relu=False, out=new_feat(g.N, g.H, g.W, g.C, g.buf.device))
        nhwc.wgrad(dy2, s.a1, 3, 3, 1, 1, gv(self.conv2.weight))
        da1 = new_feat(s.a1.N, s.a1.H, s.a1.W, self.cout, s.a1.buf.device)
        part, tiles = nhwc.conv_dgrad(dy2, self.conv2.weight, da1, 3, 3, 1, 1, bnr=(s.y1, s.bn1, True))
        del dy2
        dy1 = nhwc.bn_backward_fused(da1, s.y1, s.bn1, self.bn1, part, tiles, gv(self.bn1.weight),
                                     gv(self.bn1.bias))
        del da1
        nhwc.wgrad(dy1, src, 3, 3, self.stride, 1, gv(self.conv1.weight))
        if self.sc_conv is None:
            # identity shortcut: d_src = g + dgrad(conv1)
            if dsrc is not None:
                raise NotImplementedError("identity-shortcut blocks produce their input gradient in place")
            nhwc.conv_dgrad(dy1, self.conv1.weight, g, 3, 3, self.stride, 1, accumulate=True)
            return g
        dyd = nhwc.bn_backward(s.yd, s.bnd, self.sc_bn, gv(self.sc_bn.weight), gv(self.sc_bn.bias), dz=g,
                               relu=False)
        nhwc.wgrad(dyd, src, 1, 1, self.stride, 0, gv(self.sc_conv.weight))
        if not need_dsrc:
            return None
        acc = dsrc is not None
        if dsrc is None:
            dsrc = new_feat(src.N, src.H, src.W, src.C, src.buf.device)
        nhwc.conv_dgrad(dyd, self.sc_conv.weight, dsrc, 1, 1, self.stride, 0, accumulate=acc)
        nhwc.conv_dgrad(dy1, self.conv1.weight, dsrc, 3, 3, self.stride, 1, accumulate=True)
        return dsrc


class LSTMProgram:
    """nn.LSTM(C, C) over T steps for every pixel, only h_T kept (src/stf_lstm_unet.py:214-242).

    ``lbuf``: [T*B images][h][w][2C] with rows of step t = [x_t | h_{t-1}] (x_t written
    by the encoder, h_{-1} = 0).  Step t is one implicit GEMM (K = 2C, N = 4C
    gate-interleaved) with the cell update in its epilogue; h_t lands in step t+1's
    rows and h_T in ``hT`` (e.g. the decoder's concat slice).  Only the cell states
    c_t (fp32) are kept for the backward: each backward step reruns step t's GEMM on
    the same rows (same kernel, bitwise the forward's gates) with the cell backward in
    its epilogue, instead of storing T x P x 4C fp32 activated gates.
    """

    def __init__(self, lstm, max_wg=0):
        self.lstm = lstm
        self.C = lstm.hidden_size
        # workgroup budget of the cooperative kernels (one per CU; 0 = the whole chip): an LSTM
        # on a side stream leaves the rest to the encoder / decoder of the main stream
        self.max_wg = max_wg
        # polls before a cooperative hand-off gives up (0 = the library's ~4 s; tests force 1)
        self.spin_limit = 0
        # the owning program's sticky device error word (STFProgram.err_word): every cooperative
        # launch ORs its timeout flag into it, the program raises at the next step boundary
        self.err_word = None

    def _note_coop(self, sync, npix, T):
        self.last_sync = (sync, npix, T)
        if self.err_word is not None:
            call("stf_lstm_coop_error", _p(sync), npix, T, _p(self.err_word), stream())

    def fused(self, lbuf: Feat, hT: Feat):
        """Whole-sequence kernel (stf_lstm_seq_fwd) for this hidden size and layout?
        STF_LSTM_SEQ=0 keeps the per-step launches (A/B)."""
        return (os.environ.get("STF_LSTM_SEQ", "1") != "0" and bool(_lib.load().stf_lstm_seq_supported(self.C))
                and lbuf.off == 0 and lbuf.cs == 2 * self.C and hT.cs >= self.C)

    def coop(self, lbuf: Feat, hT: Feat):
        """Cooperative whole-sequence forward (stf_lstm_coop_fwd, C = 128 / 256 / 512)?
        STF_LSTM_COOP: 1 = every supported C, 0 = the per-step launches, or a comma list of
        hidden sizes ("512", the default: only lstm4, the one on the main stream).
        STF_LSTM_COOP_BWD=1 also runs the cooperative backward (off by default, see above)."""
        # default: lstm4 only (the main-stream LSTM).  Measured (same box, cfg3, round 3): coop
        # forward of lstm4 +1.0 %; coop lstm2 / lstm3 on their side streams -0.5..-4 % (a launch
        # that needs its whole group resident spins on CUs the encoder needs); coop backward
        # -0.4..-2 % (lstm3's and lstm4's backward start together and contend)
        mode = os.environ.get("STF_LSTM_COOP", "512")
        on = mode == "1" or (mode not in ("0", "") and str(self.C) in mode.split(","))
        return (on and bool(_lib.load().stf_lstm_coop_supported(self.C))
                and lbuf.off == 0 and lbuf.cs == 2 * self.C and hT.cs >= self.C and hT.cs % 8 == 0
                and hT.ptr() % 16 == 0)

    def coop_error(self):
        """Nonzero if the last cooperative launch's in-launch hand-off timed out (syncs)."""
        if getattr(self, "last_sync", None) is None:
            return 0
        sync, npix, T = self.last_sync
        out = torch.zeros(1, dtype=torch.int32, device=sync.device)
        call("stf_lstm_coop_error", _p(sync), npix, T, _p(out), stream())
        return int(out.item())

    def forward(self, lbuf: Feat, T, B, hT: Feat, need_bwd=True):
        C, dev = self.C, lbuf.buf.device
        L = self.lstm
        npix = B * lbuf.H * lbuf.W
        wcat = nhwc.empty(8 * C * C, nhwc.sdt(), dev)
        wcat_t = nhwc.empty(8 * C * C, nhwc.sdt(), dev)
        bias = nhwc.empty(4 * C, torch.float32, dev)
        call("stf_lstm_pack", _p(L.weight_ih_l0.detach()), _p(L.weight_hh_l0.detach()), _p(L.bias_ih_l0.detach()),
             _p(L.bias_hh_l0.detach()), C, _p(wcat), _p(wcat_t), _p(bias), stream())
        cst = nhwc.empty((T, npix, C), torch.float32, dev)
        fused = self.fused(lbuf, hT)
        coop = not fused and self.coop(lbuf, hT)
        if fused:
            # all T steps in one launch: c in registers, h_{t-1} in LDS (same values)
            lbuf.check()
            hT.check()
            call("stf_lstm_seq_fwd", _p(wcat), _p(bias), lbuf.ptr(), npix, T, C, _p(cst), hT.ptr(), hT.cs, stream())
        elif coop:
            # C >= 128: all T steps in one persistent launch, the C/32 workgroups of a pixel
            # block hand h_t to each other in-launch (same values as the per-step launches)
            lbuf.check()
            hT.check()
            lib = _lib.load()
            sync = nhwc.empty(lib.stf_lstm_coop_sync_bytes(npix, T) // 4, torch.int32, dev)
            # the activated gates (fp32) are kept for the cooperative backward (no recompute)
            gates = nhwc.empty((T, npix, 4 * C), torch.float32, dev) if need_bwd else None
            call("stf_lstm_coop_fwd", _p(wcat), _p(bias), lbuf.ptr(), npix, T, C, _p(cst), hT.ptr(), hT.cs,
                 _p(gates), _p(sync), self.max_wg, self.spin_limit, stream())
            self._note_coop(sync, npix, T)
        else:
            for t in range(T):
                src = rows(lbuf, t * B, B)
                hdst = rows(lbuf, (t + 1) * B, B).slice(C, C) if t < T - 1 else hT
                epi = LstmEpi(_p(cst[t - 1]) if t > 0 else None, _p(cst[t]), hdst.ptr(), hdst.cs, None)
                nhwc.igemm(src, wcat, 4 * C, src, 1, 1, 1, 0, bias=bias, lstm=epi)
        st = _S()
        st.lbuf, st.T, st.B, st.wcat, st.wcat_t, st.bias, st.c = lbuf, T, B, wcat, wcat_t, bias, cst
        st.fused = fused
        st.coop = coop and need_bwd and os.environ.get("STF_LSTM_COOP_BWD", "0") == "1"
        st.gates = gates if coop else None
        return st

    def backward(self, st, dhT: Feat, gv):
        """Returns d x_t for every t as a Feat slice [T*B][h][w][C] (stride 2C)."""
        L, C, lb, T, B = self.lstm, self.C, st.lbuf, st.T, st.B
        dev = lb.buf.device
        npix = B * lb.H * lb.W
        d2 = new_feat(T * B, lb.H, lb.W, 2 * C, dev)           # rows of step t: [dx_t | dh_{t-1}]
        dg = new_feat(T * B, lb.H, lb.W, 4 * C, dev)           # pre-activation gate grads (interleaved)
        if st.fused:
            # all T steps backward in one launch (dc in registers, dh_{t-1} in LDS)
            dhT.check()
            call("stf_lstm_seq_bwd", _p(st.wcat), _p(st.wcat_t), _p(st.bias), lb.ptr(), npix, T, C, _p(st.c),
                 dhT.ptr(), dhT.cs, dg.ptr(), d2.ptr(), d2.cs, stream())
        elif st.coop:
            # C >= 128: all T steps backward in one persistent launch (dgates and [dx | dh]
            # exchanged in-launch inside each pixel block; the forward's gates, no recompute)
            dhT.check()
            lib = _lib.load()
            sync = nhwc.empty(lib.stf_lstm_coop_sync_bytes(npix, T) // 4, torch.int32, dev)
            call("stf_lstm_coop_bwd", _p(st.wcat_t), _p(st.gates), _p(st.c), npix, T, C, dhT.ptr(), dhT.cs,
                 dg.ptr(), d2.ptr(), d2.cs, _p(sync), self.max_wg, self.spin_limit, stream())
            self._note_coop(sync, npix, T)
        else:
            # BPTT over the per-step launches.  Per step: the cell backward -- from the activated
            # gates the cooperative forward kept (elementwise stf_lstm_cell_bwd, the arithmetic of
            # the recompute epilogue, so the same dgates bit for bit), or a recompute of step t's
            # gates (the forward's GEMM) with the cell backward in its epilogue -- then ONLY the
            # recurrent half dh_{t-1} = dgates_t W_hh (N = C).  The input half d x_t = dgates_t W_ih
            # does not feed the recurrence: it is ONE GEMM over all T steps after the loop (SURVEY
            # section 2.1 K10, src/stf_lstm_unet.py:124-127; STF_LSTM_HOIST=0: [dx | dh] per step).
            hoist = os.environ.get("STF_LSTM_HOIST", "1") != "0"
            gates = st.gates is not None and os.environ.get("STF_LSTM_GATES", "1") != "0"
            w_h = st.wcat_t[4 * C * C:]                     # rows C..2C-1 of [2C][4C]: the h outputs
            dc = nhwc.empty((npix, C), torch.float32, dev)
            for t in range(T - 1, -1, -1):
                dh = dhT if t == T - 1 else rows(d2, (t + 1) * B, B).slice(C, C)
                dgt = rows(dg, t * B, B)
                if gates:
                    call("stf_lstm_cell_bwd", _p(st.gates[t]), _p(st.c[t]), _p(st.c[t - 1]) if t > 0 else None,
                         dh.ptr(), dh.cs, _p(dc) if t < T - 1 else None, _p(dc), dgt.ptr(), npix, C, stream())
                else:
                    src = rows(lb, t * B, B)
                    epi = LstmEpi(_p(st.c[t - 1]) if t > 0 else None, _p(st.c[t]), None, 0, None,
                                  1, dh.ptr(), dh.cs, _p(dc) if t < T - 1 else None, _p(dc), dgt.ptr())
                    nhwc.igemm(src, st.wcat, 4 * C, src, 1, 1, 1, 0, bias=st.bias, lstm=epi)
                if not hoist:
                    nhwc.igemm(dgt, st.wcat_t, 2 * C, rows(d2, t * B, B), 1, 1, 1, 0)
                elif t > 0:                                  # dh_{-1} feeds nothing
                    nhwc.igemm(dgt, w_h, C, rows(d2, t * B, B).slice(C, C), 1, 1, 1, 0)
            if hoist:
                nhwc.igemm(dg, st.wcat_t[:4 * C * C], C, d2.slice(0, C), 1, 1, 1, 0)
        dwcat = nhwc.empty(8 * C * C, torch.float32, dev)
        nhwc.wgrad(dg, lb, 1, 1, 1, 0, dwcat, defer=False)
        dbcat = nhwc.empty(4 * C, torch.float32, dev)
        nhwc.channel_sum(dg, dbcat)
        call("stf_lstm_unpack_grad", _p(dwcat), _p(dbcat), C, _p(gv(L.weight_ih_l0)), _p(gv(L.weight_hh_l0)),
             _p(gv(L.bias_ih_l0)), _p(gv(L.bias_hh_l0)), stream())
        return d2.slice(0, C)


# ------------------------------------------------------------------ program
class STFProgram:
    def __init__(self, m):
        self.m = m
        self.packs = nhwc.PackCache()
        self.flat = FlatParams(m)
        self.grad_ready_hook = None
        self.want_dx = False           # set by _STFFunction.backward for an input that requires grad
        self.dx = None
        self.layers = []
        for layer in (m.layer1, m.layer2, m.layer3, m.layer4):
            progs = []
            for blk in layer:
                ds = blk.downsample
                progs.append(ResBlockProgram(blk.conv1, blk.bn1, blk.conv2, blk.bn2,
                                             ds[0] if ds is not None else None, ds[1] if ds is not None else None))
            self.layers.append(progs)
        self.decoders = [m.decoder4, m.decoder3, m.decoder2]
        self.dec_res = [ResBlockProgram(d.res_conv.conv_block[0], d.res_conv.conv_block[1],
                                        d.res_conv.conv_block[3], d.res_conv.conv_block[4])
                        for d in self.decoders]
        fr = m.final_res
        self.final_res = ResBlockProgram(fr.conv_block[0], fr.conv_block[1], fr.conv_block[3], fr.conv_block[4])
        self.lstms = [m.lstm1, m.lstm2, m.lstm3, m.lstm4]
        side_wg = int(os.environ.get("STF_LSTM_SIDE_WG", "64"))
        self.lstm_progs = [LSTMProgram(lstm, side_wg if k < 3 else 0) for k, lstm in enumerate(self.lstms)]
        self._side = None
        self._wstream = None
        self._ident = {}
        self.err_word = None          # sticky device flag of the cooperative LSTM launches
        self._err_host = None         # its pinned host copy, issued at each step boundary
        self._err_event = None
        self.runtime = StepRuntime(self)

    def plan_knobs(self):
        """Per-program scalars a recorded plan carries by value (part of its signature)."""
        return tuple((lp.spin_limit, lp.max_wg) for lp in self.lstm_progs)

    def check_device_errors(self, dev=None, block=False):
        """Raise if a cooperative LSTM launch of an earlier step timed out in its in-launch
        hand-off (its outputs, and so that step's update, are wrong).

        Called at every step boundary (``STFLSTMUNet.forward``): the flag that an earlier
        boundary copied to pinned host memory is read once the copy has landed (no host sync),
        then the current flag is copied out behind the work enqueued so far.  ``block``: also
        wait for that copy, so every launch enqueued before the call is covered."""
        if self.err_word is None:
            if dev is None:
                return
            self.err_word = torch.zeros(1, dtype=torch.int32, device=dev)
            self._err_host = torch.zeros(1, dtype=torch.int32).pin_memory()
            for lp in self.lstm_progs:
                lp.err_word = self.err_word
        if self._err_event is not None and (block or self._err_event.query()):
            self._read_error_flag()
        if self._err_event is None:
            self._err_host.copy_(self.err_word, non_blocking=True)
            self._err_event = torch.cuda.Event()
            self._err_event.record()
            if block:
                self._read_error_flag()

    def _read_error_flag(self):
        self._err_event.synchronize()
        self._err_event = None
        if int(self._err_host[0]) != 0:
            self.err_word.zero_()
            self._err_host.zero_()
            raise RuntimeError("stfunet: a cooperative LSTM launch (stf_lstm_coop_fwd/bwd) timed out in its "
                               "in-launch hand-off (its workgroups could not all be resident), so that step's "
                               "LSTM outputs and gradients are invalid; STF_LSTM_COOP=0 selects the per-step "
                               "launches")

    def _identity(self, C, dev):
        """BatchNorm-identity state of the head's input (no BN there), made once per (C, device)."""
        key = (C, str(dev), nhwc.sdt())
        if key not in self._ident:
            self._ident[key] = BNState.identity(C, dev)
        return self._ident[key]

    def side_streams(self, dev):
        """One HIP stream per LSTM scale 1-3.  The four per-pixel LSTMs are independent
        of each other: lstm k forward runs beside the deeper encoder layers and lstm k
        backward beside the remaining decoder backward, which leave most CUs idle at
        1/16 and 1/32 resolution (lstm4 stays on the main stream: the decoder and the
        encoder backward need it first).

        ``STF_SIDE_STREAMS`` maps lstm 1-3 to streams, one character each: a digit names a
        private stream, ``w`` the weight-gradient side stream (``nhwc.wgrad_side_stream``)."""
        if self._side is None or self._side[0].device != dev:
            spec = os.environ.get("STF_SIDE_STREAMS", "00w")
            if len(spec) != 3 or any(c not in "012w" for c in spec):
                raise ValueError(f"STF_SIDE_STREAMS={spec!r}: three of 0 1 2 w")
            own, ws = {}, nhwc.wgrad_side_stream(dev)
            side = []
            for c in spec:
                if c == "w" and ws is not None:
                    side.append(ws)
                else:
                    if c not in own:
                        own[c] = nhwc.side_stream(dev, "side" + c)
                    side.append(own[c])
            self._side = side
        return self._side

    def _done(self, module, side=None):
        """The gradients of ``module`` and of everything after it in flat order are final once
        the current stream's work, the weight-gradient stream's and (``side``) the stream that ran
        the module's own backward have run: the hook gets those streams as dependencies, so the
        main stream never waits for a side stream on its account."""
        nhwc.flush_bn_grads()          # grouped BN dgamma/dbeta before the buckets read them
        if self.grad_ready_hook is not None:
            deps = tuple(s for s in (self._wstream, side) if s is not None)
            first = next(module.parameters())
            self.grad_ready_hook(self.flat.offsets[self.flat.index[id(first)]], deps)

    # ------------------------------------------------------------------ forward
    def forward(self, x, training, need_bwd):
        """Refresh the packed weights (one launch) and run the forward schedule."""
        self.packs.refresh()
        nhwc.ACTIVE_PACKS = self.packs
        try:
            return self._forward(x, training, need_bwd)
        finally:
            nhwc.ACTIVE_PACKS = None

    def backward(self, S, dlogits):
        nhwc.ACTIVE_PACKS = self.packs
        ws = self._wstream = nhwc.wgrad_side_stream(dlogits.device)
        nhwc.WGRAD_STREAM = ws
        nhwc.WGRAD_MAIN = torch.cuda.current_stream(dlogits.device)
        try:
            return self._backward(S, dlogits)
        finally:
            nhwc.WGRAD_STREAM = nhwc.WGRAD_MAIN = None
            if ws is not None:
                nhwc.wait(torch.cuda.current_stream(dlogits.device), ws)
            nhwc.flush_bn_grads()
            nhwc.ACTIVE_PACKS = None

    def _forward(self, x, training, need_bwd):
        m = self.m
        nhwc._NBT_PENDING.clear()
        dev = x.device
        B, Ttot, Cf, H, W = x.shape
        P = m.pk_channels if m.use_pk_maps else 0
        T = Ttot - P
        _check_input_shape(x.shape, P)
        x = x.contiguous().float()
        S = _S()
        S.B, S.T, S.P, S.H, S.W = B, T, P, H, W
        N = T * B
        # ---- stem: conv 7x7/s2 over (Cf + P) <= 4 input channels as a 1x1 GEMM over the
        # im2col columns (49 (Cf+P) of them, padded): a per-tap gather would pad every tap
        # to 8 channels (8x the MFMA work at Cf = 1) and its weight gradient re-reads dy
        # once per 64 columns
        # With PK maps (Cf + P = 4 channels) the im2col columns would be 196 per output
        # pixel (3.5 GB at cfg5's 512^2 x T=32 x B=4): there the input is packed to 8
        # channels instead and the 7x7/s2 conv gathers its taps (8-channel tap path).
        h2, w2 = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        kreal = (Cf + P) * 49
        w1 = m.conv1.weight
        y0 = new_feat(N, h2, w2, 64, dev)
        S.stem_gather = Cf + P > 1 and Cf + P <= 8
        if S.stem_gather:
            xin = new_feat(N, H, W, 8, dev)
            call("stf_pack_sequence", _p(x), B, Ttot, Cf, H, W, T, P, 8, xin.ptr(), stream())
            stats, tiles = nhwc.igemm(xin, nhwc.pack_weight(w1, 0, 8), 64, y0, 7, 7, 2, 3,
                                      want_stats=training, groups=T)
        elif kreal == 49 and _STEM_DIRECT and N * h2 * w2 * 64 * 2 < 0xFFFFFF00:    # (32-bit store offsets)
            # one frame channel: the direct 7x7/s2 kernel (no im2col tensor: 268 MB written and read
            # back at cfg3), and in the backward its weight gradient straight from the frames too
            xin = None
            wp = nhwc.pack_weight(w1.view(w1.shape[0], -1, 1, 1), 0, 64)
            tiles = _lib.load().stf_stem_conv7_grid(B, T, H, W)
            stats = nhwc.empty(T * tiles * 2 * 64, torch.float32, dev) if training else None
            call("stf_stem_conv7", _p(x), B, Ttot, H, W, T, _p(wp), y0.ptr(), _p(stats), stream())
            if not training:
                tiles = 0
            S.x = x
        else:
            kpad = 64 if kreal <= 64 else (kreal + 31) // 32 * 32
            xin = new_feat(N, h2, w2, kpad, dev)
            call("stf_stem_im2col", _p(x), B, Ttot, Cf, H, W, T, P, 7, 2, 3, kpad, xin.ptr(), stream())
            stats, tiles = nhwc.igemm(xin, nhwc.pack_weight(w1.view(w1.shape[0], -1, 1, 1), 0, kpad), 64, y0, 1, 1,
                                      1, 0, want_stats=training, groups=T)
        S.bn0 = nhwc.bn_finalize(stats, tiles, m.bn1, y0.M, training, T)
        h4, w4 = (h2 - 1) // 2 + 1, (w2 - 1) // 2 + 1
        p0 = new_feat(N, h4, w4, 64, dev)
        # the window argmax the backward routes through (eval-mode backward needs it too)
        S.pool_arg = nhwc.empty(N * h4 * w4 * 64, torch.uint8, dev) if need_bwd else None
        # bn1 + relu + maxpool in one pass: the activation relu(bn1(y0)) is never stored (the
        # backward needs only y0 and the argmax)
        y0.check()
        call("stf_bn_act_maxpool3s2", y0.ptr(), N, h2, w2, 64, T, _p(S.bn0.scale), _p(S.bn0.shift), p0.ptr(),
             _p(S.pool_arg), stream())
        S.xin, S.y0, S.p0 = xin, y0, p0
        # ---- encoder; layer outputs land in the LSTM [x | h] buffers (or PK concat);
        # lstm li (li < 3) starts on its side stream as soon as layer li is done
        S.enc, S.lbuf, S.pkbuf = [], [], []
        S.dpk_parts = []                 # the input gradient's PK-map shares (eager input-gradient backward)
        side = self.side_streams(dev)
        main = torch.cuda.current_stream(dev)
        S.lstm = [None] * 4
        dcat = [None] * 3          # decoder concat buffers (skip half = h_T of the LSTM one scale up)
        cur = p0
        for li, progs in enumerate(self.layers):
            C = progs[0].cout
            hh, ww = ((cur.H - 1) // progs[0].stride + 1, (cur.W - 1) // progs[0].stride + 1)
            lbuf = zeros_feat(N, hh, ww, 2 * C, dev)            # [e_t | h_{t-1}], h_{-1} = 0
            pkb = None
            if P:
                pkb = zeros_feat(N, hh, ww, C + 8, dev)
                call("stf_pk_resize", _p(x), B, Ttot, T, P, H, W, hh, ww, pkb.ptr(), pkb.cs, C, stream())
            saved = []
            for bi, bp in enumerate(progs):
                last = bi == len(progs) - 1
                if last:
                    out = pkb.slice(0, C) if P else lbuf.slice(0, C)
                else:
                    out = new_feat(N, hh, ww, C, dev)
                saved.append(bp.forward(cur, out, training, T))
                cur = out
            if P:
                fus = getattr(m, f"pk_fusion{li + 1}")
                wf = nhwc.pack_weight(fus.weight, 0, C + 8)
                nhwc.igemm(pkb, wf, C, lbuf.slice(0, C), 1, 1, 1, 0, bias=fus.bias.detach())
            S.enc.append(saved)
            S.lbuf.append(lbuf)
            S.pkbuf.append(pkb)
            # ---- per-pixel LSTM of this scale over T
            lp = self.lstm_progs[li]
            if li < 3:
                d = self.decoders[2 - li]
                Cout = d.up.out_channels
                dc = dcat[2 - li] = new_feat(B, hh, ww, Cout + d.fusion.in_channels - Cout, dev)
                nhwc.wait(side[li], main)
                with torch.cuda.stream(side[li]):
                    S.lstm[li] = lp.forward(lbuf, T, B, dc.slice(dc.C - lp.C, lp.C), need_bwd)
            else:
                e4f = new_feat(B, hh, ww, lp.C, dev)
                S.lstm[li] = lp.forward(lbuf, T, B, e4f, need_bwd)
        S.dcat = dcat
        # ---- decoder
        S.dec = []
        cur = e4f
        for i, d in enumerate(self.decoders):
            nhwc.wait(main, side[2 - i])       # h_T of lstm 2-i fills the skip half of dcat[i]
            cat = dcat[i]
            Cout = d.up.out_channels
            up = None
            if (2 * cur.H, 2 * cur.W) == (cat.H, cat.W):
                nhwc.igemm(cur, nhwc.pack_weight(d.up.weight, 4), Cout, cat.slice(0, Cout), 3, 3, 2, 1,
                           transposed=True, bias=d.up.bias.detach())
            else:
                # H or W not divisible by 32: the transposed conv's 2h x 2w output is resized to the
                # skip's size (bilinear, align_corners=True; src/stf_lstm_unet.py:56-57)
                up = new_feat(B, 2 * cur.H, 2 * cur.W, Cout, dev)
                nhwc.igemm(cur, nhwc.pack_weight(d.up.weight, 4), Cout, up, 3, 3, 2, 1, transposed=True,
                           bias=d.up.bias.detach())
                sl = cat.slice(0, Cout)
                call("stf_bilinear_ac_fwd", up.ptr(), B, up.H, up.W, Cout, up.cs, sl.ptr(), cat.H, cat.W, sl.cs,
                     stream())
            yf = new_feat(B, cat.H, cat.W, Cout, dev)
            nhwc.igemm(cat, nhwc.pack_weight(d.fusion.weight, 0, cat.C), Cout, yf, 1, 1, 1, 0,
                       bias=d.fusion.bias.detach())
            out = new_feat(B, cat.H, cat.W, Cout, dev)
            rs = self.dec_res[i].forward(yf, out, training, 1)
            dsv = _S()
            dsv.x, dsv.cat, dsv.yf, dsv.res, dsv.up = cur, cat, yf, rs, up
            S.dec.append(dsv)
            cur = out
        # ---- upconv1 + final_res + final (head)
        up = m.upconv1
        u1 = new_feat(B, 2 * cur.H, 2 * cur.W, up.out_channels, dev)
        nhwc.igemm(cur, nhwc.pack_weight(up.weight, 4), up.out_channels, u1, 3, 3, 2, 1, transposed=True,
                   bias=up.bias.detach())
        fr_out = new_feat(B, u1.H, u1.W, up.out_channels, dev)
        S.fr = self.final_res.forward(u1, fr_out, training, 1)
        S.d2out, S.u1 = cur, u1
        K = m.final.out_channels
        logits = nhwc.empty((B, K, u1.H, u1.W), torch.float32, dev)
        S.ident = self._identity(fr_out.C, dev)
        S.head_w = m.final.weight.detach().reshape(K, -1).contiguous()
        call("stf_head_fwd", fr_out.ptr(), B, u1.H, u1.W, fr_out.C, _p(S.ident.scale), _p(S.ident.shift),
             _p(S.head_w), _p(m.final.bias.detach()), K, _p(logits), stream())
        nhwc.flush_batches_tracked()
        return logits, (S if need_bwd else None)

    # ------------------------------------------------------------------ backward
    def _backward(self, S, dlogits):
        m = self.m
        gv = self.flat.grad_view
        dev = dlogits.device
        dlogits = dlogits.contiguous().float()
        B, T, P = S.B, S.T, S.P
        fr_out = S.fr.out
        K = dlogits.shape[1]
        C = fr_out.C
        lib = _lib.load()
        tiles = lib.stf_head_tiles(B, fr_out.H, fr_out.W, C)
        g = new_feat(B, fr_out.H, fr_out.W, C, dev)
        bnp = nhwc.empty(tiles * 2 * C, torch.float32, dev)
        hp = nhwc.empty((tiles + 1) * K * (C + 1), torch.float32, dev)
        call("stf_head_bwd", _p(dlogits), fr_out.ptr(), B, fr_out.H, fr_out.W, C, _p(S.ident.scale),
             _p(S.ident.shift), _p(S.ident.mean), _p(S.ident.invstd), _p(S.head_w), K, g.ptr(), _p(bnp), _p(hp),
             _p(gv(m.final.weight)), _p(gv(m.final.bias)), stream())
        self._done(m.final)
        d_u1 = self.final_res.backward(S.fr, gv, g=g)
        self._done(m.final_res)
        up = m.upconv1
        nhwc.wgrad(S.d2out, d_u1, 3, 3, 2, 1, gv(up.weight))
        nhwc.channel_sum(d_u1, gv(up.bias))
        dcur = new_feat(B, S.d2out.H, S.d2out.W, S.d2out.C, dev)
        nhwc.igemm(d_u1, nhwc.pack_weight(up.weight, 3), S.d2out.C, dcur, 3, 3, 2, 1)
        del d_u1
        self._done(up)
        # decoders 2, 3, 4 (reverse of forward order); lstm k's backward starts on its
        # side stream as soon as its h_T gradient (the decoder's skip slice) is final
        side = self.side_streams(dev)
        main = torch.cuda.current_stream(dev)

        dhT = [None] * 4
        de = [None] * 4

        def lstm_bwd(k):
            de[k] = self.lstm_progs[k].backward(S.lstm[k], dhT[k], gv)
            de[k].buf.record_stream(main)
        for i in (2, 1, 0):
            d, dsv = self.decoders[i], S.dec[i]
            Cout = d.up.out_channels
            d_yf = self.dec_res[i].backward(dsv.res, gv, dout=dcur)
            nhwc.wgrad(d_yf, dsv.cat, 1, 1, 1, 0, gv(d.fusion.weight))
            nhwc.channel_sum(d_yf, gv(d.fusion.bias))
            dcat = new_feat(B, dsv.cat.H, dsv.cat.W, dsv.cat.C, dev)
            nhwc.conv_dgrad(d_yf, d.fusion.weight, dcat, 1, 1, 1, 0)
            del d_yf
            dup = dcat.slice(0, Cout)
            if dsv.up is not None:                             # through the bilinear size fallback
                du = new_feat(B, dsv.up.H, dsv.up.W, Cout, dev)
                call("stf_bilinear_ac_bwd", dup.ptr(), B, dup.H, dup.W, Cout, dup.cs, du.ptr(), du.H, du.W, du.cs,
                     stream())
                dup = du
            nhwc.wgrad(dsv.x, dup, 3, 3, 2, 1, gv(d.up.weight))
            nhwc.channel_sum(dup, gv(d.up.bias))
            dx = new_feat(B, dsv.x.H, dsv.x.W, dsv.x.C, dev)
            nhwc.igemm(dup, nhwc.pack_weight(d.up.weight, 3), dsv.x.C, dx, 3, 3, 2, 1)
            k = 2 - i                                          # skip of scale k (decoder4 -> idx 2)
            dhT[k] = dcat.slice(Cout, dcat.C - Cout)
            nhwc.wait(side[k], main)
            with torch.cuda.stream(side[k]):
                lstm_bwd(k)
            dcur = dx
            self._done(d)
        dhT[3] = dcur                                          # decoder4 input = h_T of lstm4
        lstm_bwd(3)
        # join the side streams: all of them now when PK fusion needs every scale, else each
        # just before the encoder block that first touches its d x_t; a gradient bucket holding
        # lstm k's gradients waits for side stream k itself (ready-hook dependency), not the main
        # stream
        for k in (3, 2, 1, 0):
            if P and k < 3:
                nhwc.wait(main, side[k])
            self._done(self.lstms[k], side[k] if k < 3 else None)
        if P:
            for k in (3, 2, 1, 0):
                de[k] = self._pk_fusion_backward(S, k, de[k], gv)
            self._done(m.pk_fusion1)
        # encoder: layer4 -> layer1; d(layer k-1 output) accumulates into de[k-1]
        # layer li reads d(its output) = de[li] (lstm li's d x_t, side stream li) and its first
        # block ACCUMULATES d(its input) into de[li - 1], which lstm li-1's backward writes on side
        # stream li-1: main waits for each side stream before the first of those two uses
        for li in (3, 2, 1, 0):
            progs, saved = self.layers[li], S.enc[li]
            dout = de[li]                           # (li < 3: side stream li waited in layer li+1)
            for bi in range(len(progs) - 1, -1, -1):
                bp, s = progs[bi], saved[bi]
                if bi == 0:
                    target = de[li - 1] if li > 0 else None
                    if li > 0 and not P:
                        nhwc.wait(main, side[li - 1])
                    dout = bp.backward(s, gv, dout=dout, dsrc=target)
                else:
                    dout = bp.backward(s, gv, dout=dout)
            self._done(getattr(m, f"layer{li + 1}"))
        # stem: maxpool(3,2,1) <- relu(bn1(conv1 x))
        # the pooled gradient routed by the argmax inside the BN backward's passes (no full-size
        # d relu(bn1(y0)) tensor)
        dy0 = nhwc.bn_backward_maxpool3(S.y0, S.bn0, m.bn1, gv(m.bn1.weight), gv(m.bn1.bias), S.pool_arg, dout)
        w1 = m.conv1.weight
        kreal = w1[0].numel()
        if self.want_dx:
            self.dx = self._input_grad(S, dy0, w1, B, T, P, dev)
        if S.xin is None:                      # direct stem conv: the gradient gathers the input too
            assert dy0.cs == 64 and dy0.off == 0
            lib = _lib.load()
            grid = lib.stf_stem_conv7_grid(B, T, S.H, S.W)
            ws = nhwc.empty(grid * 64 * 64, torch.float32, dev)
            call("stf_stem_wgrad7", _p(S.x), B, S.x.shape[1], S.H, S.W, T, dy0.ptr(), _p(ws), stream())
            tmp = nhwc.empty(64 * 64, torch.float32, dev)
            call("stf_wgrad_reduce", _p(ws), grid, 64, 1, 1, 64, _p(tmp), stream())
            nhwc.copy_rows(tmp, 64, gv(w1), kreal, w1.shape[0], kreal)
        elif S.stem_gather:                    # 8-channel packed input, 7x7/s2 gather
            tmp = nhwc.empty(w1.shape[0] * 8 * 49, torch.float32, dev)
            nhwc.wgrad(dy0, S.xin, 7, 7, 2, 3, tmp, defer=False)
            nhwc.copy_rows(tmp, 8 * 49, gv(w1), w1.shape[1] * 49, w1.shape[0], w1.shape[1] * 49)
        elif S.xin.C == kreal:
            nhwc.wgrad(dy0, S.xin, 1, 1, 1, 0, gv(w1))
        else:
            tmp = nhwc.empty(w1.shape[0] * S.xin.C, torch.float32, dev)
            nhwc.wgrad(dy0, S.xin, 1, 1, 1, 0, tmp, defer=False)
            nhwc.copy_rows(tmp, S.xin.C, gv(w1), kreal, w1.shape[0], kreal)

    def _input_grad(self, S, dy0, w1, B, T, P, dev):
        """d(loss)/d(x) for x [B, T + P, Cf, H, W]: the stem conv's input gradient over its Cf + P input
        channels (frame t's channels, then the P PK maps every frame's stem also reads,
        src/stf_lstm_unet.py:146-160), plus with PK maps the fusion branches' gradient w.r.t. the
        resized maps (saved by _pk_fusion_backward) taken back through the bilinear resize
        (align_corners=True, stf_bilinear_ac_bwd), summed over the T frames and the 4 scales."""
        assert dy0.cs == 64 and dy0.off == 0
        H, W = S.H, S.W
        cin = w1.shape[1]
        Cf = cin - P
        dxt = nhwc.empty((B, T, cin, H, W), torch.float32, dev)
        call("stf_stem_dgrad7", dy0.ptr(), _p(w1.detach().float().contiguous()), B, T, cin, H, W, T, _p(dxt),
             stream())
        if P == 0:
            return dxt
        dx = nhwc.empty((B, T + P, Cf, H, W), torch.float32, dev)
        dx[:, :T].copy_(dxt[:, :, :Cf])
        dx[:, T:, 0].copy_(dxt[:, :, Cf:].sum(1))                       # (PK maps: Cf == 1)
        for part in S.dpk_parts:                                        # [T*B, h, w, C + 8]: [.., C:C+P]
            C = part.C - 8
            src = part.slice(C, 8)
            # summed over the T frames at the low resolution in fp32, resized once, added into dx
            call("stf_bilinear_ac_bwd_tsum", src.ptr(), T, B, part.H, part.W, src.cs, P, _p(dx[:, T:]),
                 (T + P) * H * W, H * W, H, W, stream())
        S.dpk_parts = []
        return dx

    def _pk_fusion_backward(self, S, k, de: Feat, gv):
        fus = getattr(self.m, f"pk_fusion{k + 1}")
        pkb = S.pkbuf[k]
        C = de.C
        tmp = nhwc.empty(C * pkb.C, torch.float32, de.buf.device)
        nhwc.wgrad(de, pkb, 1, 1, 1, 0, tmp, defer=False)
        cin = fus.in_channels
        nhwc.copy_rows(tmp, pkb.C, gv(fus.weight), cin, C, cin)
        nhwc.channel_sum(de, gv(fus.bias))
        dpk = new_feat(pkb.N, pkb.H, pkb.W, pkb.C, de.buf.device)
        w = nhwc.memset0(nhwc.empty((C, pkb.C, 1, 1), torch.float32, de.buf.device))
        nhwc.copy_rows(fus.weight.detach(), cin, w, pkb.C, C, cin)
        nhwc.conv_dgrad(de, w, dpk, 1, 1, 1, 0, cache=False)
        if self.want_dx:                  # the resized PK maps' share, for _input_grad
            S.dpk_parts.append(dpk)
        return dpk.slice(0, C)


_STEM_DIRECT = os.environ.get("STF_STEM_DIRECT", "1") != "0"     # (A/B: 0 = im2col + 1x1 GEMM)


def _check_input_shape(shape, P):
    """[B, T + P, C, H, W] with at least one frame and H, W >= 32 (ResNet-34's five halvings leave
    layer4 at least one pixel).  Sizes not divisible by 32 take the reference's decoder size
    fallback: the transposed conv's output is resized to the skip's size by bilinear
    interpolation, align_corners=True (src/stf_lstm_unet.py:56-57, stf_bilinear_ac_fwd/_bwd)."""
    if len(shape) != 5:
        raise ValueError(f"STFLSTMUNet expects [B, T, C, H, W], got shape {tuple(shape)}")
    Ttot, H, W = shape[1], shape[3], shape[4]
    if Ttot - P < 1:
        raise ValueError(f"STFLSTMUNet: {Ttot} input frames leave no time steps after {P} PK maps")
    if H < 32 or W < 32:
        raise ValueError(f"STFLSTMUNet needs H, W >= 32 (got {H}x{W})")


class _STFFunction(torch.autograd.Function):
    """``res`` = (logits, saved state) of the forward STFLSTMUNet.forward already enqueued: the GPU
    starts on the step while autograd processes the ~160 parameter inputs of this call (~100 us of
    host time at every synced step boundary); or None (input gradients: the eager forward runs
    here)."""
    @staticmethod
    def forward(ctx, x, prog, storage, res, *params):
        ctx.need_dx = ctx.needs_input_grad[0]
        if res is not None:
            logits, saved = res
            prog.runtime.own(saved, ctx)
        else:
            need_bwd = any(ctx.needs_input_grad[4:]) or ctx.need_dx
            with _lib.storage(storage):
                logits, saved = prog.forward(x, prog.m.training, need_bwd)
        ctx.storage = storage
        ctx.prog, ctx.saved = prog, saved
        return logits.detach()        # the plan's static logits: a fresh tensor object per step

    @staticmethod
    def backward(ctx, dlogits):
        prog = ctx.prog
        dlogits = dlogits.float().contiguous()     # autocast / GradScaler callers: any float dtype
        prog.flat.fresh_grad()
        prog.want_dx, prog.dx = ctx.need_dx, None
        try:
            with _lib.storage(ctx.storage):
                prog.runtime.backward(ctx.saved, dlogits)
        finally:
            prog.want_dx = False
        ctx.saved = None
        if prog.grad_ready_hook is not None:
            prog.grad_ready_hook(0, ())
        dx, prog.dx = prog.dx, None
        return (dx, None, None, None, *prog.flat.grad_views())


class STFLSTMUNet(nn.Module):
    def __init__(self, in_channels=1, num_classes=2, time_steps=8, use_pk_maps=False, pk_channels=3):
        super().__init__()
        self.time_steps = time_steps
        self.use_pk_maps = use_pk_maps
        self.pk_channels = pk_channels if use_pk_maps else 0
        actual_in = in_channels + (pk_channels if use_pk_maps else 0)
        self.conv1 = nn.Conv2d(actual_in, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = _resnet_layer(64, 64, 3, 1)
        self.layer2 = _resnet_layer(64, 128, 4, 2)
        self.layer3 = _resnet_layer(128, 256, 6, 2)
        self.layer4 = _resnet_layer(256, 512, 3, 2)
        if use_pk_maps:
            self.pk_fusion1 = nn.Conv2d(64 + pk_channels, 64, kernel_size=1)
            self.pk_fusion2 = nn.Conv2d(128 + pk_channels, 128, kernel_size=1)
            self.pk_fusion3 = nn.Conv2d(256 + pk_channels, 256, kernel_size=1)
            self.pk_fusion4 = nn.Conv2d(512 + pk_channels, 512, kernel_size=1)
        self.lstm1 = nn.LSTM(64, 64, batch_first=True)
        self.lstm2 = nn.LSTM(128, 128, batch_first=True)
        self.lstm3 = nn.LSTM(256, 256, batch_first=True)
        self.lstm4 = nn.LSTM(512, 512, batch_first=True)
        self.decoder4 = DecoderBlock(512, 256, 256)
        self.decoder3 = DecoderBlock(256, 128, 128)
        self.decoder2 = DecoderBlock(128, 64, 64)
        self.upconv1 = nn.ConvTranspose2d(64, 32, kernel_size=3, stride=2, padding=1, output_padding=1)
        self.final_res = ResidualConvBlock(32, 32)
        self.final = nn.Conv2d(32, num_classes, kernel_size=1)
        self._program = None
        # 16-bit activation storage: None = bf16, or fp16 under autocast(float16) (the
        # reference's --amp); torch.bfloat16 / torch.float16 force one (_lib.storage_for)
        self.storage_dtype = None

    @property
    def program(self):
        if self._program is None:
            self._program = STFProgram(self)
        return self._program

    def forward(self, x, pk_maps=None):
        # pk_maps is ignored, as in the reference (PK maps ride on the T axis, :146-156)
        _check_input_shape(x.shape, self.pk_channels if self.use_pk_maps else 0)
        if not x.is_cuda:
            raise RuntimeError("stfunet.STFLSTMUNet runs on the gfx950 HIP kernels only; move the model and "
                               "input to a ROCm device (no CPU fallback)")
        prog = self.program
        prog.check_device_errors(x.device)       # step boundary: an earlier step's LSTM timeout raises
        prog.flat.ensure()
        grad = torch.is_grad_enabled()
        storage = _lib.storage_for(self.storage_dtype)
        res = None
        if grad and x.requires_grad:
            # the input gradient (reference autograd returns it, src/stf_lstm_unet.py:139-256): the
            # eager forward inside the autograd Function, the stem's input gradient in the backward
            # (with PK maps also their fusion branches' gradient through the resize)
            pass
        else:
            need_bwd = grad and prog.flat.any_requires_grad()
            with _lib.storage(storage), torch.no_grad():    # (as inside autograd.Function.forward)
                res = prog.runtime.forward(x, self.training, need_bwd)      # launched before autograd's bookkeeping
        return {"out": _STFFunction.apply(x, prog, storage, res, *prog.flat.params)}
