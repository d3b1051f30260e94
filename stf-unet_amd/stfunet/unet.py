"""Drop-in ``UNet`` (reference ``src/unet.py:5-57``) running on gfx950 kernels.

Surface kept from the reference: class attribute ``input_format =
"flat_channels"`` (read by ``preprocess_input``, train_and_eval.py:9-22), the
constructor ``UNet(in_channels=8, num_classes=2, base_c=64)``, the module tree
(``enc1..4``, ``pool``, ``bottleneck``, ``up1..4``, ``dec1..4``, ``out_conv``; each
DoubleConv an ``nn.Sequential(Conv2d, BatchNorm2d, ReLU, Conv2d, BatchNorm2d,
ReLU)``) and therefore the 136 ``state_dict`` keys and PyTorch's default init,
and ``forward(x) -> {"out": logits}`` with logits [B, classes, H, W] fp32.

What runs is not those modules' forward: ``forward`` hands the input and every
parameter to ``_UNetFunction``, an explicit schedule over NHWC bf16 buffers:

  forward, per DoubleConv (src/unet.py:10-18):
    igemm conv3x3 (+bias, +BN partial sums) -> bn_finalize -> bn_act
    igemm conv3x3 (+bias, +BN partial sums) -> bn_finalize -> bn_act writing
        the skip half of the level's concat buffer and the 2x2-pooled input of
        the next level in one pass (Down = MaxPool2d(2), src/unet.py:25,41-45)
  Up (src/unet.py:28-35,47-54): igemm with a ConvTranspose2d(2,2) scatter
        epilogue writes the other half of the concat buffer: no torch.cat
  OutConv (src/unet.py:37,56): fused with dec1's last BN+ReLU in stf_head_fwd
  backward: the mirror schedule, gradients written into one flat fp32 buffer.
"""

import torch
import torch.nn as nn

from . import _lib, nhwc
from .flat import FlatParams
from .nhwc import Feat, new_feat
from .plan import StepRuntime


def _double_conv(cin, cout):
    # src/unet.py:10-18 -- module indices 0/1/3/4 are the state_dict contract
    return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True),
                         nn.Conv2d(cout, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


def _cpad(c):
    return (c + 7) // 8 * 8


class _Saved:
    pass


class DoubleConvProgram:
    """Forward/backward schedule of one DoubleConv block on NHWC buffers."""

    def __init__(self, blk, name=""):
        self.blk = blk
        self.cout = blk[0].out_channels
        self.name = name

    def forward(self, src: Feat, training, need_bwd, out: Feat = None, pooled: Feat = None):
        with nhwc.timed_block(f"{self.name}.fwd"):
            return self._forward(src, training, need_bwd, out, pooled)

    def backward(self, s, grads, need_dsrc, dz: Feat = None, dpool: Feat = None, dy2: Feat = None,
                 dsrc_stats=False):
        with nhwc.timed_block(f"{self.name}.bwd"):
            return self._backward(s, grads, need_dsrc, dz, dpool, dy2, dsrc_stats)

    def _forward(self, src: Feat, training, need_bwd, out: Feat = None, pooled: Feat = None):
        conv1, bn1, conv2, bn2 = self.blk[0], self.blk[1], self.blk[3], self.blk[4]
        C, dev = self.cout, src.buf.device
        s = _Saved()
        s.src = src
        y1 = new_feat(src.N, src.H, src.W, C, dev)
        w1 = nhwc.pack_weight(conv1.weight, 0, src.C)
        st, tiles = nhwc.igemm(src, w1, C, y1, 3, 3, 1, 1, bias=conv1.bias.detach(), want_stats=training)
        s.bn1 = nhwc.bn_finalize(st, tiles, bn1, y1.M, training)
        a1 = new_feat(src.N, src.H, src.W, C, dev)
        nhwc.bn_act(y1, s.bn1, a1)
        y2 = new_feat(src.N, src.H, src.W, C, dev)
        w2 = nhwc.pack_weight(conv2.weight, 0, C)
        st, tiles = nhwc.igemm(a1, w2, C, y2, 3, 3, 1, 1, bias=conv2.bias.detach(), want_stats=training)
        s.bn2 = nhwc.bn_finalize(st, tiles, bn2, y2.M, training)
        if out is not None:
            nhwc.bn_act(y2, s.bn2, out, pooled=pooled)
        s.y1, s.a1, s.y2 = y1, a1, y2
        return s if need_bwd else None

    def _backward(self, s, grads, need_dsrc, dz: Feat = None, dpool: Feat = None, dy2: Feat = None,
                  dsrc_stats=False):
        """Either (dz and/or dpool) w.r.t. the block output, or dy2 (grad w.r.t.
        the raw second conv output, when the BN backward was fused upstream).  ``dsrc_stats``:
        return (dsrc, statistics rows, tiles) -- the per-tile column sums of the stored input
        gradient (a decoder block's concat gradient: the up-conv's bias gradient, no extra pass)."""
        conv1, bn1, conv2, bn2 = self.blk[0], self.blk[1], self.blk[3], self.blk[4]
        gv = grads.grad_view
        if dy2 is None:
            dy2 = nhwc.bn_backward(s.y2, s.bn2, bn2, gv(bn2.weight), gv(bn2.bias), dz=dz, dpool=dpool,
                                   dbias=gv(conv2.bias))
        nhwc.wgrad(dy2, s.a1, 3, 3, 1, 1, gv(conv2.weight))
        da1 = new_feat(s.a1.N, s.a1.H, s.a1.W, self.cout, s.a1.buf.device)
        # dgrad of conv2 also reduces BN1's backward sums (fused epilogue)
        part, tiles = nhwc.conv_dgrad(dy2, conv2.weight, da1, 3, 3, 1, 1, bnr=(s.y1, s.bn1, True))
        dy1 = nhwc.bn_backward_fused(da1, s.y1, s.bn1, bn1, part, tiles, gv(bn1.weight), gv(bn1.bias),
                                     dbias=gv(conv1.bias))
        del da1
        self._wgrad_conv1(dy1, s.src, gv(conv1.weight))
        if not need_dsrc:
            return None
        dsrc = new_feat(s.src.N, s.src.H, s.src.W, s.src.C, s.src.buf.device)
        w1 = conv1.weight
        if s.src.C != w1.shape[1]:
            # zero-padded input channels (in_channels % 8 != 0): the weight padded the same way, so the
            # padded channels' gradient is computed and dropped by the caller
            cin = w1.shape[1]
            wp = nhwc.memset0(nhwc.empty((self.cout, s.src.C, 3, 3), torch.float32, w1.device))
            nhwc.copy_rows(w1.detach(), cin * 9, wp, s.src.C * 9, self.cout, cin * 9)
            w1 = wp
        st, tiles = nhwc.conv_dgrad(dy1, w1, dsrc, 3, 3, 1, 1, cache=w1 is conv1.weight, want_stats=dsrc_stats)
        return (dsrc, st, tiles) if dsrc_stats else dsrc

    def _wgrad_conv1(self, dy1, src, out):
        cin = self.blk[0].in_channels
        if src.C == cin:
            nhwc.wgrad(dy1, src, 3, 3, 1, 1, out)
        else:   # zero-padded input channels (in_channels % 8 != 0): drop the padded columns
            tmp = nhwc.empty(self.cout * src.C * 9, torch.float32, out.device)
            nhwc.wgrad(dy1, src, 3, 3, 1, 1, tmp, defer=False)
            nhwc.copy_rows(tmp, src.C * 9, out, cin * 9, self.cout, cin * 9)


class UNetProgram:
    def __init__(self, model):
        self.m = model
        self.packs = nhwc.PackCache()
        self.levels = [DoubleConvProgram(b, f"enc{i}") for i, b in
                       enumerate((model.enc1, model.enc2, model.enc3, model.enc4), start=1)]
        self.bott = DoubleConvProgram(model.bottleneck, "bottleneck")
        self.ups = [model.up4, model.up3, model.up2, model.up1]
        self.decs = [DoubleConvProgram(b, f"dec{i}") for i, b in
                     zip((4, 3, 2, 1), (model.dec4, model.dec3, model.dec2, model.dec1))]
        self.flat = FlatParams(model)
        # grad_ready_hook(begin): flat-gradient elements [begin, numel) are final.  Backward
        # finishes blocks in exactly the reverse of registration (= flat) order, so the
        # finished gradients always form a suffix of the flat buffer (DDP buckets).
        self.grad_ready_hook = None
        # set by _UNetFunction for the backward in flight: also return d(loss)/d(input)
        self.want_dx = False
        self.dx = None
        self.runtime = StepRuntime(self)

    def _done(self, module):
        if self.grad_ready_hook is not None:
            # (with weight gradients on a side stream, the bucket waits for that stream too)
            deps = (nhwc.WGRAD_STREAM,) if nhwc.WGRAD_STREAM is not None else ()
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
        # weight gradients stay on the current stream here: a side stream (as in the STF
        # program) measured +1.2 / -0.3..-3.8 % at cfg2 (full / one-per-CU grid, round 5) and makes
        # every concurrent kernel's duration a shared-machine number; the variant was removed
        nhwc.ACTIVE_PACKS = self.packs
        try:
            return self._backward(S, dlogits)
        finally:
            nhwc.ACTIVE_PACKS = None

    def _forward(self, x, training, need_bwd):
        m = self.m
        nhwc._NBT_PENDING.clear()
        N, _, H, W = x.shape
        assert H % 16 == 0 and W % 16 == 0, "UNet needs H, W divisible by 16 (four 2x2 pools)"
        dev = x.device
        S = _Saved()
        src = nhwc.pack_input(x, _cpad(m.in_channels))
        S.enc, S.cats = [], []
        h, w = H, W
        for lvl in self.levels:
            C = lvl.cout
            cat = new_feat(N, h, w, 2 * C, dev)
            pooled = new_feat(N, h // 2, w // 2, C, dev)
            S.enc.append(lvl.forward(src, training, need_bwd, out=cat.slice(C, C), pooled=pooled))
            S.cats.append(cat)
            src = pooled
            h, w = h // 2, w // 2
        Cb = self.bott.cout
        a_b = new_feat(N, h, w, Cb, dev)
        S.bott = self.bott.forward(src, training, need_bwd, out=a_b)
        cur = a_b
        S.dec, S.dec_in = [], []
        for i, (up, dec) in enumerate(zip(self.ups, self.decs)):
            cat = S.cats[3 - i]
            Clo = dec.cout
            wt = nhwc.pack_weight(up.weight, 2)
            nhwc.igemm(cur, wt, 4 * Clo, cat.slice(0, Clo), 1, 1, 1, 0, bias=up.bias.detach(), scatter2x2=True)
            S.dec_in.append(cur)
            last = i == 3
            if not last:
                out = new_feat(cat.N, cat.H, cat.W, Clo, dev)
                S.dec.append(dec.forward(cat, training, need_bwd, out=out))
                cur = out
            else:
                s = dec.forward(cat, training, True)
                S.dec.append(s)
        # OutConv fused with dec1's last BN+ReLU
        s = S.dec[-1]
        K = m.out_conv.out_channels
        logits = nhwc.empty((N, K, H, W), torch.float32, dev)
        S.head_w = m.out_conv.weight.detach().reshape(K, -1).contiguous()
        nhwc.call("stf_head_fwd", s.y2.ptr(), N, H, W, s.y2.C, nhwc._p(s.bn2.scale), nhwc._p(s.bn2.shift),
                  nhwc._p(S.head_w), nhwc._p(m.out_conv.bias.detach()), K, nhwc._p(logits), nhwc.stream())
        if not need_bwd:
            S.enc = S.cats = S.dec = None
        nhwc.flush_batches_tracked()
        return logits, (S if need_bwd else None)

    # ------------------------------------------------------------------ backward
    def _backward(self, S, dlogits):
        m = self.m
        gv = self.flat.grad_view
        dev = dlogits.device
        dlogits = dlogits.contiguous().float()
        # head + dec1's last BN+ReLU
        s = S.dec[-1]
        N, K, H, W = dlogits.shape
        C = s.y2.C
        lib = nhwc._lib.load()
        tiles = lib.stf_head_tiles(N, H, W, C)
        g = new_feat(N, H, W, C, dev)
        bnp = nhwc.empty(tiles * 2 * C, torch.float32, dev)
        hp = nhwc.empty((tiles + 1) * K * (C + 1), torch.float32, dev)
        nhwc.call("stf_head_bwd", nhwc._p(dlogits), s.y2.ptr(), N, H, W, C, nhwc._p(s.bn2.scale),
                  nhwc._p(s.bn2.shift), nhwc._p(s.bn2.mean), nhwc._p(s.bn2.invstd), nhwc._p(S.head_w), K,
                  g.ptr(), nhwc._p(bnp), nhwc._p(hp), nhwc._p(gv(m.out_conv.weight)),
                  nhwc._p(gv(m.out_conv.bias)), nhwc.stream())
        dec1 = self.decs[3]
        dy2 = nhwc.bn_backward_from_partial(g, s.y2, s.bn2, dec1.blk[4], bnp, tiles, gv(dec1.blk[4].weight),
                                            gv(dec1.blk[4].bias), gv(dec1.blk[3].bias))
        # the concat gradient of each decoder block comes with the per-tile column sums of what its
        # dgrad stored (statistics epilogue): the up-conv's bias gradient is their up-half fold
        dcat, cst, ctiles = dec1.backward(s, self.flat, True, dy2=dy2, dsrc_stats=True)
        self._done(dec1.blk)
        dcats = [None] * 4
        dcats[0] = (dcat, cst, ctiles)
        # decoder levels 2..4 and the up-convs, deepest last
        for i in (3, 2, 1, 0):                       # index into self.ups / S.dec_in (up1 is i=3)
            up = self.ups[i]
            dcat, cst, ctiles = dcats[3 - i]
            dcats[3 - i] = dcat
            Clo = self.decs[i].cout
            dup = dcat.slice(0, Clo)
            src = S.dec_in[i]
            nhwc.wgrad(src, dup, 2, 2, 2, 0, gv(up.weight))
            nhwc.stat_sums(cst, ctiles, dcat.C, 0, Clo, gv(up.bias))       # (= channel_sum(dup))
            dsrc = new_feat(src.N, src.H, src.W, src.C, dev)
            nhwc.igemm(dup, nhwc.pack_weight(up.weight, 3), src.C, dsrc, 2, 2, 2, 0)
            self._done(up)
            if i > 0:
                dcats[4 - i] = self.decs[i - 1].backward(S.dec[i - 1], self.flat, True, dz=dsrc, dsrc_stats=True)
                self._done(self.decs[i - 1].blk)
            else:
                d_b = dsrc
        dpool = self.bott.backward(S.bott, self.flat, True, dz=d_b)
        self._done(self.bott.blk)
        for j in (3, 2, 1, 0):
            lvl = self.levels[j]
            C = lvl.cout
            dskip = dcats[j].slice(C, C)
            dpool = lvl.backward(S.enc[j], self.flat, j > 0 or self.want_dx, dz=dskip, dpool=dpool)
            dcats[j] = None
            self._done(lvl.blk)
        if self.want_dx:     # enc1's input gradient, NHWC 16-bit -> the input's [N, C, H, W] fp32
            self.dx = dpool.dense()[:, : m.in_channels].contiguous()


class _UNetFunction(torch.autograd.Function):
    """``res``: (logits, saved state) of the plan-cached forward UNet.forward already enqueued (the
    GPU starts while autograd processes the parameter inputs), or None (input gradients: the eager
    forward runs here)."""
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
        ctx.prog = prog
        ctx.saved = saved
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


class UNet(nn.Module):
    input_format = "flat_channels"  # [B, T*C, H, W], train_and_eval.py:12-14

    def __init__(self, in_channels=8, num_classes=2, base_c=64):
        super().__init__()
        self.in_channels = in_channels
        self.enc1 = _double_conv(in_channels, base_c)
        self.enc2 = _double_conv(base_c, base_c * 2)
        self.enc3 = _double_conv(base_c * 2, base_c * 4)
        self.enc4 = _double_conv(base_c * 4, base_c * 8)
        self.pool = nn.MaxPool2d(2)
        self.bottleneck = _double_conv(base_c * 8, base_c * 16)
        self.up4 = nn.ConvTranspose2d(base_c * 16, base_c * 8, kernel_size=2, stride=2)
        self.dec4 = _double_conv(base_c * 16, base_c * 8)
        self.up3 = nn.ConvTranspose2d(base_c * 8, base_c * 4, kernel_size=2, stride=2)
        self.dec3 = _double_conv(base_c * 8, base_c * 4)
        self.up2 = nn.ConvTranspose2d(base_c * 4, base_c * 2, kernel_size=2, stride=2)
        self.dec2 = _double_conv(base_c * 4, base_c * 2)
        self.up1 = nn.ConvTranspose2d(base_c * 2, base_c, kernel_size=2, stride=2)
        self.dec1 = _double_conv(base_c * 2, base_c)
        self.out_conv = nn.Conv2d(base_c, num_classes, kernel_size=1)
        self._program = None
        # 16-bit activation storage: None = bf16, or fp16 under autocast(float16) (the
        # reference's --amp); torch.bfloat16 / torch.float16 force one (_lib.storage_for)
        self.storage_dtype = None

    @property
    def program(self):
        if self._program is None:
            self._program = UNetProgram(self)
        return self._program

    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("stfunet.UNet runs on the gfx950 HIP kernels only; move the model and input "
                               "to a ROCm device (no CPU fallback)")
        prog = self.program
        prog.flat.ensure()
        storage = _lib.storage_for(self.storage_dtype)
        grad = torch.is_grad_enabled()
        res = None
        if not (grad and x.requires_grad):
            need_bwd = grad and prog.flat.any_requires_grad()
            with _lib.storage(storage), torch.no_grad():   # (as inside autograd.Function.forward)
                res = prog.runtime.forward(x, self.training, need_bwd)   # launched before autograd's bookkeeping
        return {"out": _UNetFunction.apply(x, prog, storage, res, *prog.flat.params)}
