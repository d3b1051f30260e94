"""NHWC 16-bit feature maps and thin wrappers over the C-ABI kernels.

A ``Feat`` is a channel slice of an NHWC 16-bit buffer (bf16, or fp16 when the fp16
library is active: ``_lib.storage``): (buffer, N, H, W, C, channel stride, channel
offset).  Concat buffers are ordinary buffers whose
slices are written by different producers (virtual concat, no copy).

Every wrapper validates shapes on the host before launching (a kernel that
walks off a buffer can take the whole GPU down) and launches on torch's
current stream.  Workspaces come from torch's caching allocator.
"""
import ctypes
import os
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import BnrEpi, ConvGeom, IgemmArgs, WgradArgs, call, stream

BF16 = torch.bfloat16


def sdt():
    """16-bit storage dtype of the active library (bf16 or fp16)."""
    return _lib.storage_dtype()


def _p(t):
    """Device address of ``t`` (None -> NULL) as an int: the entry points declare their
    pointer arguments c_void_p and the descriptor structs c_void_p fields, which ctypes
    fills from ints (no c_void_p object per argument on the launch path)."""
    return t.data_ptr() if t is not None else None


class KernelTimer:
    """Brackets kernel launches with HIP events on the launching stream and
    accumulates algorithmic FLOPs per device kernel (bench.py's roofline).
    ``only``: instrument just this kernel name (the others cost nothing)."""

    def __init__(self, only=None, log=False):
        self.rec = {}
        self.rec_main = {}   # the same, launches on the stream current at construction only
        self.main_stream = torch.cuda.current_stream().stream_id if torch.cuda.is_available() else None
        self.only = only
        self.tags = {}       # tag -> {"conv": [(ev0, ev1, flops)], "block": [(ev0, ev1)]}
        self.log = [] if log else None     # per launch: (shape, kernel, ev0, ev1, stream) in issue order

    def wants(self, name):
        return self.only is None or name == self.only

    def block(self, tag):
        """Context manager: events around a whole program block (e.g. one DoubleConv
        forward or backward); conv launches inside are also summed under ``tag``."""
        timer = self

        class _Blk:
            def __enter__(self):
                global TIMER_TAG
                self.prev = TIMER_TAG
                TIMER_TAG = tag
                self.ev = timer.begin()

            def __exit__(self, *exc):
                global TIMER_TAG
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record(torch.cuda.current_stream())
                timer.tags.setdefault(tag, {"conv": [], "block": []})["block"].append((self.ev, ev1))
                TIMER_TAG = self.prev
        return _Blk()

    def tag_summary(self):
        torch.cuda.synchronize()
        out = {}
        for tag, d in self.tags.items():
            cms = sum(a.elapsed_time(b) for a, b, _ in d["conv"])
            cfl = sum(f for _, _, f in d["conv"])
            bms = sum(a.elapsed_time(b) for a, b in d["block"])
            out[tag] = dict(conv_ms=cms, block_ms=bms, flops=cfl,
                            conv_tflops=cfl / (cms * 1e-3) / 1e12 if cms > 0 else 0.0,
                            block_tflops=cfl / (bms * 1e-3) / 1e12 if bms > 0 else 0.0)
        return out

    def begin(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream())
        return ev

    def end(self, ev0, family, flops, desc=None):
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record(torch.cuda.current_stream())
        self.rec.setdefault(family, []).append((ev0, ev1, flops))
        if torch.cuda.current_stream().stream_id == self.main_stream:
            self.rec_main.setdefault(family, []).append((ev0, ev1, flops))
        if self.log is not None:
            self.log.append((desc, family, ev0, ev1, torch.cuda.current_stream().stream_id, flops))
        if TIMER_TAG is not None:
            self.tags.setdefault(TIMER_TAG, {"conv": [], "block": []})["conv"].append((ev0, ev1, flops))

    def summary(self, main_only=False):
        """Per device kernel: launches, summed ms, FLOPs, average us, TF/s (``main_only``: the
        launches on the constructing stream -- the step's compute stream -- only)."""
        torch.cuda.synchronize()
        out = {}
        for fam, items in (self.rec_main if main_only else self.rec).items():
            ms = sum(a.elapsed_time(b) for a, b, _ in items)
            fl = sum(f for _, _, f in items)
            out[fam] = dict(launches=len(items), ms=ms, flops=fl,
                            avg_us=1e3 * ms / len(items), tflops=fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0)
        return out


TIMER = None   # set to a KernelTimer to instrument igemm / wgrad launches
TIMER_TAG = None


def timed_block(tag):
    """KernelTimer.block(tag) when a full (census) timer is active, else a no-op."""
    t = TIMER
    if t is not None and t.only is None:
        return t.block(tag)
    import contextlib
    return contextlib.nullcontext()
_NAMES = {}    # launch signature -> device kernel name (stf_*_kernel_name)


def _kernel_name(fn, key, args):
    n = _NAMES.get(key)
    if n is None:
        n = _NAMES[key] = getattr(_lib.load(), fn)(ctypes.byref(args)).decode()
    return n


@dataclass
class Feat:
    buf: torch.Tensor      # 16-bit storage (bf16 / fp16), >= N*H*W*cs elements
    N: int
    H: int
    W: int
    C: int
    cs: int                # channel stride (elements per pixel)
    off: int = 0           # first channel

    @property
    def M(self):
        return self.N * self.H * self.W

    def ptr(self):
        return self.buf.data_ptr() + 2 * self.off

    def slice(self, c0, c):
        assert 0 <= c0 and c0 + c <= self.C
        return Feat(self.buf, self.N, self.H, self.W, c, self.cs, self.off + c0)

    def check(self):
        b = self.buf
        assert b.dtype == _lib._active and b.is_cuda
        assert b.numel() >= self.N * self.H * self.W * self.cs, "feature buffer too small"
        assert self.off + self.C <= self.cs

    def dense(self):
        """Debug/test view as a [N, C, H, W] float tensor (copies)."""
        v = self.buf[: self.M * self.cs].view(self.N, self.H, self.W, self.cs)
        return v[..., self.off: self.off + self.C].permute(0, 3, 1, 2).float()


# While a launch plan records (stfunet/plan.py): every buffer the step allocates is
# appended here and stays alive with the plan, whose ops hold its address
KEEP = None
RECORDING = False


def empty(shape, dtype, device):
    """torch.empty for the programs' buffers (kept alive while a plan records)."""
    t = torch.empty(shape, dtype=dtype, device=device)
    if KEEP is not None:
        KEEP.append(t)
    return t


def memset0(t):
    """Zero a device tensor's storage with a library launch (plan-recordable)."""
    call("stf_memset", t.data_ptr(), 0, t.numel() * t.element_size(), stream())
    return t


def wait(waiter, waitee):
    """Stream ``waiter`` waits for the work enqueued on ``waitee`` so far (torch Streams;
    an event record + stream wait inside the library, so a recording plan keeps it)."""
    call("stf_stream_wait", waiter.cuda_stream, waitee.cuda_stream)


def copy_rows(src, src_ld, dst, dst_ld, rows, cols):
    """dst[r][:cols] = src[r][:cols] for fp32 row-major tensors (row strides in elements)."""
    assert src.dtype == torch.float32 and dst.dtype == torch.float32
    assert src.numel() >= (rows - 1) * src_ld + cols and dst.numel() >= (rows - 1) * dst_ld + cols
    call("stf_copy_rows", src.data_ptr(), src_ld, dst.data_ptr(), dst_ld, rows, cols, stream())


def new_feat(N, H, W, C, device, cs=None):
    cs = cs or C
    return Feat(empty(N * H * W * cs, sdt(), device), N, H, W, C, cs, 0)


def zeros_feat(N, H, W, C, device, cs=None):
    cs = cs or C
    return Feat(memset0(empty(N * H * W * cs, sdt(), device)), N, H, W, C, cs, 0)


# ------------------------------------------------------------------ packs
def pack_input(x, cpad):
    """x [N, C, H, W] float -> Feat (NHWC bf16, cpad channels, zero padded)."""
    x = x.contiguous().float()
    N, C, H, W = x.shape
    f = new_feat(N, H, W, cpad, x.device)
    call("stf_pack_input", _p(x), N, C, H, W, cpad, f.ptr(), stream())
    return f


class _PackDesc(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p), ("out", ctypes.c_void_p), ("d0", ctypes.c_int), ("d1", ctypes.c_int),
                ("R", ctypes.c_int), ("S", ctypes.c_int), ("mode", ctypes.c_int), ("cpad", ctypes.c_int)]


class PackCache:
    """Persistent bf16 GEMM packings of one model's fp32 master weights.

    The first step packs on demand and records every (weight, layout) request;
    from then on ``refresh()`` (called at the start of each forward, after the
    optimizer step) repacks the whole recorded list with ONE stf_pack_weights
    launch and ``get()`` returns the cached buffers.  Only the owning program
    uses it (``ACTIVE_PACKS`` while its forward/backward runs), and the keys are
    that model's parameters, so a cached packing is never stale."""

    def __init__(self):
        self.bufs = {}
        self.seen = {}
        self.recorded = ()
        self.fresh = set()
        self._desc = None
        self.dtype = None

    def _match_storage(self):
        """The packed buffers are in the storage type of the library that wrote them:
        when the active storage changes, forget them (repacked on demand)."""
        if self.dtype != sdt():
            self.__init__()
            self.dtype = sdt()

    def refresh(self):
        self._match_storage()
        if self.seen:
            self.recorded = tuple(self.seen)
        self.seen = {}
        self.fresh = set()
        if not self.recorded:
            return
        if self._desc is None or self._desc[0] != self.recorded:
            arr = (_PackDesc * len(self.recorded))()
            mx, tiles = 0, 0
            for i, key in enumerate(self.recorded):
                w, buf, mode, cpad = self.bufs[key]
                d0, d1, R, S = w.shape
                arr[i] = _PackDesc(w.data_ptr(), buf.data_ptr(), d0, d1, R, S, mode, cpad)
                mx = max(mx, buf.numel())
                nt = _lib.load().stf_pack_tiles(d0, d1, R, S, mode, cpad)
                tiles = max(tiles, nt) if tiles >= 0 and nt >= 0 else -1
            if os.environ.get("STF_PACK_TILED", "1") == "0":
                tiles = -1
            dev = self.bufs[self.recorded[0]][1].device
            t = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
            self._desc = (self.recorded, t, mx, tiles)
        _, t, mx, tiles = self._desc
        if KEEP is not None:       # a recording plan's pack launch reads these
            KEEP.append(t)
            KEEP.extend(self.bufs[k][1] for k in self.recorded)
        if tiles > 0:           # LDS-tiled transposes (every descriptor qualifies)
            call("stf_pack_weights_tiled", _p(t), len(self.recorded), tiles, stream())
        else:
            call("stf_pack_weights", _p(t), len(self.recorded), mx, stream())
        self.fresh = set(self.recorded)

    def get(self, w, mode, cpad):
        if self.dtype is not _lib._active:
            self._match_storage()
        key = (w.data_ptr(), w.shape, mode, cpad)
        self.seen[key] = None
        ent = self.bufs.get(key)
        if ent is None:
            w = w.detach()
            ent = self.bufs[key] = (w, _pack_into(w, mode, cpad, None, launch=False), mode, cpad)
        if key not in self.fresh:
            _pack_into(w, mode, cpad, ent[1])
            self.fresh.add(key)
        if KEEP is not None:
            KEEP.append(ent[1])
        return ent[1]


ACTIVE_PACKS = None    # the running program's PackCache (None: pack on every call)


def _pack_into(w, mode, cpad, out, launch=True):
    assert w.dtype == torch.float32 and w.is_contiguous()
    d0, d1, R, S = w.shape
    n = d0 * R * S * cpad if mode == 0 else d0 * d1 * R * S
    if out is None:
        out = torch.empty(n, dtype=sdt(), device=w.device)
    if launch:
        call("stf_pack_weight", _p(w), d0, d1, R, S, mode, cpad, _p(out), stream())
    return out


def pack_weight(w, mode, cpad=0, cache=True):
    """fp32 master weight -> 16-bit GEMM rows (modes: include/stfunet.h); served
    from the active program's PackCache when one is running.  ``cache=False`` for
    per-call temporaries (a zero-padded copy of a weight): the PackCache keys by
    address and would keep every dead temporary alive."""
    if cache and ACTIVE_PACKS is not None:
        return ACTIVE_PACKS.get(w, mode, cpad)
    w = w.detach()
    assert w.dtype == torch.float32 and w.is_contiguous()
    d0, d1, R, S = w.shape
    n = d0 * R * S * cpad if mode == 0 else d0 * d1 * R * S
    out = empty(n, sdt(), w.device)
    call("stf_pack_weight", _p(w), d0, d1, R, S, mode, cpad, _p(out), stream())
    return out


# ------------------------------------------------------------------ implicit GEMM
_QUERIES = {}    # igemm launch signature -> (statistics / BN-backward tiles, split-K workspace bytes)
_PLANS = {}      # wgrad launch signature -> (splits, workspace bytes)


def _ws_bytes_with(a, want_stats):
    """stf_igemm_ws_bytes with the statistics pointer set (non-NULL) as it will be at launch."""
    if want_stats:
        a.stats = 16
    try:
        return _lib.load().stf_igemm_ws_bytes(ctypes.byref(a))
    finally:
        a.stats = None


def _geom(src: Feat, Hd, Wd, R, S, stride, pad, transposed):
    return ConvGeom(src.N, src.H, src.W, src.C, src.cs, Hd, Wd, R, S, stride, pad, int(transposed))


def igemm(src: Feat, wgt, nout, dst: Feat, R, S, stride, pad, transposed=False, bias=None,
          want_stats=False, scatter2x2=False, groups=1, accumulate=False, lstm=None, bnr=None):
    """Launch stf_igemm; returns the per-tile stats tensor (or None) and tiles per group.
    ``bnr`` = (y, BNState, relu): dst is dz = d act(BN(y)); the launch also produces the
    BN-backward partial sums (stf_bnr_epi), returned in place of the stats."""
    src.check()
    dst.check()
    Hd, Wd = (dst.H // 2, dst.W // 2) if scatter2x2 else (dst.H, dst.W)
    assert dst.N == src.N and src.N % groups == 0
    if lstm is None:
        assert dst.C == (nout // 4 if scatter2x2 else nout)
    assert wgt.dtype == sdt() and wgt.numel() == nout * R * S * src.C
    if transposed:
        assert stride in (1, 2)
    else:
        # every gathered tap must stay inside (or be zero padding of) the source
        assert (Hd - 1) * stride - pad + R - 1 <= src.H - 1 + pad
    M = src.N * Hd * Wd
    dptr = dst.ptr()
    a = IgemmArgs(_geom(src, Hd, Wd, R, S, stride, pad, transposed), src.ptr(), _p(wgt), nout, dptr,
                  dst.cs, _p(bias), None, int(scatter2x2), M // groups if groups > 1 else 0, int(accumulate),
                  ctypes.pointer(lstm) if lstm is not None else None)
    # the size queries below are pure functions of the launch signature (geometry, flags,
    # which optional pointers are set, the destination's 16-B alignment): asked once each
    qkey = (src.N, src.H, src.W, src.C, src.cs, Hd, Wd, R, S, stride, pad, transposed, nout, dst.cs,
            bias is None, scatter2x2, groups, accumulate, None if lstm is None else lstm.backward,
            bnr is not None, want_stats, dptr & 15)
    q = _QUERIES.get(qkey)
    stats, tiles = None, 0
    if bnr is not None:
        y, st, relu = bnr
        y.check()
        assert not want_stats and st.groups == groups and (y.N, y.H, y.W, y.C) == (dst.N, dst.H, dst.W, dst.C)
        epi = BnrEpi(y.ptr(), y.cs, _p(st.scale), _p(st.shift), _p(st.mean), _p(st.invstd), int(relu), None)
        a.bnr = ctypes.pointer(epi)
    if q is None:
        lib = _lib.load()
        tq = 0
        if bnr is not None:
            tq = lib.stf_igemm_bnr_tiles(ctypes.byref(a))
        elif want_stats:
            tq = lib.stf_igemm_stat_tiles(ctypes.byref(a))
        q = _QUERIES[qkey] = (tq, _ws_bytes_with(a, want_stats))
    tiles, nb = q
    if bnr is not None:
        stats = empty(groups * tiles * 2 * nout, torch.float32, dst.buf.device)
        epi.partial = stats.data_ptr()
    if want_stats:
        stats = empty(groups * tiles * 2 * nout, torch.float32, dst.buf.device)
        a.stats = stats.data_ptr()
    t = TIMER
    if t is not None:
        name = _kernel_name("stf_igemm_kernel_name", ("i", src.N, src.H, src.W, src.C, Hd, Wd, nout, R, S, stride,
                                                      pad, transposed, scatter2x2, lstm is not None, groups,
                                                      bnr is not None, want_stats), a)
        if not t.wants(name):
            t = None
    ws = None
    if nb:
        ws = empty(nb // 4, torch.float32, dst.buf.device)
        a.ws = ws.data_ptr()
    ev = t.begin() if t is not None else None
    if RECORDING:        # name the launch range for the plan's timed replays (bench roofline)
        _plan_tag(a, "stf_igemm_kernel_name",
                  ("i", src.N, src.H, src.W, src.C, Hd, Wd, nout, R, S, stride, pad, transposed, scatter2x2,
                   lstm is not None, groups, bnr is not None, want_stats),
                  2.0 * src.N * Hd * Wd * nout * R * S * src.C / (stride * stride if transposed else 1))
    call("stf_igemm", ctypes.byref(a), stream())
    if RECORDING:
        call("stf_plan_tag_end")
    if t is not None:
        macs = src.N * Hd * Wd * nout * R * S * src.C
        t.end(ev, name, 2.0 * macs / (stride * stride if transposed else 1),
              f"igemm M={src.N * Hd * Wd} N={nout} K={R * S * src.C} {R}x{S}/s{stride}{' T' if transposed else ''}"
              f"{' lstm' if lstm is not None else ''}{' bnr' if bnr is not None else ''}")
    return stats, tiles


def _plan_tag(a, fn, key, flops):
    call("stf_plan_tag", _kernel_name(fn, key, a).encode(), float(flops))


def conv_dgrad(dy: Feat, w, dx: Feat, R, S, stride, pad, accumulate=False, bnr=None, cache=True, want_stats=False):
    """Conv2d input gradient: stride 1 runs as a forward gather over flipped taps
    (pack mode 5, pad' = R-1-pad); strided convs use the transposed gather.
    ``accumulate``: dx += gradient (residual / multi-consumer tensors).
    ``bnr`` = (y, BNState, relu): dx feeds the backward of act(BN(y)); returns the
    fused partial sums and tiles for bn_backward_fused.  ``cache=False``: ``w`` is a per-call
    temporary (pack_weight).  ``want_stats``: also the per-tile (sum, sum of squares) rows of the
    stored dx (stride-1 only; stat_sums folds columns of them)."""
    groups = bnr[1].groups if bnr is not None else 1
    if stride == 1 and 2 * pad == R - 1 and R == S:
        return igemm(dy, pack_weight(w, 5, cache=cache), dx.C, dx, R, S, 1, R - 1 - pad, accumulate=accumulate,
                     bnr=bnr, groups=groups, want_stats=want_stats)
    assert not want_stats
    return igemm(dy, pack_weight(w, 1, cache=cache), dx.C, dx, R, S, stride, pad, transposed=True,
                 accumulate=accumulate,
                 bnr=bnr, groups=groups)


def rows(f: Feat, n0, n):
    """Images [n0, n0+n) of a Feat (same H, W, channel slice)."""
    return Feat(f.buf[n0 * f.H * f.W * f.cs:], n, f.H, f.W, f.C, f.cs, f.off)


WGRAD_STREAM = None   # set by a program: weight gradients run there, off the critical path
_STREAMS = {}


def side_stream(device, name):
    """The process's side stream ``name`` on ``device``: the programs' side streams, the
    weight-gradient stream and the DDP joiner, one each per process however many programs are
    built.  High priority: HIP puts high-priority streams in a hardware-queue pool of their own,
    so a side stream never shares (and is never serialized behind) the caller's compute stream's
    queue, whatever streams the process made before -- e.g. RCCL's, which shifted the STF side
    streams onto the compute stream's queue (STF_SIDE_PRIO=0: normal priority, A/B)."""
    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    key = (dev.index, name)
    st = _STREAMS.get(key)
    if st is None:
        st = _STREAMS[key] = torch.cuda.Stream(device=dev, priority=_SIDE_PRIO)
    return st


_SIDE_PRIO = int(os.environ.get("STF_SIDE_PRIO", "-1"))


def wgrad_side_stream(device):
    """The stream a program's backward sends its weight gradients to, beside the dgrad /
    BatchNorm chain that carries the critical path (one per device; STF_WGRAD_SIDE=0:
    inline, for A/B measurements)."""
    if os.environ.get("STF_WGRAD_SIDE", "1") == "0":
        return None
    return side_stream(device, "wgrad")


def wgrad(dy: Feat, x: Feat, R, S, stride, pad, out, defer=True):
    """Weight gradient into ``out`` (fp32, [dy.C][x.C][R][S] contiguous view).  With
    ``WGRAD_STREAM`` set and ``defer``, the launches go to that stream after the current
    stream's work so far (dy, x complete); the program joins it before ``out`` is read
    (``defer=False``: ``out`` is consumed right away on the current stream)."""
    side = WGRAD_STREAM if defer else None
    if side is not None:
        # host fast path (the STF step issues ~55 of these and is host-bound): one pooled
        # event instead of wait_stream's fresh Event, torch's current stream switched by id
        main = WGRAD_MAIN
        if main is None or _lib.stream() != main.cuda_stream:   # e.g. called on another side stream
            main = torch.cuda.current_stream()
        call("stf_stream_wait", side.cuda_stream, main.cuda_stream)
        dy.buf.record_stream(side)
        x.buf.record_stream(side)
        _set_stream(side)
        try:
            # one workgroup per CU beside the critical path (two per CU inline): the
            # fused kernel's two 250-register waves per SIMD would leave the dgrad /
            # BatchNorm chain no registers on any CU (STF cfg3 11.3-11.5 vs 11.8-12.3 ms)
            return _wgrad(dy, x, R, S, stride, pad, out, _num_cus(dy.buf.device))
        finally:
            _set_stream(main)
    return _wgrad(dy, x, R, S, stride, pad, out)


WGRAD_MAIN = None     # the program's main stream while WGRAD_STREAM is set


def _set_stream(s):
    torch._C._cuda_setStream(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)


_CUS = {}


def _num_cus(device):
    n = _CUS.get(device)
    if n is None:
        n = torch.cuda.get_device_properties(device).multi_processor_count
        _CUS[device] = n
    return n


def _wgrad(dy: Feat, x: Feat, R, S, stride, pad, out, grid_blocks=0):
    dy.check()
    x.check()
    assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() == dy.C * x.C * R * S
    g = ConvGeom(x.N, x.H, x.W, x.C, x.cs, dy.H, dy.W, R, S, stride, pad, 0)
    a = WgradArgs(g, dy.ptr(), dy.cs, dy.C, x.ptr(), None, 0, grid_blocks)
    pkey = (x.N, x.H, x.W, x.C, x.cs, dy.H, dy.W, dy.C, dy.cs, R, S, stride, pad, grid_blocks)
    plan = _PLANS.get(pkey)
    if plan is None:       # stf_wgrad_plan is a pure function of the geometry and grid request
        splits = ctypes.c_int(0)
        nbytes = ctypes.c_size_t(0)
        call("stf_wgrad_plan", ctypes.byref(a), ctypes.byref(splits), ctypes.byref(nbytes))
        plan = _PLANS[pkey] = (splits.value, nbytes.value)
    splits, nbytes = plan
    ws = empty(nbytes // 4, torch.float32, out.device)
    a.ws = ws.data_ptr()
    a.splits = splits
    t = TIMER
    if t is not None:
        name = _kernel_name("stf_wgrad_kernel_name", ("w", x.N, x.H, x.W, x.C, dy.H, dy.W, dy.C, R, S, stride, pad), a)
        if not t.wants(name):
            t = None
    ev = t.begin() if t is not None else None
    if RECORDING:
        _plan_tag(a, "stf_wgrad_kernel_name", ("w", x.N, x.H, x.W, x.C, dy.H, dy.W, dy.C, R, S, stride, pad),
                  2.0 * dy.M * dy.C * R * S * x.C)
    call("stf_wgrad", ctypes.byref(a), stream())
    if RECORDING:
        call("stf_plan_tag_end")
    if t is not None:
        t.end(ev, name, 2.0 * dy.M * dy.C * R * S * x.C,
              f"wgrad M={dy.M} N={dy.C} K={R * S * x.C} {R}x{S}/s{stride} splits={splits}")
    call("stf_wgrad_reduce", ws.data_ptr(), splits, dy.C, R, S, x.C, out.data_ptr(), stream())


def stat_sums(stats, tiles, nout, c0, C, out):
    """out[c] = sum of column c0 + c of the sum half of igemm statistics rows [tiles][2][nout]."""
    assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() == C
    call("stf_stat_sums", _p(stats), tiles, nout, c0, C, _p(out), stream())


def channel_sum(x: Feat, out):
    x.check()
    tiles = min(1024, max(1, (x.M * (x.C // 8) + 255) // 256))
    part = empty(tiles * x.C, torch.float32, out.device)
    call("stf_channel_sum", x.ptr(), x.cs, x.M, x.C, _p(part), _p(out), stream())


# ------------------------------------------------------------------ BatchNorm
class BNState:
    """Per-forward BatchNorm quantities ([groups][C] each) kept for backward."""
    __slots__ = ("mean", "invstd", "scale", "shift", "M", "groups", "training")

    def __init__(self, C, device, M, groups=1, training=True):
        t = empty((4, groups, C), torch.float32, device)
        self.mean, self.invstd, self.scale, self.shift = t.unbind(0)
        self.M = M
        self.groups = groups
        # training: normalised with the batch statistics (mean / invstd above); eval:
        # with the running statistics, which the backward treats as constants
        self.training = training

    @staticmethod
    def identity(C, device):
        st = BNState(C, device, 0, 1)
        st.mean.zero_()
        st.invstd.fill_(1.0)
        st.scale.fill_(1.0)
        st.shift.zero_()
        return st


# num_batches_tracked increments are deferred and applied per forward with one
# multi-tensor launch per increment value (instead of one tiny kernel per module)
_NBT_PENDING = {}
_RUN_PENDING = []      # (stf_bn_run_desc, (stats slab, running_mean, running_var) kept alive until the flush)
_GSUM_PENDING = []     # (stf_bn_gsum_desc, partial slab)


class _RunDesc(ctypes.Structure):
    _fields_ = [("stats", ctypes.c_void_p), ("running_mean", ctypes.c_void_p), ("running_var", ctypes.c_void_p),
                ("Mg", ctypes.c_int64), ("tiles", ctypes.c_int), ("groups", ctypes.c_int), ("C", ctypes.c_int),
                ("momentum", ctypes.c_float)]


class _GsumDesc(ctypes.Structure):
    _fields_ = [("partial", ctypes.c_void_p), ("dgamma", ctypes.c_void_p), ("dbeta", ctypes.c_void_p),
                ("tiles", ctypes.c_int), ("groups", ctypes.c_int), ("C", ctypes.c_int)]


def flush_batches_tracked():
    """End of a training forward: the deferred running-statistics updates of the
    grouped BatchNorms (one stf_bn_running_batch launch) and num_batches_tracked."""
    if _RUN_PENDING:
        arr = (_RunDesc * len(_RUN_PENDING))(*[d for d, _ in _RUN_PENDING])
        call("stf_bn_running_batch", arr, len(_RUN_PENDING), stream())
        _RUN_PENDING.clear()
    for inc, ts in _NBT_PENDING.items():
        arr = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
        call("stf_i64_add_batch", arr, len(ts), inc, stream())
    _NBT_PENDING.clear()


def flush_bn_grads():
    """dgamma/dbeta of the grouped BatchNorm backwards run so far (one
    stf_bn_groupsum_batch launch); call before those gradients are read."""
    if _GSUM_PENDING:
        arr = (_GsumDesc * len(_GSUM_PENDING))(*[d for d, _ in _GSUM_PENDING])
        call("stf_bn_groupsum_batch", arr, len(_GSUM_PENDING), stream())
        _GSUM_PENDING.clear()


def bn_finalize(stats, tiles, bn, M, training, groups=1):
    """``bn`` is the nn.BatchNorm2d holding weight/bias/running stats (its
    num_batches_tracked advances by ``groups`` at flush_batches_tracked())."""
    C = bn.num_features
    st = BNState(C, bn.weight.device, M, groups, training)
    mom = 0.1 if bn.momentum is None else bn.momentum
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    if training and groups > 1 and rm is not None:
        # grouped: (mean, var) of every group stay parked in the slab; the running
        # stats advance group by group in ONE batched launch at the end of forward
        _RUN_PENDING.append((_RunDesc(stats.data_ptr(), rm.data_ptr(), rv.data_ptr(), M // groups, tiles, groups, C,
                                      float(mom)), (stats, rm, rv)))
        rm = rv = None
    call("stf_bn_finalize", _p(stats) if training else None, tiles, groups, C, M, bn.weight.data_ptr(),
         bn.bias.data_ptr(), float(mom), float(bn.eps), _p(rm) if rm is not None else None,
         _p(rv) if rv is not None else None, _p(st.mean), _p(st.invstd), _p(st.scale), _p(st.shift),
         stream())
    if training and bn.track_running_stats:
        _NBT_PENDING.setdefault(groups, []).append(bn.num_batches_tracked)
    return st


def bn_act(y: Feat, st: BNState, out: Feat, relu=True, pooled: Feat = None, res: Feat = None,
           res_st: BNState = None):
    """out = act(BN(y) [+ res | + BN_res(res)]) (+ 2x2 max pool into ``pooled``)."""
    y.check()
    out.check()
    assert (y.N, y.H, y.W, y.C) == (out.N, out.H, out.W, out.C)
    if pooled is not None:
        pooled.check()
        assert pooled.cs == pooled.C and pooled.off == 0 and (pooled.H, pooled.W) == (y.H // 2, y.W // 2)
    if res is not None:
        res.check()
        assert (res.N, res.H, res.W, res.C) == (y.N, y.H, y.W, y.C)
    call("stf_bn_act", y.ptr(), y.cs, y.N, y.H, y.W, y.C, st.groups, _p(st.scale), _p(st.shift), int(relu),
         res.ptr() if res is not None else None, res.cs if res is not None else 0,
         _p(res_st.scale) if res_st is not None else None, _p(res_st.shift) if res_st is not None else None,
         out.ptr(), out.cs, pooled.ptr() if pooled is not None else None, stream())


def bn_backward(y: Feat, st: BNState, bn, dgamma, dbeta, dz: Feat = None, dpool: Feat = None, relu=True,
                dbias=None, mask: Feat = None, out: Feat = None, keep_g=False):
    """Gradient of act(BN(y)) [+ maxpool] w.r.t. y; returns dy as a Feat.

    ``dz``: grad w.r.t. the BN(+ReLU) output (may be a concat slice);
    ``dpool``: grad w.r.t. its 2x2 max-pooled output; ``mask``: take the ReLU
    mask from this saved output instead of recomputing it (ReLU after a
    residual add).  ``relu=False`` and no mask: plain BN backward.
    dgamma/dbeta/dbias: fp32 views in the flat gradient buffer (dbias = bias of
    the producing conv).  ``out``: optional destination Feat for dy.
    ``keep_g``: return (dy, g) with g = the masked incoming gradient (the
    residual-shortcut gradient of a block whose ReLU follows the add).
    """
    y.check()
    C = y.C
    dev = y.buf.device
    G = st.groups
    tiles = _lib.load().stf_bn_bwd_tiles(y.N, y.H, y.W, C, G, int(dpool is not None))
    part = empty(G * tiles * 2 * C, torch.float32, dev)
    if dz is not None:
        dz.check()
        assert (dz.N, dz.H, dz.W, dz.C) == (y.N, y.H, y.W, C)
    if dpool is not None:
        dpool.check()
        assert dpool.cs == C and dpool.off == 0 and (dpool.H, dpool.W) == (y.H // 2, y.W // 2)
    mode = 2 if mask is not None else (1 if relu else 0)
    if mask is not None:
        mask.check()
    # without pooling / saved mask / a caller that needs it, the masked gradient is
    # never stored: the apply pass re-reads dz and recomputes the ReLU mask from y
    direct = dpool is None and mode != 2 and not keep_g
    g = None if direct else new_feat(y.N, y.H, y.W, C, dev)
    call("stf_bn_bwd_reduce", dz.ptr() if dz is not None else None, dz.cs if dz is not None else 0,
         dpool.ptr() if dpool is not None else None, y.ptr(), y.cs, y.N, y.H, y.W, C, G, _p(st.scale),
         _p(st.shift), _p(st.mean), _p(st.invstd), mode, mask.ptr() if mask is not None else None,
         mask.cs if mask is not None else 0, g.ptr() if g is not None else None, _p(part), stream())
    if keep_g and out is None:
        out = new_feat(y.N, y.H, y.W, C, dev)
    if direct:
        if out is None:
            out = new_feat(y.N, y.H, y.W, C, dev)
        dy = bn_backward_from_partial(dz, y, st, bn, part, tiles, dgamma, dbeta, dbias, out=out,
                                      mask_relu=(mode == 1))
    else:
        dy = bn_backward_from_partial(g, y, st, bn, part, tiles, dgamma, dbeta, dbias, out=out)
    return (dy, g) if keep_g else dy


def bn_backward_fused(dz: Feat, y: Feat, st: BNState, bn, part, tiles, dgamma, dbeta, dbias=None, relu=True):
    """Backward of act(BN(y)) when the producer of dz (conv_dgrad with ``bnr``) already
    reduced the partial sums: finalize + apply, dy written over dz."""
    assert dz.cs == dz.C and dz.off == 0
    return bn_backward_from_partial(dz, y, st, bn, part, tiles, dgamma, dbeta, dbias, out=dz if relu else None,
                                    mask_relu=relu)


def bn_backward_maxpool3(y: Feat, st: BNState, bn, dgamma, dbeta, argmax, dpool: Feat):
    """Backward of maxpool3s2(relu(BN(y))) w.r.t. y (the STF stem): the pooled gradient is
    routed by the forward's argmax inside the reduce and apply passes (stf_bn_bwd_*_pool3),
    never materialized at full size.  Returns dy."""
    y.check()
    dpool.check()
    C, dev, G = y.C, y.buf.device, st.groups
    assert y.cs == C and y.off == 0 and dpool.cs == C and dpool.off == 0
    assert (dpool.N, dpool.H, dpool.W) == (y.N, (y.H - 1) // 2 + 1, (y.W - 1) // 2 + 1)
    tiles = _lib.load().stf_bn_bwd_tiles(y.N, y.H, y.W, C, G, 0)
    part = empty(G * tiles * 2 * C, torch.float32, dev)
    call("stf_bn_bwd_reduce_pool3", _p(argmax), dpool.ptr(), y.ptr(), y.N, y.H, y.W, C, G, _p(st.scale),
         _p(st.shift), _p(st.mean), _p(st.invstd), _p(part), stream())
    coef = _bn_bwd_coef(y, st, bn, part, tiles, dgamma, dbeta)
    dy = new_feat(y.N, y.H, y.W, C, dev)
    call("stf_bn_bwd_apply_pool3", _p(argmax), dpool.ptr(), y.ptr(), y.N, y.H, y.W, C, G, _p(st.scale),
         _p(st.shift), _p(coef), dy.ptr(), stream())
    return dy


def _bn_bwd_coef(y: Feat, st: BNState, bn, part, tiles, dgamma, dbeta):
    """stf_bn_bwd_finalize: dy = A g + B y + C coefficients [G][3][C] from the partial sums
    (dgamma / dbeta written, or parked for flush_bn_grads when grouped; eval mode: A only)."""
    C, dev, G = y.C, y.buf.device, st.groups
    coef = empty(G * 3 * C, torch.float32, dev)
    if G > 1 and (dgamma is not None or dbeta is not None):
        _GSUM_PENDING.append((_GsumDesc(part.data_ptr(), dgamma.data_ptr() if dgamma is not None else None,
                                        dbeta.data_ptr() if dbeta is not None else None, tiles, G, C), part))
        dgamma = dbeta = None
    call("stf_bn_bwd_finalize", _p(part), tiles, G, C, y.M, bn.weight.data_ptr(), _p(st.mean),
         _p(st.invstd), _p(dgamma), _p(dbeta), _p(coef), stream())
    if not st.training:
        cv = coef.view(G, 3, C)
        cv[:, 0].copy_(bn.weight.detach() * st.invstd)
        cv[:, 1:].zero_()
    return coef


def bn_backward_from_partial(g: Feat, y: Feat, st: BNState, bn, part, tiles, dgamma, dbeta, dbias=None,
                             out: Feat = None, mask_relu=False):
    """Finalize + apply.  ``mask_relu``: g is the raw incoming gradient and the
    ReLU mask is recomputed from y with the forward affine (g is not written)."""
    C = y.C
    dev = y.buf.device
    G = st.groups
    if st.training:
        # the bias of a conv feeding a training-mode BatchNorm has gradient exactly 0:
        # sum_m dy_m = gamma * invstd * (sum g - M mean(g) - mean(g xhat) sum xhat) and
        # sum xhat = 0 over the normalised batch -- left at the zero of the fresh flat
        # gradient instead of summing the rounded dy (the reference's autograd returns
        # fp32 noise around 0 there)
        dbias = None
    coef = empty(G * 3 * C, torch.float32, dev)
    if G > 1 and (dgamma is not None or dbeta is not None):
        # grouped: the per-group sums stay parked; flush_bn_grads() adds them up for
        # every pending BatchNorm in one launch
        _GSUM_PENDING.append((_GsumDesc(part.data_ptr(), dgamma.data_ptr() if dgamma is not None else None,
                                        dbeta.data_ptr() if dbeta is not None else None, tiles, G, C), part))
        dgamma = dbeta = None
    call("stf_bn_bwd_finalize", _p(part), tiles, G, C, y.M, bn.weight.data_ptr(), _p(st.mean),
         _p(st.invstd), _p(dgamma), _p(dbeta), _p(coef), stream())
    if not st.training:
        # eval mode (running statistics are constants): dy = gamma * invstd * g, i.e. the
        # apply pass's dy = A g + B y + C with B = C = 0; dgamma = sum g xhat and
        # dbeta = sum g come out of the same partial sums as in training mode
        cv = coef.view(G, 3, C)
        cv[:, 0].copy_(bn.weight.detach() * st.invstd)
        cv[:, 1:].zero_()
    bpart = None
    if dbias is not None:
        bpart = empty(_lib.load().stf_bn_bwd_apply_tiles(y.M, C) * C, torch.float32, dev)
    dst = out if out is not None else g
    if out is not None:
        out.check()
        assert (out.N, out.H, out.W, out.C) == (y.N, y.H, y.W, C)
    if mask_relu:
        assert out is not None
    call("stf_bn_bwd_apply", g.ptr(), g.cs, y.ptr(), y.cs, y.M, C, G, _p(st.scale) if mask_relu else None,
         _p(st.shift) if mask_relu else None, _p(coef), dst.ptr(), dst.cs, _p(bpart), _p(dbias), stream())
    return dst
