"""Native step runtime: a program's forward / backward recorded once, replayed from C++.

The reference's training step is Python issuing PyTorch ops layer by layer (and, in
``STFLSTMUNet``, time step by time step: ``src/stf_lstm_unet.py:168-254``).  The
programs here (``UNetProgram``, ``STFProgram``) issue the same step as a schedule of
C-ABI calls from Python: ~500 calls / ~600 launches per STF step, ~7 ms of host time
(DESIGN.md section 5).  ``StepRuntime`` takes that Python out of the steady state:

  * the first ``warm`` training steps of a shape run the schedule eagerly (the weight
    pack list, the size queries and the code objects settle);
  * the next one RECORDS it: the schedule runs as usual while the library appends every
    launch, memset, device copy and cross-stream wait -- with its final arguments -- to
    a native plan (``stf_plan_record``, csrc/plan.hip); every buffer the step allocates
    is kept alive by the runtime (``nhwc.KEEP``, from a private memory pool), so no
    address the plan holds is ever handed to anyone else;
  * later steps copy the input (and, in backward, the incoming logits gradient) into the
    recorded static buffers and replay the plan with one C call per segment
    (``stf_plan_replay``): the same kernels, streams, events and buffers, bit for bit
    the eager step's results.  Backward segments end where the data-parallel hook must
    see a finished gradient bucket (``grad_ready_hook``), which runs live in Python.

Anything that changes what the step would launch -- shapes, train / eval, storage
dtype, the current stream, parameter or buffer addresses, the gradient buffer, a DDP
hook appearing, a scalar baked into a recorded launch (BatchNorm momentum / eps, the
``STF_*`` environment switches the schedule reads per call, the programs' own knobs such as
the LSTM spin limit) -- changes the signature and the plan is recorded again.

Pool lifetime: a recorded entry's private ``MemPool`` is never destroyed implicitly.  When an
entry dies (evicted, its runtime closed, or its program collected -- by refcount or by the
cyclic GC, at a moment the allocator does not choose) its pool moves to a graveyard that is
emptied only at safe points, when no recording's pool context is open in any thread: torch
refuses to destroy a pool while any ``use_mem_pool`` context is active (an exception inside a
destructor, i.e. an abort).  The forward
returns the recorded (static) logits tensor, as a captured graph does: a step's logits
are overwritten by the next step's forward.

``STF_PLAN=0`` keeps every step eager (A/B, debugging); ``STF_PLAN_WARM`` sets the
number of eager steps before recording (default 1).
"""
import contextlib
import ctypes
import gc
import os
import threading
import weakref
from collections import OrderedDict

import torch

from . import _lib, nhwc
from ._lib import call

TIMED = None           # kernel name whose ranges replays bracket with HIP events (bench.py)
RECORD_HOOK = None     # tests: called inside every recording, with its pool context open

# ---------------------------------------------------------------- pool lifetime
_POOL_LOCK = threading.RLock()
_POOL_ACTIVE = 0       # recording pool contexts open in this process (any thread)
_GRAVEYARD = []        # released pools, destroyed by drain_pools() at a safe point


POOL_EVENTS = {"buried": 0, "destroyed": 0, "entry_del": 0}   # counters (tests)


def _bury(pool):
    if pool is not None:
        with _POOL_LOCK:
            _GRAVEYARD.append(pool)
            POOL_EVENTS["buried"] += 1


def drain_pools():
    """Destroy the released pools if no recording's pool context is open (else leave them
    for the next safe point).  Holding the lock keeps another thread from opening one
    meanwhile; a destructor that releases more pools re-enters (RLock) and appends them to the
    fresh list."""
    with _POOL_LOCK:
        if _POOL_ACTIVE or not _GRAVEYARD:
            return
        dead = _GRAVEYARD[:]
        _GRAVEYARD.clear()
        POOL_EVENTS["destroyed"] += len(dead)
        dead.clear()


@contextlib.contextmanager
def _pool_context(pool):
    """torch.cuda.use_mem_pool(pool), counted, so that no pool is destroyed while it is open."""
    global _POOL_ACTIVE
    if pool is None:
        yield
        return
    with _POOL_LOCK:
        _POOL_ACTIVE += 1
    try:
        with torch.cuda.use_mem_pool(pool):
            yield
    finally:
        with _POOL_LOCK:
            _POOL_ACTIVE -= 1
        drain_pools()


def _stf_env():
    """The STF_* environment as a sorted tuple.  Read from os.environ's underlying bytes dict where
    CPython has one: decoding every variable through the os.environ mapping took ~95 us per step
    (97 variables), spent at the step boundary where the GPU waits for the forward replay."""
    data = getattr(os.environ, "_data", None)
    if isinstance(data, dict):
        return tuple(sorted((k, v) for k, v in data.items() if k.startswith(b"STF_")))
    return tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("STF_")))


def enabled():
    # inside a caller's HIP-graph capture the eager launches are what gets captured
    return os.environ.get("STF_PLAN", "1") != "0" and not torch.cuda.is_current_stream_capturing()


class Plan:
    """One recorded launch sequence (a ``stf_plan``) in the active storage's library."""

    def __init__(self):
        self.lib = _lib.load()
        self.h = self.lib.stf_plan_create()
        if not self.h:
            raise MemoryError("stf_plan_create failed")
        self.n = 0

    def record(self, fn):
        _lib.check(self.lib.stf_plan_record(self.h), "stf_plan_record")
        nhwc.RECORDING = True
        try:
            return fn()
        finally:
            nhwc.RECORDING = False
            _lib.check(self.lib.stf_plan_stop(), "stf_plan_stop")
            self.n = self.lib.stf_plan_size(self.h)

    def size(self):
        return self.lib.stf_plan_size(self.h)

    def replay(self, first=0, last=None):
        last = self.n if last is None else last
        if last > first:
            tag = TIMED.encode() if TIMED is not None else None
            _lib.check(self.lib.stf_plan_replay(self.h, first, last, tag), "stf_plan_replay")

    def timing(self):
        """(launches, ms, flops) of the TIMED ranges replayed since the last call (syncs)."""
        n, ms, fl = ctypes.c_int(0), ctypes.c_double(0.0), ctypes.c_double(0.0)
        _lib.check(self.lib.stf_plan_timing(self.h, ctypes.byref(n), ctypes.byref(ms), ctypes.byref(fl)),
                   "stf_plan_timing")
        return n.value, ms.value, fl.value

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h:
            self.lib.stf_plan_destroy(h)


@contextlib.contextmanager
def _no_gc():
    """No cyclic garbage collection while a recording runs.  Belt and braces only: pools no
    longer die inside a collection (``_Entry.__del__`` hands them to the graveyard, see the
    module docstring); this just keeps a long collection out of the recorded step."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def _new_pool():
    """A private memory pool for the recorded step's buffers (a backstop behind
    ``nhwc.KEEP``: nothing outside the plan can ever be given one of its blocks)."""
    if os.environ.get("STF_PLAN_POOL", "1") == "0" or not hasattr(torch.cuda, "MemPool"):
        return None
    return torch.cuda.MemPool()


class _Entry:
    """One signature's recorded step: its plans, static buffers and private pool."""

    def __init__(self):
        self.seen = 0
        self.fwd = self.bwd = None
        self.x = self.logits = self.S = None
        self.bsig = None
        self.dl = None
        self.marks = []
        self.keep = []
        self.bkeep = []
        self.pool = None
        self.owner = None      # weakref to the autograd ctx holding the static S until its backward

    def release(self):
        """Drop the plans and buffers; the pool goes to the graveyard (drain_pools)."""
        pool, self.pool = self.pool, None
        self.fwd = self.bwd = None
        self.x = self.logits = self.S = self.dl = None
        self.keep, self.bkeep = [], []
        _bury(pool)

    def __del__(self):
        # by refcount or inside a cyclic collection, possibly while another recording's pool
        # context is open: never destroy the pool here
        POOL_EVENTS["entry_del"] += 1
        pool = getattr(self, "pool", None)
        if pool is not None:
            self.pool = None
            _bury(pool)

    def busy(self):
        """The static buffers still belong to an earlier forward whose backward has not run
        (two forwards before their backwards): a new forward must not overwrite them."""
        o = self.owner() if self.owner is not None else None
        return o is not None and self.S is not None and getattr(o, "saved", None) is self.S


class StepRuntime:
    """Plan cache of one program (UNetProgram / STFProgram): per signature the training step's
    forward and backward, recorded at the ``warm``-th step of that signature and replayed after.
    Up to ``STF_PLAN_SLOTS`` (default 2) signatures stay recorded, least recently used evicted:
    an epoch's smaller last batch gets its own plan instead of throwing away the full batch's."""

    def __init__(self, prog):
        # a weak back-pointer: program -> runtime -> entries is the only ownership chain, so a
        # dropped program's plans and pools go at a known point (its refcount), not in a cycle
        self._prog = weakref.ref(prog)
        self._bns = None
        self.warm = int(os.environ.get("STF_PLAN_WARM", "1"))
        self.slots = max(1, int(os.environ.get("STF_PLAN_SLOTS", "2")))
        self._bufs = None
        self.entries = OrderedDict()
        self.cur = None         # entry of the last planned forward

    @property
    def prog(self):
        p = self._prog()
        if p is None:
            raise RuntimeError("StepRuntime: its program is gone")
        return p

    def close(self):
        """Release every recorded entry (their pools are destroyed at the next safe point)."""
        for e in self.entries.values():
            e.release()
        self.entries.clear()
        self.cur = None
        drain_pools()

    # the most recent entry's plans (bench.py / tests)
    @property
    def fwd(self):
        return self.cur.fwd if self.cur is not None else None

    @property
    def bwd(self):
        return self.cur.bwd if self.cur is not None else None

    # ------------------------------------------------------------------ signatures
    def _signature(self, x, training):
        p = self.prog
        if self._bufs is None:
            # (module, name) of every buffer, walked once: checking the slots per step costs
            # ~20 us instead of ~0.5 ms for module.buffers() over the STF module tree
            self._bufs = [(mod, n) for mod in p.m.modules() for n in mod._buffers
                          if mod._buffers[n] is not None]
            self._bufd = ([mod._buffers for mod, _ in self._bufs], [n for _, n in self._bufs])
            self._bns = [mod for mod in p.m.modules() if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm)]
        bufs = tuple(map(torch.Tensor.data_ptr, map(dict.__getitem__, *self._bufd)))
        # scalars the recorded launches carry by value: BatchNorm momentum / eps, the STF_*
        # switches the schedule reads per call, the program's own knobs
        bn = tuple((b.momentum, b.eps) for b in self._bns)
        env = _stf_env()
        knobs = p.plan_knobs() if hasattr(p, "plan_knobs") else ()
        return (tuple(x.shape), x.dtype, x.device, training, _lib.storage_dtype(), _lib.stream(),
                p.flat.data.data_ptr(), bufs, bn, env, knobs)

    def _entry(self, sig):
        e = self.entries.get(sig)
        if e is None:
            while len(self.entries) >= self.slots:
                _, old = self.entries.popitem(last=False)
                if old is self.cur:
                    self.cur = None
                old.release()
            e = self.entries[sig] = _Entry()
        else:
            self.entries.move_to_end(sig)
        return e

    # ------------------------------------------------------------------ forward
    def forward(self, x, training, need_bwd, ctx=None):
        """The program's forward(x, training, need_bwd) through the plan cache; only the
        training step (training and need_bwd) is planned, everything else runs eagerly.
        ``ctx``: the autograd ctx that will hold the returned state until its backward."""
        p = self.prog
        drain_pools()                         # a safe point: no recording of ours is open
        if not (enabled() and training and need_bwd and nhwc.TIMER is None):
            return p.forward(x, training, need_bwd)
        e = self._entry(self._signature(x, training))
        if e.busy():
            return p.forward(x, training, need_bwd)
        if e.fwd is None:
            e.seen += 1
            if e.seen <= self.warm:
                return p.forward(x, training, need_bwd)
            self._record_forward(e, x, training)
        else:
            e.x.copy_(x)
            e.fwd.replay()
        if ctx is not None:
            e.owner = weakref.ref(ctx)
        self.cur = e
        return e.logits, e.S

    def own(self, S, ctx):
        """``ctx`` (an autograd ctx) now holds the state ``S`` that forward just returned: when that
        is a plan entry's static state, the entry is busy until ctx's backward (forward's ``ctx``
        argument, given after the launches -- the models enqueue the replay before autograd's
        per-parameter bookkeeping)."""
        e = self.cur
        if e is not None and S is not None and e.S is S:
            e.owner = weakref.ref(ctx)

    def _record_forward(self, e, x, training):
        with _no_gc():
            self._record_forward_pooled(e, x, training)

    def _record_forward_pooled(self, e, x, training):
        e.pool = _new_pool()
        nhwc.KEEP = e.keep
        prog = self.prog

        def run():
            if RECORD_HOOK is not None:
                RECORD_HOOK(self, "forward")
            return prog.forward(e.x, training, True)
        try:
            with _pool_context(e.pool):
                e.x = nhwc.empty(tuple(x.shape), x.dtype, x.device)
                e.x.copy_(x)
                plan = Plan()
                e.logits, e.S = plan.record(run)
        finally:
            nhwc.KEEP = None
        e.fwd = plan

    # ------------------------------------------------------------------ backward
    def backward(self, S, dlogits):
        p = self.prog
        e = next((v for v in self.entries.values() if v.fwd is not None and v.S is S), None)
        if e is None or not enabled() or nhwc.TIMER is not None:
            return p.backward(S, dlogits)
        bsig = (tuple(dlogits.shape), p.flat.grad.data_ptr(), p.grad_ready_hook is not None, _lib.stream())
        if e.bwd is None or bsig != e.bsig:
            return self._record_backward(e, S, dlogits, bsig)
        e.dl.copy_(dlogits)
        pos = 0
        hook = p.grad_ready_hook
        for idx, off, deps in e.marks:
            e.bwd.replay(pos, idx)
            hook(off, deps)
            pos = idx
        e.bwd.replay(pos)

    def _record_backward(self, e, S, dlogits, bsig):
        with _no_gc():
            self._record_backward_pooled(e, S, dlogits, bsig)

    def _record_backward_pooled(self, e, S, dlogits, bsig):
        p = self.prog
        e.bwd = None
        e.bkeep = []
        nhwc.KEEP = e.bkeep
        plan = Plan()
        marks = []
        real_hook = p.grad_ready_hook
        pend = []                       # dependencies of hook calls that launched nothing
        if real_hook is not None:
            # a hook point splits the replay into segments with a Python call between them; keep
            # only the points where the hook acted (it returns False when it launched nothing:
            # its later calls carry those calls' offsets -- the suffix only grows -- and their
            # dependencies are handed on with the next kept point)
            def hook(off, deps=()):
                pend.extend(d for d in deps if all(d is not q for q in pend))
                acted = real_hook(off, deps)
                if acted is None or acted:
                    marks.append((plan.size(), off, tuple(pend)))
                    pend.clear()
            p.grad_ready_hook = hook

        def run():
            if RECORD_HOOK is not None:
                RECORD_HOOK(self, "backward")
            return p.backward(S, e.dl)
        try:
            with _pool_context(e.pool):
                e.dl = nhwc.empty(tuple(dlogits.shape), dlogits.dtype, dlogits.device)
                e.dl.copy_(dlogits)
                plan.record(run)
        finally:
            nhwc.KEEP = None
            p.grad_ready_hook = real_hook
        e.bwd, e.bsig, e.marks = plan, bsig, marks

    def timing(self):
        """Summed (launches, ms, flops) of the TIMED kernel in this runtime's replays."""
        tot = [0, 0.0, 0.0]
        for e in self.entries.values():
            for pl in (e.fwd, e.bwd):
                if pl is not None:
                    n, ms, fl = pl.timing()
                    tot[0] += n
                    tot[1] += ms
                    tot[2] += fl
        return tuple(tot)
