"""Data-parallel gradient all-reduce over RCCL (torch ``nccl`` backend), bucketed
and overlapped with backward.

The reference has no data parallelism.  Here one
process per GPU runs the same program on its own batch; BatchNorm statistics
stay per rank (torch DDP's default, no SyncBN in the reference).  Gradients live
in one flat fp32 buffer and backward finishes parameter blocks in reverse flat
order, so the finished gradients always form a suffix of that buffer: as soon as
``bucket_mb`` of new suffix is final, an all-reduce of that contiguous slice is
enqueued while the remaining backward kernels keep the GPU busy.  ``finish()``
reduces the last bucket and makes the compute stream wait.

Gradients written on side streams (the STF program's LSTM backwards and weight-gradient
stream) reach the hook as ``deps``.  A bucket's collective is enqueued ON the joiner stream
(``async_op=False`` under it: with PyTorch >= 2.7 -- 2.10 here -- ProcessGroupNCCL launches a
synchronous collective on the CURRENT stream and the host does not block; an older build that
still launches on the process group's internal stream stays correct, because a synchronous call
makes the current stream (the joiner) wait for that stream, but then the hardware-queue argument
below and its measured 3-5 % no longer hold -- ``rccl_stream_note()`` says which applies),
after the joiner waits for the compute stream and those side streams -- so the compute stream
never waits for a side stream on the hook's account, and no stream of RCCL's own is involved:
on HIP, streams share GPU_MAX_HW_QUEUES hardware queues (4) and two streams on one queue run in
order, so a collective stream that lands on the compute stream's queue turns its event wait into
a join of the side streams (the STF step was 3-5 % slower with the hook that way; the joiner
and the programs' side streams are high-priority streams, a queue pool of their own).

Buckets are large and few on purpose: xGMI is point-to-point (7 links per GPU),
RCCL's ring/tree bandwidth per call grows with message size, and each call costs
tens of microseconds of launch/sync, so ~25-64 MB buckets (2-5 per UNet step)
amortise both.
"""
import torch
import torch.distributed as dist


def rccl_stream_note():
    """Which stream a synchronous RCCL collective runs on under this PyTorch build (the
    assumption the joiner design rests on), for bench output."""
    v = tuple(int(p) for p in torch.__version__.split("+")[0].split(".")[:2])
    return ("current stream (the joiner)" if v >= (2, 7) else
            "process group's internal stream (joined by the current stream)") + f", torch {torch.__version__}"


class GradAllReduce:
    def __init__(self, model, bucket_mb=32, group=None):
        self.prog = model.program
        self.flat = self.prog.flat
        self.group = group
        self.world = dist.get_world_size(group)
        self.bucket = max(1, int(bucket_mb * (1 << 20) // 4))
        # RCCL's AVG is one fused pass (pre-multiplied sum); gloo has no AVG (SUM, then a divide).
        # One rank: SUM in place is no work at all, while RCCL's one-rank AVG still launches a
        # scaling kernel over every bucket (oneRankReduce, ~107 us per 54 MB bucket on MI355X)
        # that contends with the backward for CUs and changes nothing
        self.avg = dist.get_backend(group) == "nccl" and self.world > 1
        self.prog.grad_ready_hook = self._ready
        self.after_launch = None        # bench.py --contend: called on the joiner after each collective
        self._reset()

    def _reset(self):
        self.works = []
        self.launched_from = None       # suffix [launched_from, numel) already enqueued
        self.ready_from = None
        self.deps = []                  # side streams the next bucket must wait for

    def _joiner(self, dev):
        from .nhwc import side_stream
        return side_stream(dev, "ddp_join")

    def _launch(self, lo, hi):
        if hi <= lo:
            return
        t = self.flat.grad[lo:hi]
        op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
        deps, self.deps = self.deps, []
        if t.is_cuda:
            js = self._joiner(t.device)
            js.wait_stream(torch.cuda.current_stream(t.device))
            for s in deps:
                js.wait_stream(s)
            with torch.cuda.stream(js):
                dist.all_reduce(t, op=op, group=self.group, async_op=False)
                if self.after_launch is not None:
                    self.after_launch(t)
            self.works.append((None, t))
        else:
            self.works.append((dist.all_reduce(t, op=op, group=self.group, async_op=True), t))

    def _ready(self, begin, deps=()):
        """Flat-gradient elements [begin, numel) are final once the current stream's work and
        that of the streams in ``deps`` (enqueued so far) have run.  Returns whether a bucket was
        launched (a recording step plan keeps a hook point only where one was)."""
        for s in deps:
            if all(s is not d for d in self.deps):
                self.deps.append(s)
        if self.launched_from is None:
            self.launched_from = self.ready_from = self.flat.numel
        self.ready_from = min(self.ready_from, begin)
        if self.launched_from - self.ready_from >= self.bucket or self.ready_from == 0:
            self._launch(self.ready_from, self.launched_from)
            self.launched_from = self.ready_from
            return True
        return False

    def finish(self):
        """Complete every outstanding bucket (call after loss.backward())."""
        if self.launched_from is not None and self.launched_from > 0:
            self._launch(0, self.launched_from)
        joined = set()
        for w, t in self.works:
            if w is None:
                if t.device not in joined:
                    torch.cuda.current_stream(t.device).wait_stream(self._joiner(t.device))
                    joined.add(t.device)
            else:
                w.wait()
            if not self.avg and self.world > 1:
                t.div_(self.world)
        self._reset()
