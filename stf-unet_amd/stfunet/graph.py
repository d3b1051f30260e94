"""One training step as a HIP graph.

The STF-LSTM-UNet step issues ~600 kernels from Python, ~180 of them through ctypes,
plus the LSTM time loops on side streams: the host spends ~9 ms per step enqueueing
and leaves the GPU idle in its slower stretches (around the loss and the optimizer,
between LSTM steps; ``tools/trace_gaps.py``).  Captured once, the whole step --
forward, criterion, backward (side streams included: they fork from and join back
into the capture stream), the flat AdamW update -- replays with one launch from the
host.  Everything the step allocates comes from the graph's private pool, so the
replayed kernels see the same buffers every time; the inputs are copied into static
buffers, and the learning rate reaches the captured optimizer through device memory
(``AdamW(capturable=True)``, ``graph_sync``).

Requirements: eager warm-up steps first (they record the weight-pack list, size the
BatchNorm partials and compile the code objects) whose losses / autograd graphs are no
longer referenced at capture (a live graph keeps AccumulateGrad nodes bound to the
eager stream, which breaks the capture), one process per GPU without a data-parallel
hook (RCCL calls are not captured here), and ``AdamW(capturable=True)``.
"""
import torch


class TrainStepGraph:
    def __init__(self, model, optimizer, criterion, x, target):
        if not getattr(optimizer, "capturable", False):
            raise ValueError("TrainStepGraph needs stfunet.optim.AdamW(capturable=True)")
        self.model, self.opt, self.criterion = model, optimizer, criterion
        self.x = x.detach().clone()
        self.target = target.detach().clone()
        self.graph = None
        self.loss = None

    def capture(self):
        """Record one step (after eager warm-up steps)."""
        torch.cuda.synchronize()
        self.opt.graph_sync()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = self.criterion(self.model(self.x), self.target)
            self.opt.zero_grad(set_to_none=True)
            loss.backward()
            self.opt.step()
        self.graph, self.loss = g, loss
        return self

    def step(self, x=None, target=None):
        """One training step on (x, target) (copied into the static inputs); returns the
        device loss tensor of this replay."""
        if x is not None:
            self.x.copy_(x, non_blocking=True)
        if target is not None:
            self.target.copy_(target, non_blocking=True)
        self.opt.graph_sync()
        self.graph.replay()
        return self.loss
