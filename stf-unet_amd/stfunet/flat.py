"""One flat fp32 buffer for all parameters and one for their gradients.

The modules keep ordinary ``nn.Parameter`` objects (so ``state_dict`` keys and
``named_parameters`` match the reference), but their storage is re-pointed into
a single contiguous fp32 buffer.  Backward writes every gradient into the
matching slice of a flat gradient buffer, so AdamW is one kernel over one
buffer and the data-parallel all-reduce moves contiguous buckets.

Slices are 16-byte aligned (offsets rounded up to 4 floats) for float4 access;
the gaps stay zero in both buffers.
"""
import operator

import torch


_REQ = operator.attrgetter("requires_grad")


def _align4(n):
    return (n + 3) & ~3


class FlatParams:
    def __init__(self, module):
        self.module = module
        self.params = [p for p in module.parameters()]
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += _align4(p.numel())
        self.numel = off
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.data = None
        self._ptrs = None
        self.grad = None
        self._views = None

    def _aliased(self):
        """Every parameter still a contiguous view of its slice of ``self.data``.  Runs on every
        forward, at the step boundary where the GPU waits for the host: one list of addresses
        compared at once (an address inside the fp32 device buffer pins device and dtype), then
        contiguity -- a quarter of the per-parameter attribute checks' host time."""
        if self.data is None:
            return False
        if list(map(torch.Tensor.data_ptr, self.params)) != self._ptrs:
            return False
        return all(map(torch.Tensor.is_contiguous, self.params))

    def ensure(self):
        """(Re)build the flat buffers if any parameter was re-allocated (``.to()``,
        ``load_state_dict`` keeps storage, so usually a no-op)."""
        if self._aliased():
            return
        dev = self.params[0].device
        data = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        for p, off in zip(self.params, self.offsets):
            n = p.numel()
            data[off:off + n].copy_(p.detach().reshape(-1).float())
            p.data = data[off:off + n].view(p.shape)
        self.data = data
        self._ptrs = [data.data_ptr() + 4 * off for off in self.offsets]
        self._spare = None
        self._use(torch.zeros(self.numel, dtype=torch.float32, device=dev))

    def _use(self, buf):
        self.grad = buf
        self._views = [buf[off:off + p.numel()].view(p.shape) for p, off in zip(self.params, self.offsets)]

    def _aliases(self, buf):
        lo = buf.data_ptr()
        hi = lo + 4 * self.numel
        return any(p.grad is not None and lo <= p.grad.data_ptr() < hi for p in self.params)

    def fresh_grad(self):
        """Zero the gradient buffer for a new backward.  If a parameter's ``.grad`` still
        aliases it (``zero_grad(set_to_none=False)``, or gradient accumulation: autograd then
        adds the new gradients into ``.grad``), the backward writes the other of TWO buffers
        instead, so that the two tensors autograd adds are distinct and the buffer the recorded
        backward plan writes stays the same from step to step (its address is part of the plan's
        signature: a fresh buffer per step would re-record the backward every step)."""
        if self._aliases(self.grad):
            other = self._spare
            if other is None or self._aliases(other):
                other = torch.empty_like(self.grad)
            self._spare = self.grad
            self._use(other)
        self.grad.zero_()

    def any_requires_grad(self):
        return any(map(_REQ, self.params))

    def grad_view(self, p):
        return self._views[self.index[id(p)]]

    def grad_views(self):
        """Fresh view objects (nothing else references them), so autograd's
        AccumulateGrad can adopt them as ``p.grad`` without a copy."""
        return [self.grad[off:off + p.numel()].view(p.shape) for p, off in zip(self.params, self.offsets)]

    def owns(self, params):
        """True when ``params`` are exactly this buffer's parameters, in order."""
        return len(params) == len(self.params) and all(a is b for a, b in zip(params, self.params))
