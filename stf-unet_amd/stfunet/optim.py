"""AdamW over the flat parameter buffer (one kernel per step).

Drop-in for ``torch.optim.AdamW(params, lr, betas, weight_decay, eps, fused=True)``
as built at ``train.py:230-237``: a ``torch.optim.Optimizer`` subclass, so
``LambdaLR`` (``create_lr_scheduler``, train_and_eval.py:414-438), GradScaler and
``state_dict()`` keep working.  Per-parameter state (``step``, ``exp_avg``,
``exp_avg_sq``) is exposed as views into two flat buffers.

When the parameters are exactly one model's ``FlatParams`` and their ``.grad``
tensors are the flat gradient views written by backward, the update is one
``stf_adamw`` launch over the whole buffer; otherwise gradients are first packed
into a flat scratch (one copy) and the same kernel runs.

Under ``torch.amp.GradScaler`` (the reference's ``--amp`` step, train_and_eval.py:396-404)
the optimizer takes the scaler's device-side scale and inf flag (``stf_adamw_amp``)
instead of letting the scaler unscale the gradients and read ``found_inf`` on the host:
the contract torch's fused AdamW implements, so the gradients stay scaled after
``step()`` exactly as with the reference's ``AdamW(fused=True)``, and the step costs no
host synchronisation.
"""
import os

import torch

from ._lib import call, stream
from .nhwc import _p


def _align4(n):
    return (n + 3) & ~3


class AdamW(torch.optim.Optimizer):
    # torch/amp/grad_scaler.py GradScaler.step: an optimizer advertising this receives
    # ``grad_scale`` / ``found_inf`` (device tensors) as attributes for the step
    # (STF_AMP_DEVICE_STEP=0: the scaler's own unscale_ + host inf check, for A/B)
    _step_supports_amp_scaling = os.environ.get("STF_AMP_DEVICE_STEP", "1") != "0"

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, fused=None,
                 capturable=False, **unused):
        """``capturable=True``: lr and the step count live on the device ({lr, step}
        per group, ``stf_adamw_dev``), so ``step()`` can be captured in a caller's HIP graph
        (torch's ``capturable`` contract); call ``graph_sync()`` after the LR scheduler and
        before each replay to publish the new lr.  Same arithmetic as the host-scalar path."""
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._flat = {}
        self.capturable = capturable
        self._hyper = {}

    def _hyper_of(self, gi, group, fb):
        h = self._hyper.get(gi)
        if h is None:
            h = self._hyper[gi] = torch.zeros(2, dtype=torch.float32, device=fb["m"].device)
            h[1] = float(fb["step"])
        return h

    def graph_sync(self):
        """Publish every group's current lr to the device (outside graph capture)."""
        for gi, group in enumerate(self.param_groups):
            h = self._hyper.get(gi)
            if h is not None:
                h[0:1].fill_(float(group["lr"]))

    def _group_buffers(self, gi, group):
        params = group["params"]
        key = (gi, tuple(id(p) for p in params))
        fb = self._flat.get(gi)
        if fb is not None and fb["key"] == key and fb["pptr"][0] == params[0].data_ptr() and \
                fb["pptr"][-1] == params[-1].data_ptr():
            return fb
        if fb is not None:      # re-laying: the device step count (GradScaler steps) is the truth
            self._sync_host_step(gi, fb)
        offs, off = [], 0
        for p in params:
            offs.append(off)
            off += _align4(p.numel())
        dev = params[0].device
        # contiguous parameter storage? (FlatParams lays params out exactly like this)
        base = params[0].data_ptr()
        contiguous = all(p.dtype == torch.float32 and p.is_contiguous() and p.device == dev and
                         p.data_ptr() == base + 4 * o for p, o in zip(params, offs))
        m = torch.zeros(off, dtype=torch.float32, device=dev)
        v = torch.zeros(off, dtype=torch.float32, device=dev)
        # one step counter shared by the group (every parameter steps together): the
        # per-step bookkeeping is one fill_, not one per parameter (host-bound STF step)
        step = torch.zeros((), dtype=torch.float32)
        for p, o in zip(params, offs):
            st = self.state[p]
            n = p.numel()
            if "exp_avg" in st:                       # resumed / pre-existing state
                m[o:o + n].copy_(st["exp_avg"].reshape(-1))
                v[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
            if "step" in st:
                step.fill_(max(float(step), float(st["step"])))
            st["exp_avg"] = m[o:o + n].view(p.shape)
            st["exp_avg_sq"] = v[o:o + n].view(p.shape)
            st["step"] = step
        pflat = None
        if contiguous:
            pflat = torch.empty(0, dtype=torch.float32, device=dev)
            pflat.set_(params[0].untyped_storage(), params[0].storage_offset(), (off,))
        gptr = None
        fb = dict(key=key, pptr=[p.data_ptr() for p in params], offs=offs, n=off, m=m, v=v, p=pflat,
                  gscratch=None, step=step, gptr=gptr)
        self._flat[gi] = fb
        return fb

    def load_state_dict(self, state_dict):
        """Resume (train.py:249-256): torch rebuilds ``self.state`` with new tensors, so
        the flat buffers are re-laid from them at the next step."""
        super().load_state_dict(state_dict)
        self._flat = {}

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"]]
            if not params or all(p.grad is None for p in params):
                continue
            if not params[0].is_cuda:
                raise RuntimeError("stfunet.optim.AdamW runs on the gfx950 kernel only (no CPU fallback)")
            fb = self._group_buffers(gi, group)
            b1, b2 = group["betas"]
            found_inf = getattr(self, "found_inf", None)
            if found_inf is not None:
                self._amp_step(gi, group, params, fb, getattr(self, "grad_scale", None), found_inf)
                continue
            self._sync_host_step(gi, fb)
            if self.capturable:
                h = self._hyper_of(gi, group, fb)
                if not torch.cuda.is_current_stream_capturing():
                    h[0:1].fill_(float(group["lr"]))
                    fb["step"].fill_(int(fb["step"].item()) + 1)    # host mirror (state_dict)
                h[1:2].add_(1.0)
                g = self._flat_grad(params, fb)
                pf = fb["p"]
                assert pf is not None, "capturable AdamW needs the model's flat parameters"
                call("stf_adamw_dev", _p(pf), _p(g), _p(fb["m"]), _p(fb["v"]), fb["n"], _p(h), float(b1), float(b2),
                     float(group["eps"]), float(group["weight_decay"]), stream())
                continue
            step = int(fb["step"].item()) + 1
            fb["step"].fill_(step)
            bc1 = 1.0 - b1 ** step
            bc2 = 1.0 - b2 ** step
            g = self._flat_grad(params, fb)
            if fb["p"] is not None:
                call("stf_adamw", _p(fb["p"]), _p(g), _p(fb["m"]), _p(fb["v"]), fb["n"], float(group["lr"]),
                     float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]), bc1, bc2, stream())
            else:   # scattered parameters: gather, update, scatter back
                pf = torch.zeros(fb["n"], dtype=torch.float32, device=params[0].device)
                for p, o in zip(params, fb["offs"]):
                    pf[o:o + p.numel()].copy_(p.reshape(-1))
                call("stf_adamw", _p(pf), _p(g), _p(fb["m"]), _p(fb["v"]), fb["n"], float(group["lr"]),
                     float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]), bc1, bc2, stream())
                for p, o in zip(params, fb["offs"]):
                    p.copy_(pf[o:o + p.numel()].view_as(p))
        return loss

    def _amp_step(self, gi, group, params, fb, grad_scale, found_inf):
        """GradScaler step: unscale (x 1/scale) and the inf skip inside the kernel, the step
        count advanced on the device (host mirror refreshed lazily, _sync_host_step)."""
        b1, b2 = group["betas"]
        dev = fb["m"].device
        h = self._hyper_of(gi, group, fb)
        if not fb.get("dev_step"):          # the host mirror was authoritative until now
            h[1:2].fill_(float(fb["step"]))
        h[0:1].fill_(float(group["lr"]))
        fb["dev_step"] = True
        if grad_scale is not None and not torch.is_tensor(grad_scale):
            grad_scale = torch.full((1,), float(grad_scale), dtype=torch.float32, device=dev)
        gsc = grad_scale.to(device=dev, dtype=torch.float32) if grad_scale is not None else None
        fin = found_inf.to(device=dev, dtype=torch.float32)
        g = self._flat_grad(params, fb)
        pf = fb["p"]
        if pf is None:       # scattered parameters: gather, update (or skip), scatter back
            pf = torch.zeros(fb["n"], dtype=torch.float32, device=dev)
            for p, o in zip(params, fb["offs"]):
                pf[o:o + p.numel()].copy_(p.reshape(-1))
        call("stf_adamw_amp", _p(pf), _p(g), _p(fb["m"]), _p(fb["v"]), fb["n"], _p(h), _p(gsc), _p(fin),
             float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]), stream())
        if fb["p"] is None:
            for p, o in zip(params, fb["offs"]):
                p.copy_(pf[o:o + p.numel()].view_as(p))

    def _sync_host_step(self, gi, fb):
        """After GradScaler steps the device count is authoritative (a skipped step does not
        advance it): copy it to the host mirror before a host-scalar step or a state_dict."""
        if fb.get("dev_step"):
            fb["step"].fill_(float(self._hyper[gi][1].item()))
            fb["dev_step"] = False

    def state_dict(self):
        for gi, fb in self._flat.items():
            self._sync_host_step(gi, fb)
        return super().state_dict()

    def _flat_grad(self, params, fb):
        g0 = params[0].grad
        if g0 is not None:
            base = g0.data_ptr()
            ptrs = [p.grad.data_ptr() if p.grad is not None else -1 for p in params]
            if ptrs == fb["gptr"]:                    # the same flat gradient views as last step
                g = torch.empty(0, dtype=torch.float32, device=g0.device)
                g.set_(g0.untyped_storage(), g0.storage_offset(), (fb["n"],))
                return g
            if all(p.grad is not None and p.grad.is_contiguous() and p.grad.data_ptr() == base + 4 * o
                   for p, o in zip(params, fb["offs"])):
                fb["gptr"] = ptrs
                g = torch.empty(0, dtype=torch.float32, device=g0.device)
                g.set_(g0.untyped_storage(), g0.storage_offset(), (fb["n"],))
                return g
        if fb["gscratch"] is None:
            fb["gscratch"] = torch.zeros(fb["n"], dtype=torch.float32, device=params[0].device)
        gs = fb["gscratch"]
        for p, o in zip(params, fb["offs"]):
            n = p.numel()
            if p.grad is None:
                gs[o:o + n].zero_()
            else:
                gs[o:o + n].copy_(p.grad.reshape(-1))
        return gs
